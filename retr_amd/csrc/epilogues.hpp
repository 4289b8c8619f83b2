// GEMM epilogues (per-element functors, fused into the MFMA GEMM store).
#pragma once
#include "common.hpp"

namespace retr {

// out = relu2( [res +] drop( relu1( acc + bias ) ) )     (linear / conv forward)
template <typename TO, typename TR>
struct EpiFwd {
  TO* out;
  long ldo;
  const float* bias;  // [N] or null
  const TR* res;      // residual [M][ldr] or null
  long ldr;
  int relu;           // 0 none, 1 before the residual add (Linear->ReLU), 2 after it (ResNet block)
  DropoutParams dp;   // dropout applied to the branch before the residual add
  long drop_ld;       // logical row length used for the dropout counter
  RETR_DEVICE void apply(int m, int n, float v) const {
    if (bias) v += bias[n];
    if (relu == 1) v = fmaxf(v, 0.f);
    if (dp.thresh) v = retr_keep(dp.seed, (uint64_t)m * drop_ld + n, dp.thresh) ? v * dp.scale : 0.f;
    if (res) v += to_f(res[(long)m * ldr + n]);
    if (relu == 2) v = fmaxf(v, 0.f);
    out[(long)m * ldo + n] = from_f<TO>(v);
  }
  RETR_DEVICE void empty_split(int, int) const {}
};

// out = ( acc [+ addend] ) * (gate > 0 ? 1 : 0)     (data-gradient GEMMs; gate = forward ReLU output)
template <typename TO, typename TA, typename TG>
struct EpiDgrad {
  TO* out;
  long ldo;
  const TA* addend;  // or null
  long lda;
  const TG* gate;    // or null
  long ldg;
  RETR_DEVICE void apply(int m, int n, float v) const {
    if (addend) v += to_f(addend[(long)m * lda + n]);
    if (gate && !(to_f(gate[(long)m * ldg + n]) > 0.f)) v = 0.f;
    out[(long)m * ldo + n] = from_f<TO>(v);
  }
  RETR_DEVICE void empty_split(int, int) const {}
};

// fp32 accumulation target (weight gradients): atomic when the GEMM is split over K.
struct EpiAccF32 {
  float* out;
  long ldo;
  int atomic;
  RETR_DEVICE void apply(int m, int n, float v) const {
    float* p = out + (long)m * ldo + n;
    if (atomic) atomicAdd(p, v);
    else *p += v;
  }
  RETR_DEVICE void empty_split(int, int) const {}
};

}  // namespace retr
