// GEMM epilogues.  The GEMM core hands each thread 8 consecutive output columns of one row
// (apply8, n % 8 == 0, n + 8 <= N) or single elements at a ragged right edge (apply).  All
// vector accesses are 16-byte (bf16 x 8) or 2 x 16-byte (f32 x 8); an epilogue falls back to
// scalar accesses when one of its row strides / base pointers is not 8-element aligned.
#pragma once
#include "../../include/retr_hip.h"
#include "common.hpp"

namespace retr {

template <typename T> RETR_DEVICE void load8(const T* p, float (&v)[8]);
template <> RETR_DEVICE void load8<bf16>(const bf16* p, float (&v)[8]) {
  bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
}
template <> RETR_DEVICE void load8<float>(const float* p, float (&v)[8]) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  v[0] = a[0], v[1] = a[1], v[2] = a[2], v[3] = a[3];
  v[4] = b[0], v[5] = b[1], v[6] = b[2], v[7] = b[3];
}
template <typename T> RETR_DEVICE void store8(T* p, const float (&v)[8]);
template <> RETR_DEVICE void store8<bf16>(bf16* p, const float (&v)[8]) {
  bf16x8 x;
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
  *(bf16x8*)p = x;
}
template <> RETR_DEVICE void store8<float>(float* p, const float (&v)[8]) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
// 8 raw elements as loaded (bf16: one 16-byte register quad), widened at use
template <typename T> struct Raw8;
template <> struct Raw8<bf16> {
  bf16x8 x;
  RETR_DEVICE void load(const bf16* p) { x = *(const bf16x8*)p; }
  RETR_DEVICE float operator[](int e) const { return (float)x[e]; }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  RETR_DEVICE void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
  RETR_DEVICE float operator[](int e) const { return e < 4 ? a[e] : b[e - 4]; }
};

// streaming (non-temporal) variant: outputs read back only by a later kernel
template <typename T> RETR_DEVICE void store8_nt(T* p, const float (&v)[8]);
template <> RETR_DEVICE void store8_nt<bf16>(bf16* p, const float (&v)[8]) {
  bf16x8 x;
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4, x), (u32x4*)p);
}
template <> RETR_DEVICE void store8_nt<float>(float* p, const float (&v)[8]) {
  __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, (f32x4*)p);
  __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, (f32x4*)(p + 4));
}

// host helper: can rows of `ld` elements starting at `p` be accessed 8-wide?
template <typename T>
inline bool vec8_ok(const void* p, long ld) {
  return p == nullptr || (((uintptr_t)p % (8 * sizeof(T) < 16 ? 8 * sizeof(T) : 16)) == 0 &&
                          ld % 8 == 0);
}

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
  int vec;            // 8-wide accesses allowed (set by the host from alignment)
  RETR_DEVICE void apply(int m, int n, float v) const {
    if (bias) v += bias[n];
    if (relu == 1) v = fmaxf(v, 0.f);
    if (dp.thresh)
      v = drop_keep(drop_row_key(dp_seed(dp), (uint32_t)m), (uint32_t)n, drop_th16(dp.thresh))
              ? v * dp.scale : 0.f;
    if (res) v += to_f(res[(long)m * ldr + n]);
    if (relu == 2) v = fmaxf(v, 0.f);
    out[(long)m * ldo + n] = from_f<TO>(v);
  }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const {
    if (!vec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) apply(m, n + e, v[e]);
      return;
    }
    if (bias) {
      float b[8];
      load8<float>(bias + n, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += b[e];
    }
    if (relu == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (dp.thresh) {
      const uint32_t km = drop_keep8(drop_row_key(dp_seed(dp), (uint32_t)m), (uint32_t)n,
                                     drop_th16(dp.thresh));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((km >> e) & 1u) ? v[e] * dp.scale : 0.f;
    }
    if (res) {
      float r[8];
      load8<TR>(res + (long)m * ldr + n, r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    if (relu == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (nt) store8_nt<TO>(out + (long)m * ldo + n, v);
    else store8<TO>(out + (long)m * ldo + n, v);
  }
  // operand prefetch: the GEMM issues every residual load of an epilogue band before it
  // stages the accumulators, so the band's loads are in flight together
  struct Pre {
    Raw8<TR> r;
  };
  RETR_DEVICE void fetch8(int m, int n, Pre& p) const {
    if (vec && res) p.r.load(res + (long)m * ldr + n);
  }
  RETR_DEVICE void apply8p(int m, int n, float (&v)[8], const Pre& p) const {
    if (!vec || !res) return apply8(m, n, v);
    if (bias) {
      float b[8];
      load8<float>(bias + n, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += b[e];
    }
    if (relu == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (dp.thresh) {
      const uint32_t km = drop_keep8(drop_row_key(dp_seed(dp), (uint32_t)m), (uint32_t)n,
                                     drop_th16(dp.thresh));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((km >> e) & 1u) ? v[e] * dp.scale : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += p.r[e];
    if (relu == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (nt) store8_nt<TO>(out + (long)m * ldo + n, v);
    else store8<TO>(out + (long)m * ldo + n, v);
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return false; }
  static constexpr bool kRowSum = false;
  float* rowsum = nullptr;
  int nt = 0;          // non-temporal output stores
  void set_vec() {
    vec = vec8_ok<TO>(out, ldo) && vec8_ok<TR>(res, ldr) && vec8_ok<float>(bias, 8);
    nt = retr_tune_get(RETR_TUNE_NT_STORE) == 1;
  }
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
  int vec;
  RETR_DEVICE void apply(int m, int n, float v) const {
    if (addend) v += to_f(addend[(long)m * lda + n]);
    if (gate && !(to_f(gate[(long)m * ldg + n]) > 0.f)) v = 0.f;
    out[(long)m * ldo + n] = from_f<TO>(v);
  }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const {
    if (!vec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) apply(m, n + e, v[e]);
      return;
    }
    if (addend) {
      float a[8];
      load8<TA>(addend + (long)m * lda + n, a);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += a[e];
    }
    if (gate) {
      float g[8];
      load8<TG>(gate + (long)m * ldg + n, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = g[e] > 0.f ? v[e] : 0.f;
    }
    if (nt) store8_nt<TO>(out + (long)m * ldo + n, v);
    else store8<TO>(out + (long)m * ldo + n, v);
  }
  struct Pre {
    Raw8<TA> a;
    Raw8<TG> g;
  };
  RETR_DEVICE void fetch8(int m, int n, Pre& p) const {
    if (!vec) return;
    if (addend) p.a.load(addend + (long)m * lda + n);
    if (gate) p.g.load(gate + (long)m * ldg + n);
  }
  RETR_DEVICE void apply8p(int m, int n, float (&v)[8], const Pre& p) const {
    if (!vec) return apply8(m, n, v);
    if (addend) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.a[e];
    }
    if (gate) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = p.g[e] > 0.f ? v[e] : 0.f;
    }
    if (nt) store8_nt<TO>(out + (long)m * ldo + n, v);
    else store8<TO>(out + (long)m * ldo + n, v);
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return false; }
  static constexpr bool kRowSum = false;
  float* rowsum = nullptr;
  int nt = 0;          // non-temporal output stores
  void set_vec() {
    vec = vec8_ok<TO>(out, ldo) && vec8_ok<TA>(addend, lda) && vec8_ok<TG>(gate, ldg);
    nt = retr_tune_get(RETR_TUNE_NT_STORE) == 1;
  }
};

// fp32 weight-gradient target: atomic when the GEMM is split over K (target pre-zeroed or
// accumulating), else plain store (overwrite) or read-add-write (accumulate).  ``rowsum``:
// optional fp32 [M] that receives the row sums of the A operand (the bias gradient of a
// linear layer, fused into its weight-gradient GEMM — no separate column-sum pass over dY).
struct EpiAccF32 {
  float* out;
  long ldo;
  int atomic;
  int vec;
  int overwrite;
  float* rowsum;
  long split_stride = 0;   // > 0: split-K slice s writes its own slab out + s * stride
  int split = -1;          // the slice index (grouped launches); -1: blockIdx.y
  static constexpr bool kRowSum = true;
  RETR_DEVICE float* base() const {
    return out + (long)(split >= 0 ? split : (int)blockIdx.y) * split_stride;
  }
  RETR_DEVICE void apply(int m, int n, float v) const {
    float* p = base() + (long)m * ldo + n;
    if (atomic) atomicAdd(p, v);
    else if (overwrite) *p = v;
    else *p += v;
  }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const {
    float* p = base() + (long)m * ldo + n;
    if (atomic || !vec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) apply(m, n + e, v[e]);
      return;
    }
    if (overwrite) {
      store8<float>(p, v);
      return;
    }
    float o[8];
    load8<float>(p, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += v[e];
    store8<float>(p, o);
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return atomic != 0; }
  void set_vec() { vec = vec8_ok<float>(out, ldo); }
};

}  // namespace retr
