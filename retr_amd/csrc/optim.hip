// Fused gradient clipping + AdamW over flat fp32 parameter / gradient / moment arenas.
//
// Replaces the reference's per-step host sequence (engine.py:80-83, main.py:39-41):
//   torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)
//   optimizer.step()                                  # torch.optim.AdamW
// which PyTorch runs as ~20 multi-tensor / per-tensor elementwise launches reading and writing
// the 65 M-element state several times.  Here the trainable parameters live in one arena
// (retr_amd/optim.py), so the whole update is two streaming kernels:
//   1. adamw_sumsq: per-block partial sums of g^2 (deterministic two-level reduction), and the
//      device-side step counter += 1 (so a captured hipGraph replays correct bias corrections);
//   2. adamw_update: every block folds the partials into the global norm -> clip coefficient,
//      then one fused pass  p *= 1-lr*wd;  g *= coef;  m = lerp(m, g, 1-b1);
//      v = b2 v + (1-b2) g^2;  p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
// HBM traffic per element: read p g m v, write p m v (+ g when clipped) = 28-32 bytes,
// + 2 bytes when the bf16 parameter shadow is written.  retr_adamw_update2(zero_grad = 1)
// writes g = 0 instead (the captured training step consumes its gradients: no separate
// 260 MB zero fill of the arena at the next step).
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) float f32v4;
RETR_DEVICE float4 nt_load(const float4* p) {
  const f32v4 x = __builtin_nontemporal_load((const f32v4*)p);
  return float4{x[0], x[1], x[2], x[3]};
}
RETR_DEVICE void nt_store(const float4& v, float4* p) {
  __builtin_nontemporal_store(f32v4{v.x, v.y, v.z, v.w}, (f32v4*)p);
}

constexpr int kThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < kThreads / 64; ++i) s += red[i];
    red[8] = s;
  }
  __syncthreads();
  s = red[8];
  __syncthreads();
  return s;
}

__global__ void __launch_bounds__(kThreads)
adamw_sumsq_kernel(const float4* g, long n4, float* partials, float* step) {
  __shared__ float red[16];
  float s = 0.f;
  if (g) {
    // eight loads in flight per thread (one at a time left the ~230 MB pass latency-bound at
    // ~3 TB/s); the sum runs over the same elements in the same order
    const long stride = (long)gridDim.x * kThreads;
    long i = (long)blockIdx.x * kThreads + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = g[i + k * stride];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    }
    for (; i < n4; i += stride) {
      float4 v = g[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    if (partials) partials[blockIdx.x] = s;
    if (step && blockIdx.x == 0) *step += 1.f;
  }
}

// NT: non-temporal loads and stores (every byte is touched once per step, and none of the
// outputs is read again before the next step's forward / backward).  U: float4 groups per
// thread and iteration, all loaded before any is updated (U = 2: eight loads in flight); the
// per-element arithmetic is the same either way.
template <bool NT, int U = 1>
__global__ void __launch_bounds__(kThreads)
adamw_update_kernel(float4* p, float4* g, float4* m, float4* v, long n4, const float* hyper,
                    double beta1, double beta2, float eps, const float* step, float step_offset,
                    const float* partials, int nparts, float max_norm, bf16* p16, int zero_g) {
  __shared__ float red[16];
  float coef = 1.f;
  if (max_norm > 0.f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < nparts; i += kThreads) s += partials[i];
    s = block_sum(s, red);
    // clip_grad_norm_: coef = clamp(max_norm / (norm + 1e-6), max=1); a NaN norm stays NaN
    // (torch's clamp propagates it and the gradients are always multiplied)
    coef = (s != s) ? s : fminf(max_norm / (sqrtf(s) + 1e-6f), 1.f);
  }
  const float lr = hyper[0], wd = hyper[1];
  // scalars as torch forms them (python doubles rounded once to fp32)
  const double t = (double)*step + (double)step_offset;   // per-parameter step count
  const double bc1 = 1.0 - pow(beta1, t);
  const float bc2s = (float)sqrt(1.0 - pow(beta2, t));
  const float step_size = (float)((double)lr / bc1), decay = (float)(1.0 - (double)lr * wd);
  const float omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2), b2f = (float)beta2;
  const bool scale = !(coef >= 1.f);   // also for a NaN coefficient
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  auto load = [&](long i, float4& pp, float4& gg, float4& mm, float4& vv) {
    if constexpr (NT) {
      pp = nt_load(p + i);
      gg = nt_load(g + i);
      mm = nt_load(m + i);
      vv = nt_load(v + i);
    } else {
      pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    }
  };
  auto update_store = [&](long i, float4& pp, float4& gg, float4& mm, float4& vv) {
    float* pe = &pp.x; float* ge = &gg.x; float* me = &mm.x; float* ve = &vv.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float gr = scale ? ge[e] * coef : ge[e];
      ge[e] = gr;
      float pr = pe[e] * decay;
      float mr = me[e] + omb1 * (gr - me[e]);
      float vr = ve[e] * b2f + omb2 * (gr * gr);
      float denom = sqrtf(vr) / bc2s + eps;
      pe[e] = pr - step_size * (mr / denom);
      me[e] = mr;
      ve[e] = vr;
    }
    if constexpr (NT) {
      nt_store(pp, p + i);
      nt_store(mm, m + i);
      nt_store(vv, v + i);
      if (zero_g) nt_store(float4{0.f, 0.f, 0.f, 0.f}, g + i);
      else if (scale) nt_store(gg, g + i);
      if (p16) {
        const bf16x4 w = bf16x4{(bf16)pp.x, (bf16)pp.y, (bf16)pp.z, (bf16)pp.w};
        __builtin_nontemporal_store(__builtin_bit_cast(u32x2, w), (u32x2*)(p16 + 4 * i));
      }
    } else {
      p[i] = pp; m[i] = mm; v[i] = vv;
      if (zero_g) g[i] = float4{0.f, 0.f, 0.f, 0.f};   // consumed: the next step's arena is clean
      else if (scale) g[i] = gg;
      if (p16)   // bf16 shadow of the parameters: the GEMM weight operands, no cast launches
        *(bf16x4*)(p16 + 4 * i) = bf16x4{(bf16)pp.x, (bf16)pp.y, (bf16)pp.z, (bf16)pp.w};
    }
  };
  const long stride = (long)gridDim.x * kThreads;
  long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if constexpr (U > 1) {
    for (; i + (U - 1) * stride < n4; i += U * stride) {
      float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) load(i + u * stride, pp[u], gg[u], mm[u], vv[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) update_store(i + u * stride, pp[u], gg[u], mm[u], vv[u]);
    }
  }
  for (; i < n4; i += stride) {
    float4 pp, gg, mm, vv;
    load(i, pp, gg, mm, vv);
    update_store(i, pp, gg, mm, vv);
  }
}

}  // namespace

extern "C" {

int retr_adamw_update2(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n,
                       const float* hyper, double beta1, double beta2, float eps,
                       const float* step, float step_offset, const float* partials, int nparts,
                       float max_norm, void* param_bf16, int zero_grad, void* stream);

int retr_adamw_sumsq(const float* grad, long n, float* partials, int nparts, float* step,
                     void* stream) {
  RETR_REQUIRE(n % 4 == 0 && ((uintptr_t)grad & 15) == 0, "adamw_sumsq: n %%4 / 16B alignment");
  RETR_REQUIRE(nparts > 0 && nparts <= 4096, "adamw_sumsq: nparts %d", nparts);
  hipLaunchKernelGGL(adamw_sumsq_kernel, dim3(nparts), dim3(kThreads), 0, (hipStream_t)stream,
                     (const float4*)grad, n / 4, partials, step);
  return retr_check_launch("adamw_sumsq");
}

int retr_adamw_update(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n,
                      const float* hyper, double beta1, double beta2, float eps,
                      const float* step, float step_offset, const float* partials, int nparts,
                      float max_norm, void* param_bf16, void* stream) {
  return retr_adamw_update2(param, grad, exp_avg, exp_avg_sq, n, hyper, beta1, beta2, eps, step,
                            step_offset, partials, nparts, max_norm, param_bf16, 0, stream);
}

int retr_adamw_update2(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n,
                       const float* hyper, double beta1, double beta2, float eps,
                       const float* step, float step_offset, const float* partials, int nparts,
                       float max_norm, void* param_bf16, int zero_grad, void* stream) {
  RETR_REQUIRE(n % 4 == 0, "adamw_update: n must be a multiple of 4");
  RETR_REQUIRE((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) == 0,
               "adamw_update: 16-byte alignment");
  RETR_REQUIRE(max_norm <= 0.f || (partials && nparts > 0), "adamw_update: clip needs partials");
  if (n == 0) return 0;
  long n4 = n / 4;
  int blocks = (int)std::min<long>(2048, (n4 + kThreads - 1) / kThreads);
  // non-temporal streams by default (same-process A/B, profiles/r3_ab_adamw_nt.txt: graphed
  // step 11.190 -> 11.121 ms); knob 2 = plain loads / stores
  const int mode = retr_tune_get(RETR_TUNE_ADAMW_NT);
  auto kern = mode == 2 ? adamw_update_kernel<false>
              : mode == 3 ? adamw_update_kernel<true, 2>   // two groups in flight (A/B)
                          : adamw_update_kernel<true>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream,
                     (float4*)param, (float4*)grad, (float4*)exp_avg, (float4*)exp_avg_sq, n4,
                     hyper, beta1, beta2, eps, step, step_offset, partials, nparts, max_norm,
                     (bf16*)param_bf16, zero_grad);
  return retr_check_launch("adamw_update");
}

}  // extern "C"
