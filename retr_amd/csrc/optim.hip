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

namespace {

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
  if (g)
    for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kThreads) {
      float4 v = g[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    if (partials) partials[blockIdx.x] = s;
    if (step && blockIdx.x == 0) *step += 1.f;
  }
}

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
  for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kThreads) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
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
    p[i] = pp; m[i] = mm; v[i] = vv;
    if (zero_g) g[i] = float4{0.f, 0.f, 0.f, 0.f};   // consumed: the next step's arena is clean
    else if (scale) g[i] = gg;
    if (p16) {   // bf16 shadow of the parameters: the GEMM weight operands, no cast launches
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      *(bf16x4*)(p16 + 4 * i) = bf16x4{(bf16)pp.x, (bf16)pp.y, (bf16)pp.z, (bf16)pp.w};
    }
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
  hipLaunchKernelGGL(adamw_update_kernel, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream,
                     (float4*)param, (float4*)grad, (float4*)exp_avg, (float4*)exp_avg_sq, n4,
                     hyper, beta1, beta2, eps, step, step_offset, partials, nparts, max_norm,
                     (bf16*)param_bf16, zero_grad);
  return retr_check_launch("adamw_update");
}

}  // extern "C"
