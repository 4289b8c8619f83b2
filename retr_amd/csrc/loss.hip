// CrossEntropyLoss over the vocabulary head (models/caption.py:210 as called at engine.py:71:
// mean over B*T rows, no ignore_index) and the greedy argmax (eval_utils/decode.py:71).
// One 256-thread block per logit row; row statistics by online max/sum + wave shuffles.
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

RETR_DEVICE void online_merge(float& m, float& s, float m2, float s2) {
  float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__global__ void __launch_bounds__(256)
ce_fwd_kernel(const T* x, long ld, int V, const long long* tgt, float* lse, float* loss_rows) {
  __shared__ float sm[4], ss[4];
  const int row = blockIdx.x;
  const T* xr = x + (long)row * ld;
  float m = -INFINITY, s = 0.f;
  for (int j = threadIdx.x; j < V; j += 256) {
    float v = to_f(xr[j]);
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = xor_lane(m, o), s2 = xor_lane(s, o);
    online_merge(m, s, m2, s2);
  }
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sm[w] = m, ss[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) online_merge(M, S, sm[i], ss[i]);
    float l = M + logf(S);
    lse[row] = l;
    loss_rows[row] = l - to_f(xr[tgt[row]]);
  }
}

// deterministic mean of per-row losses (single block)
__global__ void mean_kernel(const float* v, int n, float* out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] / n;
}

template <typename T, typename TD>
__global__ void __launch_bounds__(256)
ce_bwd_kernel(const T* x, long ld, int V, const long long* tgt, const float* lse,
              const float* dloss, float inv_count, TD* dx, long lddx) {
  const int row = blockIdx.x;
  const T* xr = x + (long)row * ld;
  TD* dr = dx + (long)row * lddx;
  const float l = lse[row], g = dloss[0] * inv_count;
  const long long t = tgt[row];
  for (int j = threadIdx.x; j < lddx; j += 256) {
    float d = 0.f;
    if (j < V) d = (__expf(to_f(xr[j]) - l) - (j == t ? 1.f : 0.f)) * g;
    dr[j] = from_f<TD>(d);
  }
}

// One pass over a bf16 logit row for the training step: the row's 16-byte chunks stay in
// registers (NCH per thread), so the logits are read once for lse, the row loss and
// dlogits = (exp(x - lse) - onehot) * g, g = 1 * inv_count -- ce_bwd_kernel's arithmetic for
// dloss = 1.  Columns in [V, lddx) are written as 0.
template <int NCH>
__global__ void __launch_bounds__(256)
ce_fused_kernel(const bf16* x, long ld, int V, const long long* tgt, float* lse,
                float* loss_rows, float inv_count, bf16* dx, long lddx) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16* xr = x + (long)row * ld;
  const int nch = (V + 7) / 8;                  // chunks holding real columns
  bf16x8 c[NCH];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int j = tid + 256 * i;
    if (j < nch) c[i] = *(const bf16x8*)(xr + 8 * j);
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int j = tid + 256 * i;
    if (j < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * j + e < V) m = fmaxf(m, (float)c[i][e]);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, xor_lane(m, o));
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int j = tid + 256 * i;
    if (j < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * j + e < V) s += __expf((float)c[i][e] - m);
  }
  for (int o = 32; o > 0; o >>= 1) s += xor_lane(s, o);
  if (lane == 0) red[w] = s;
  __syncthreads();
  const float l = m + logf(red[0] + red[1] + red[2] + red[3]);
  const long long t = tgt[row];
  if (tid == 0) {
    lse[row] = l;
    loss_rows[row] = l - to_f(xr[t]);
  }
  bf16* dr = dx + (long)row * lddx;
  const int ndch = (int)(lddx / 8);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int j = tid + 256 * i;
    if (j >= ndch) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = 8 * j + e;
      float d = 0.f;
      if (j < nch && col < V) d = (__expf((float)c[i][e] - l) - (col == t ? 1.f : 0.f)) * inv_count;
      o[e] = (bf16)d;
    }
    *(bf16x8*)(dr + 8 * j) = o;
  }
}

// ce_bwd_kernel for a dlogits buffer the fused forward already wrote for dloss = 1: every block
// returns at once when dloss is 1, else recomputes the gradient with the given dloss
template <typename T, typename TD>
__global__ void __launch_bounds__(256)
ce_bwd_rescale_kernel(const T* x, long ld, int V, const long long* tgt, const float* lse,
                      const float* dloss, float inv_count, TD* dx, long lddx) {
  if (dloss[0] == 1.f) return;
  const int row = blockIdx.x;
  const T* xr = x + (long)row * ld;
  TD* dr = dx + (long)row * lddx;
  const float l = lse[row], g = dloss[0] * inv_count;
  const long long t = tgt[row];
  for (int j = threadIdx.x; j < lddx; j += 256) {
    float d = 0.f;
    if (j < V) d = (__expf(to_f(xr[j]) - l) - (j == t ? 1.f : 0.f)) * g;
    dr[j] = from_f<TD>(d);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
argmax_kernel(const T* x, long ld, int V, long long* out) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x;
  const T* xr = x + (long)row * ld;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  // 16-byte vector loads (bf16 x 8 / f32 x 4 x 2); the (value, first index, NaN-wins) order
  // makes the result independent of the visiting order (torch.argmax semantics)
  auto visit = [&](float v, int j) {
    if (v > bv || (v == bv && j < bi) || (v != v && bv == bv)) bv = v, bi = j;
  };
  const int V8 = ((ld % 8) == 0) ? V / 8 : 0;
  for (int c = threadIdx.x; c < V8; c += 256) {
    float v[8];
    if constexpr (sizeof(T) == 2) {
      const bf16x8 x8 = *(const bf16x8*)(xr + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (float)x8[e];
    } else {
      const f32x4 a = *(const f32x4*)(xr + 8 * c), b = *(const f32x4*)(xr + 8 * c + 4);
      v[0] = a[0], v[1] = a[1], v[2] = a[2], v[3] = a[3];
      v[4] = b[0], v[5] = b[1], v[6] = b[2], v[7] = b[3];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) visit(v[e], 8 * c + e);
  }
  for (int j = 8 * V8 + threadIdx.x; j < V; j += 256) visit(to_f(xr[j]), j);
  for (int o = 32; o > 0; o >>= 1) {
    float v2 = xor_lane(bv, o);
    int i2 = xor_lane(bi, o);
    bool nan2 = v2 != v2, nan1 = bv != bv;
    if ((nan2 && !nan1) || (nan2 == nan1 && (v2 > bv || (v2 == bv && i2 < bi)))) bv = v2, bi = i2;
  }
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sv[w] = bv, si[w] = bi;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      bool nan2 = sv[i] != sv[i], nan1 = bv != bv;
      if ((nan2 && !nan1) || (nan2 == nan1 && (sv[i] > bv || (sv[i] == bv && si[i] < bi))))
        bv = sv[i], bi = si[i];
    }
    out[row] = bi;
  }
}

// (value, first index, NaN wins) order of argmax_kernel as a comparison
RETR_DEVICE bool am_better(float v2, int i2, float v1, int i1) {
  const bool nan2 = v2 != v2, nan1 = v1 != v1;
  return (nan2 && !nan1) || (nan2 == nan1 && (v2 > v1 || (v2 == v1 && i2 < i1)));
}

// Split argmax for few long rows (decode: 64 rows x 30522 logits): blockIdx.x = segment of the
// row, blockIdx.y = row; every 16-byte load of a segment is in flight at once.  Partials
// (value, index) go to ws[row][segment]; argmax_final_kernel reduces them per row.
constexpr int kArgSeg = 16;

template <typename T>
__global__ void __launch_bounds__(256)
argmax_part_kernel(const T* x, long ld, int V, float* pv, int* pi) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.y, seg = blockIdx.x;
  const T* xr = x + (long)row * ld;
  const int V8 = V / 8;                               // 8-element chunks (ld % 8 == 0)
  const int per = (V8 + kArgSeg - 1) / kArgSeg;
  const int c0 = seg * per, c1 = min(V8, c0 + per);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = c0 + threadIdx.x; c < c1; c += 256) {
    float x8[8];
    if constexpr (sizeof(T) == 2) {
      const bf16x8 t = *(const bf16x8*)(xr + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) x8[e] = (float)t[e];
    } else {
      const f32x4 a = *(const f32x4*)(xr + 8 * c), b = *(const f32x4*)(xr + 8 * c + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) x8[e] = a[e], x8[e + 4] = b[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (am_better(x8[e], 8 * c + e, bv, bi)) bv = x8[e], bi = 8 * c + e;
  }
  if (seg == kArgSeg - 1)                             // the ragged tail
    for (int j = 8 * V8 + threadIdx.x; j < V; j += 256)
      if (am_better(to_f(xr[j]), j, bv, bi)) bv = to_f(xr[j]), bi = j;
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = xor_lane(bv, o);
    const int i2 = xor_lane(bi, o);
    if (am_better(v2, i2, bv, bi)) bv = v2, bi = i2;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sv[w] = bv, si[w] = bi;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i)
      if (am_better(sv[i], si[i], bv, bi)) bv = sv[i], bi = si[i];
    pv[row * kArgSeg + seg] = bv;
    pi[row * kArgSeg + seg] = bi;
  }
}

__global__ void argmax_final_kernel(const float* pv, const int* pi, int M, long long* out) {
  const int row = blockIdx.x * (blockDim.x / kArgSeg) + threadIdx.x / kArgSeg;
  const int s = threadIdx.x % kArgSeg;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  if (row < M) bv = pv[row * kArgSeg + s], bi = pi[row * kArgSeg + s];
  for (int o = kArgSeg / 2; o > 0; o >>= 1) {
    const float v2 = xor_lane(bv, o);
    const int i2 = xor_lane(bi, o);
    if (am_better(v2, i2, bv, bi)) bv = v2, bi = i2;
  }
  if (row < M && s == 0) out[row] = bi;
}

}  // namespace

extern "C" {

int retr_argmax_rows(int dtype, const void* x, long ld, int M, int V, long long* out,
                     void* stream);
size_t retr_argmax_workspace(int M) { return (size_t)M * kArgSeg * 8; }

int retr_argmax_rows_ws(int dtype, const void* x, long ld, int M, int V, long long* out,
                        void* workspace, void* stream) {
  if (M == 0) return 0;
  if (dtype != RETR_BF16 || ld % 8 != 0 || V < 8 * kArgSeg * 256 / 4 || !workspace)
    return retr_argmax_rows(dtype, x, ld, M, V, out, stream);
  hipStream_t st = (hipStream_t)stream;
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + (size_t)M * kArgSeg);
  hipLaunchKernelGGL(argmax_part_kernel<bf16>, dim3(kArgSeg, M), dim3(256), 0, st, (const bf16*)x,
                     ld, V, pv, pi);
  if (int e = retr_check_launch("argmax_part")) return e;
  hipLaunchKernelGGL(argmax_final_kernel, dim3(cdiv(M, 256 / kArgSeg)), dim3(256), 0, st, pv, pi,
                     M, out);
  return retr_check_launch("argmax_final");
}

int retr_ce_fwd(int dtype, const void* logits, long ld, int M, int V, const long long* targets,
                float* lse, float* loss_rows, float* loss, void* stream) {
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(ce_fwd_kernel<bf16>, dim3(M), dim3(256), 0, st, (const bf16*)logits, ld, V,
                       targets, lse, loss_rows);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(M), dim3(256), 0, st, (const float*)logits, ld,
                       V, targets, lse, loss_rows);
  if (retr_check_launch("ce_fwd")) return 1;
  if (loss) {
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, st, loss_rows, M, loss);
    return retr_check_launch("ce_mean");
  }
  return 0;
}

int retr_ce_bwd(int dtype, const void* logits, long ld, int M, int V, const long long* targets,
                const float* lse, const float* dloss, float inv_count, void* dlogits, long lddl,
                void* stream) {
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL((ce_bwd_kernel<bf16, bf16>), dim3(M), dim3(256), 0, st, (const bf16*)logits,
                       ld, V, targets, lse, dloss, inv_count, (bf16*)dlogits, lddl);
  else
    hipLaunchKernelGGL((ce_bwd_kernel<float, float>), dim3(M), dim3(256), 0, st,
                       (const float*)logits, ld, V, targets, lse, dloss, inv_count,
                       (float*)dlogits, lddl);
  return retr_check_launch("ce_bwd");
}

int retr_ce_fwd_bwd(int dtype, const void* logits, long ld, int M, int V,
                    const long long* targets, float* lse, float* loss_rows, float* loss,
                    float inv_count, void* dlogits, long lddl, void* stream) {
  if (M == 0) return 0;
  RETR_REQUIRE(dtype == RETR_BF16 && ld % 8 == 0 && lddl % 8 == 0 && lddl >= V && ld >= V &&
                   (((uintptr_t)logits | (uintptr_t)dlogits) & 15) == 0,
               "ce_fwd_bwd: bf16, 8-aligned rows");
  constexpr int kNch = 16;                       // 16 x 8 x 256 = 32768 columns per row
  RETR_REQUIRE(lddl <= 8L * 256 * kNch, "ce_fwd_bwd: row of %ld columns too long", lddl);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_fused_kernel<kNch>, dim3(M), dim3(256), 0, st, (const bf16*)logits, ld, V,
                     targets, lse, loss_rows, inv_count, (bf16*)dlogits, lddl);
  if (retr_check_launch("ce_fwd_bwd")) return 1;
  if (loss) {
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, st, loss_rows, M, loss);
    return retr_check_launch("ce_mean");
  }
  return 0;
}

int retr_ce_bwd_rescale(int dtype, const void* logits, long ld, int M, int V,
                        const long long* targets, const float* lse, const float* dloss,
                        float inv_count, void* dlogits, long lddl, void* stream) {
  if (M == 0) return 0;
  RETR_REQUIRE(dtype == RETR_BF16, "ce_bwd_rescale: bf16 only");
  hipLaunchKernelGGL((ce_bwd_rescale_kernel<bf16, bf16>), dim3(M), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)logits, ld, V, targets, lse, dloss,
                     inv_count, (bf16*)dlogits, lddl);
  return retr_check_launch("ce_bwd_rescale");
}

int retr_argmax_rows(int dtype, const void* x, long ld, int M, int V, long long* out,
                     void* stream) {
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(argmax_kernel<bf16>, dim3(M), dim3(256), 0, st, (const bf16*)x, ld, V, out);
  else
    hipLaunchKernelGGL(argmax_kernel<float>, dim3(M), dim3(256), 0, st, (const float*)x, ld, V, out);
  return retr_check_launch("argmax_rows");
}

}  // extern "C"

// Greedy bookkeeping of eval_utils/decode.py:72-79 for step i, on device (no host sync):
//   finished |= pred == eos; if all finished -> done = i (the reference returns here, so column
//   i+1 is never written); else caption[:, i+1] = pred.  tok <- pred feeds step i+1.
//   write_all (a batch decoded in independent row groups, eval_utils/decode.py DEC_SPLIT): every
//   column is written and `done` only records the group's first all-finished step -- the
//   caller ends the batch at the LAST group's and clears the columns after it.
__global__ void greedy_update_kernel(const long long* pred, int B, int T, int i, long long eos,
                                     long long* caption, unsigned char* finished, int* done,
                                     long long* tok, int write_all) {
  __shared__ int all_fin;
  if (threadIdx.x == 0) all_fin = 1;
  __syncthreads();
  const int prev_done = *done;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    unsigned char f = finished[b] | (pred[b] == eos ? 1 : 0);
    finished[b] = f;
    if (!f) atomicAnd(&all_fin, 0);
  }
  __syncthreads();
  const bool stop = !write_all && (prev_done >= 0 || all_fin);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if (!stop) caption[(long)b * T + i + 1] = pred[b];
    tok[b] = pred[b];
  }
  if (threadIdx.x == 0 && prev_done < 0 && all_fin) *done = i;
}

// argmax_final_kernel + greedy_update_kernel in one block: thread t reduces segment t % 16 of
// row (t / 16) (rows in groups of 64), the row winners go to pred and an LDS copy, then the
// bookkeeping above runs on them.  One launch fewer per decode step.
__global__ void __launch_bounds__(1024)
greedy_select_kernel(const float* pv, const int* pi, int B, int T, int i, long long eos,
                     long long* pred, long long* caption, unsigned char* finished, int* done,
                     long long* tok, int write_all) {
  __shared__ int all_fin;
  __shared__ long long sp[1024];
  if (threadIdx.x == 0) all_fin = 1;
  const int s = threadIdx.x % kArgSeg;
  for (int r0 = 0; r0 < B; r0 += 1024 / kArgSeg) {
    const int row = r0 + threadIdx.x / kArgSeg;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    if (row < B) bv = pv[row * kArgSeg + s], bi = pi[row * kArgSeg + s];
    for (int o = kArgSeg / 2; o > 0; o >>= 1) {
      const float v2 = xor_lane(bv, o);
      const int i2 = xor_lane(bi, o);
      if (am_better(v2, i2, bv, bi)) bv = v2, bi = i2;
    }
    if (row < B && s == 0) {
      pred[row] = bi;
      if (row < 1024) sp[row] = bi;
    }
  }
  __syncthreads();
  const int prev_done = *done;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const long long pb = b < 1024 ? sp[b] : pred[b];
    unsigned char f = finished[b] | (pb == eos ? 1 : 0);
    finished[b] = f;
    if (!f) atomicAnd(&all_fin, 0);
  }
  __syncthreads();
  const bool stop = !write_all && (prev_done >= 0 || all_fin);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const long long pb = b < 1024 ? sp[b] : pred[b];
    if (!stop) caption[(long)b * T + i + 1] = pb;
    tok[b] = pb;
  }
  if (threadIdx.x == 0 && prev_done < 0 && all_fin) *done = i;
}

extern "C" int retr_greedy_select(int dtype, const void* logits, long ld, int B, int V,
                                  void* workspace, int T, int i, long long eos, long long* pred,
                                  long long* caption, unsigned char* finished, int* done,
                                  long long* tok, void* stream) {
  return retr_greedy_select2(dtype, logits, ld, B, V, workspace, T, i, eos, pred, caption,
                             finished, done, tok, 0, stream);
}

extern "C" int retr_greedy_select2(int dtype, const void* logits, long ld, int B, int V,
                                   void* workspace, int T, int i, long long eos, long long* pred,
                                   long long* caption, unsigned char* finished, int* done,
                                   long long* tok, int write_all, void* stream) {
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (ld % 8 != 0 || V < 8 * kArgSeg * 256 / 4 || !workspace || B > 1024 ||
      ((uintptr_t)logits & 15) != 0) {
    if (int e = retr_argmax_rows(dtype, logits, ld, B, V, pred, stream)) return e;
    hipLaunchKernelGGL(greedy_update_kernel, dim3(1), dim3(256), 0, st, pred, B, T, i, eos,
                       caption, finished, done, tok, write_all);
    return retr_check_launch("greedy_update");
  }
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + (size_t)B * kArgSeg);
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(argmax_part_kernel<bf16>, dim3(kArgSeg, B), dim3(256), 0, st,
                       (const bf16*)logits, ld, V, pv, pi);
  else
    hipLaunchKernelGGL(argmax_part_kernel<float>, dim3(kArgSeg, B), dim3(256), 0, st,
                       (const float*)logits, ld, V, pv, pi);
  if (int e = retr_check_launch("argmax_part")) return e;
  hipLaunchKernelGGL(greedy_select_kernel, dim3(1), dim3(1024), 0, st, pv, pi, B, T, i, eos, pred,
                     caption, finished, done, tok, write_all);
  return retr_check_launch("greedy_select");
}

extern "C" int retr_greedy_update(const long long* pred, int B, int T, int i, long long eos,
                                  long long* caption, unsigned char* finished, int* done,
                                  long long* tok, void* stream) {
  hipLaunchKernelGGL(greedy_update_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, pred, B, T,
                     i, eos, caption, finished, done, tok, 0);
  return retr_check_launch("greedy_update");
}
