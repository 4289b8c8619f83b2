// LayerNorm (+ fused position add) and DecoderEmbeddings (gather + LN + dropout), fwd/bwd.
// One wave64 per row; lanes own C/64 columns; statistics by wave shuffles.
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

template <typename T, int PER>
__global__ void __launch_bounds__(256)
ln_fwd_kernel(const float* x, long ldx, const float* gamma, const float* beta, float eps, int M,
              int C, T* y, long ldy, T* y2, const float* pos, int period, float* mean_out,
              float* rstd_out) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long)row * ldx;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = xr[lane + 64 * i];
    s += v[i];
  }
  float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    float d = v[i] - mean;
    q += d * d;
  }
  float var = wave_sum(q) / C;
  float rstd = 1.0f / sqrtf(var + eps);
  const float* pr = pos ? pos + (long)(row % period) * C : nullptr;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + 64 * i;
    float o = (v[i] - mean) * rstd * gamma[c] + beta[c];
    if (y) y[(long)row * ldy + c] = from_f<T>(o);
    if (y2) y2[(long)row * ldy + c] = from_f<T>(o + pr[c]);
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// ---- C % 256 == 0: lanes own 4 consecutive columns per 256-column chunk (16-byte fp32 /
// 8-byte bf16 accesses, one load instruction per operand and chunk) ---------------------------
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
RETR_DEVICE f32x4 ld4(const float* p) { return *(const f32x4*)p; }
RETR_DEVICE f32x4 ld4(const bf16* p) {
  const bf16x4 v = *(const bf16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
RETR_DEVICE void st4(float* p, f32x4 v) { *(f32x4*)p = v; }
RETR_DEVICE void st4(bf16* p, f32x4 v) {
  *(bf16x4*)p = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

template <typename T, int NCH>
__global__ void __launch_bounds__(256)
ln_fwd4_kernel(const float* x, long ldx, const float* gamma, const float* beta, float eps, int M,
               T* y, long ldy, T* y2, const float* pos, int period, float* mean_out,
               float* rstd_out) {
  constexpr int C = 256 * NCH;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long)row * ldx + 4 * lane;
  // the row, gamma / beta and the position row in one round trip, issued behind one another
  // before the reductions (the compiler had left gamma / beta behind the row's reductions and
  // the position row behind the first stores); without y2 the position loads re-read gamma
  // (no branch around them: a conditional load drains the load counter at the join)
  const float* pr = (y2 && pos) ? pos + (long)(row % period) * C + 4 * lane : gamma + 4 * lane;
  f32x4 v[NCH], g[NCH], b[NCH], pv[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) v[j] = ld4(xr + 256 * j);
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    g[j] = ld4(gamma + 4 * lane + 256 * j);
    b[j] = ld4(beta + 4 * lane + 256 * j);
    pv[j] = ld4(pr + 256 * j);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[j][e] - mean;
      q += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * lane + 256 * j;
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mean) * rstd * g[j][e] + b[j][e];
    if (y) st4(y + (long)row * ldy + c, o);
    if (y2) st4(y2 + (long)row * ldy + c, o + pv[j]);
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// NW waves per block, 2 rows per wave in flight; per-column dgamma / dbeta partials summed over
// the block's waves in wave order (deterministic) -> part[block][2][C].
// SLAB: the incoming gradient is the fp32 split-K slabs ws[splits][M][C] of the producing data
// gradient (the FFN up-projection's), summed in slice order and rounded to bf16 exactly as that
// GEMM's slab epilogue would have stored it -- the epilogue launch and its bf16 round trip are
// gone, the result is bitwise the same.
template <typename T, int NCH, int NW, bool SLAB = false>
__global__ void __launch_bounds__(NW * 64)
ln_bwd4_kernel(const T* dy, const T* dy2, long lddy, const float* x, long ldx, const float* gamma,
               const float* mean, const float* rstd, int M, float* dx, long lddx,
               const float* addend, float* part, int rows_per_block, bf16* dxd, long lddxd,
               DropoutParams dpd, const float* ws = nullptr, int splits = 0) {
  constexpr int C = 256 * NCH;
  __shared__ f32x4 red[2][NW][64 * NCH];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4 pg[NCH], pb[NCH], gm[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    pg[j] = pb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    gm[j] = ld4(gamma + 4 * lane + 256 * j);
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  constexpr int RB = 2;
  for (int rb = r0 + wave; rb < r1; rb += NW * RB) {
    f32x4 d[RB][NCH], xv[RB][NCH], ad[RB][NCH];
    float mu[RB], rs[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = rb + NW * u;
      const bool ok = row < r1;
      mu[u] = ok ? mean[row] : 0.f;
      rs[u] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int c = 4 * lane + 256 * j;
        f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (SLAB) {
          if (ok) {
            const long MC = (long)M * C;
            const float* sp = ws + (long)row * C + c;
            for (int sl = 0; sl < splits; ++sl) t += *(const f32x4*)(sp + sl * MC);
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = (float)(bf16)t[e];
          }
        } else {
          if (ok && dy) t = ld4(dy + (long)row * lddy + c);
          if (ok && dy2) t += ld4(dy2 + (long)row * lddy + c);
        }
        d[u][j] = t;
        xv[u][j] = ok ? ld4(x + (long)row * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        ad[u][j] = (ok && addend) ? ld4(addend + (long)row * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    float s1[RB], s2[RB];
    f32x4 g[RB][NCH], xh[RB][NCH];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = 0.f;
      s2[u] = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        xh[u][j] = (xv[u][j] - mu[u]) * rs[u];
        pg[j] += d[u][j] * xh[u][j];
        pb[j] += d[u][j];
        g[u][j] = d[u][j] * gm[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[u] += g[u][j][e];
          s2[u] += g[u][j][e] * xh[u][j][e];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = wave_sum(s1[u]) / C;
      s2[u] = wave_sum(s2[u]) / C;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = rb + NW * u;
      if (row >= r1) continue;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        f32x4 o = rs[u] * (g[u][j] - s1[u] - xh[u][j] * s2[u]);
        if (addend) o += ad[u][j];
        st4(dx + (long)row * lddx + 4 * lane + 256 * j, o);
        if (dxd) {   // the producing block's residual dropout applied to dx, in bf16
          f32x4 od = o;
          if (dpd.thresh) {
            const uint32_t km = drop_keep4(drop_row_key(dp_seed(dpd), (uint32_t)row),
                                           (uint32_t)(4 * lane + 256 * j), drop_th16(dpd.thresh));
#pragma unroll
            for (int e = 0; e < 4; ++e) od[e] = ((km >> e) & 1u) ? o[e] * dpd.scale : 0.f;
          }
          st4(dxd + (long)row * lddxd + 4 * lane + 256 * j, od);
        }
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    red[0][wave][lane + 64 * j] = pg[j];
    red[1][wave][lane + 64 * j] = pb[j];
  }
  __syncthreads();
  float* pw = part + (long)blockIdx.x * 2 * C;
  for (int q = threadIdx.x; q < 2 * 64 * NCH; q += NW * 64) {
    const int which = q / (64 * NCH), cq = q - which * 64 * NCH;
    f32x4 t = red[which][0][cq];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[which][w][cq];
    // chunk cq = lane + 64 j holds columns 4 lane + 256 j .. + 3
    const int ln = cq % 64, j = cq / 64;
    st4(pw + which * C + 4 * ln + 256 * j, t);
  }
}

// rows_per_block rows handled by 4 waves; per-column dgamma/dbeta partials reduced in LDS.
constexpr int kLnBwdRows = 8;
template <typename T, int PER>
__global__ void __launch_bounds__(256)
ln_bwd_kernel(const T* dy, const T* dy2, long lddy, const float* x, long ldx, const float* gamma,
              const float* mean, const float* rstd, int M, int C, float* dx, long lddx,
              const float* addend, float* part, int rows_per_block) {
  __shared__ float red[2][4][1024];
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float pg[PER], pb[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) pg[i] = pb[i] = 0.f;
  int r0 = blockIdx.x * rows_per_block;
  int r1 = min(M, r0 + rows_per_block);
  // the wave's rows in batches of RB: every load of a batch is issued before the first
  // reduction, and the batch's independent shuffle chains interleave (latency-bound otherwise)
  constexpr int RB = 2;
  for (int rb = r0 + wave; rb < r1; rb += 4 * RB) {
    float d[RB][PER], xv[RB][PER], ad[RB][PER], mu[RB], rs[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = rb + 4 * u;
      const bool ok = row < r1;
      mu[u] = ok ? mean[row] : 0.f;
      rs[u] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        float t = (ok && dy) ? to_f(dy[(long)row * lddy + c]) : 0.f;
        if (ok && dy2) t += to_f(dy2[(long)row * lddy + c]);
        d[u][i] = t;
        xv[u][i] = ok ? x[(long)row * ldx + c] : 0.f;
        ad[u][i] = (ok && addend) ? addend[(long)row * ldx + c] : 0.f;
      }
    }
    float s1[RB], s2[RB], g[RB][PER], xh[RB][PER];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = 0.f;
      s2[u] = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        xh[u][i] = (xv[u][i] - mu[u]) * rs[u];
        pg[i] += d[u][i] * xh[u][i];
        pb[i] += d[u][i];
        g[u][i] = d[u][i] * gamma[c];
        s1[u] += g[u][i];
        s2[u] += g[u][i] * xh[u][i];
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = wave_sum(s1[u]) / C;
      s2[u] = wave_sum(s2[u]) / C;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = rb + 4 * u;
      if (row >= r1) continue;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        float o = rs[u] * (g[u][i] - s1[u] - xh[u][i] * s2[u]);
        if (addend) o += ad[u][i];
        dx[(long)row * lddx + c] = o;
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    red[0][wave][lane + 64 * i] = pg[i];
    red[1][wave][lane + 64 * i] = pb[i];
  }
  __syncthreads();
  // per-block partial sums (fixed order), reduced by ln_param_reduce_kernel: deterministic,
  // and no contention of every block adding into the same 2C words
  float* pw = part + (long)blockIdx.x * 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    pw[c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pw[C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// dgamma[c] += sum_b part[b][0][c];  dbeta[c] += sum_b part[b][1][c].  Fixed-order two-level sum
// (deterministic): one 1024-thread block per 64 of the 2C columns; wave w adds partial rows
// b = w, w + 16, ... (eight loads in flight per lane), then the 16 wave sums are added in wave
// order.  (A single thread per column walking all M/16 partials was latency-bound: ~55 us.)
__global__ void __launch_bounds__(1024)
ln_param_reduce_kernel(const float* part, int nblk, int C, float* dgamma, float* dbeta) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < 2 * C) {
    int b = wave;
    for (; b + 16 * 7 < nblk; b += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + 16 * u) * 2 * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nblk; b += 16) s += part[(long)b * 2 * C + c];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || c >= 2 * C) return;
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += red[w][lane];
  if (c < C) {
    if (dgamma) dgamma[c] += t;
  } else if (dbeta) {
    dbeta[c - C] += t;
  }
}

template <int PER>
__global__ void __launch_bounds__(256)
embed_ln_fwd_kernel(const long long* tok, int M, int T, int C, const float* word,
                    const float* posw, const float* gamma, const float* beta, float eps,
                    DropoutParams dp, float* y, float* mean_out, float* rstd_out) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  long t = tok[row];
  int p = row % T;
  float v[PER], s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + 64 * i;
    v[i] = word[t * C + c] + posw[(long)p * C + c];
    s += v[i];
  }
  float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    float d = v[i] - mean;
    q += d * d;
  }
  float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + 64 * i;
    float o = (v[i] - mean) * rstd * gamma[c] + beta[c];
    if (dp.thresh)
      o = drop_keep(drop_row_key(dp_seed(dp), (uint32_t)row), (uint32_t)c, drop_th16(dp.thresh))
              ? o * dp.scale : 0.f;
    y[(long)row * C + c] = o;
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// DecoderEmbeddings backward, deterministic (no atomics).  Kernel 1: per row the gradient of
// LN(word[t] + pos[p]) w.r.t. its input, o[row] -> workspace `dsum`, and per-block partial sums
// of the LayerNorm parameter gradients -> `part` (reduced in block order by
// ln_param_reduce_kernel).  Kernel 2 scatters o into the word-embedding rows: the block of the
// first occurrence of a token sums every row holding that token in row order (single writer
// per embedding row).  Kernel 3 sums o over the batch per position (learned position table).
template <int PER>
__global__ void __launch_bounds__(256)
embed_ln_bwd_kernel(const long long* tok, int M, int T, int C, const float* word,
                    const float* posw, const float* gamma, const float* mean, const float* rstd,
                    const float* dy, DropoutParams dp, float* dsum, float* part,
                    int rows_per_block) {
  __shared__ float red[2][4][1024];
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float pg[PER], pb[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) pg[i] = pb[i] = 0.f;
  int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int row = r0 + wave; row < r1; row += 4) {
    long t = tok[row];
    int p = row % T;
    float mu = mean[row], rs = rstd[row];
    float g[PER], xh[PER], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + 64 * i;
      float d = dy[(long)row * C + c];
      if (dp.thresh)
        d = drop_keep(drop_row_key(dp_seed(dp), (uint32_t)row), (uint32_t)c, drop_th16(dp.thresh))
                ? d * dp.scale : 0.f;
      xh[i] = (word[t * C + c] + posw[(long)p * C + c] - mu) * rs;
      pg[i] += d * xh[i];
      pb[i] += d;
      g[i] = d * gamma[c];
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + 64 * i;
      dsum[(long)row * C + c] = rs * (g[i] - s1 - xh[i] * s2);
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    red[0][wave][lane + 64 * i] = pg[i];
    red[1][wave][lane + 64 * i] = pb[i];
  }
  __syncthreads();
  float* pw = part + (long)blockIdx.x * 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    pw[c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pw[C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// one block per row i; only the block of the first occurrence of tok[i] writes dword[tok[i]]
__global__ void __launch_bounds__(256)
embed_word_scatter_kernel(const long long* tok, int M, int C, const float* dsum, float* dword,
                          int padding_idx) {
  __shared__ int list[256];
  __shared__ int cnt[4];
  __shared__ int earlier;
  const int i = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long t = tok[i];
  if (t == padding_idx) return;
  if (tid == 0) earlier = 0;
  __syncthreads();
  int e = 0;
  for (int j = tid; j < i; j += 256) e |= (tok[j] == t);
  if (e) earlier = 1;
  __syncthreads();
  if (earlier) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};   // columns tid + 256 q (C <= 1024)
  for (int j0 = i; j0 < M; j0 += 256) {
    const int j = j0 + tid;
    const bool hit = j < M && tok[j] == t;
    const unsigned long long bal = __ballot(hit);
    if (lane == 0) cnt[wave] = __popcll(bal);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += cnt[w];
    const int n = cnt[0] + cnt[1] + cnt[2] + cnt[3];
    if (hit) list[base + __popcll(bal & ((1ull << lane) - 1ull))] = j;
    __syncthreads();
    for (int k = 0; k < n; ++k) {            // matching rows in increasing row order
      const float* src = dsum + (long)list[k] * C;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (tid + 256 * q < C) acc[q] += src[tid + 256 * q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (tid + 256 * q < C) dword[t * C + tid + 256 * q] += acc[q];
}

// dposw[p][c] += sum_b dsum[b*T + p][c]  (batch order)
__global__ void embed_pos_reduce_kernel(const float* dsum, int B, int T, int C, float* dposw) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)T * C) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += dsum[(long)b * T * C + i];
  dposw[i] += s;
}


#define PER_SWITCH(C, MACRO)          \
  switch ((C) / 64) {                 \
    case 1: MACRO(1); break;          \
    case 2: MACRO(2); break;          \
    case 4: MACRO(4); break;          \
    case 8: MACRO(8); break;          \
    case 16: MACRO(16); break;        \
    default: retr_set_error("C=%d unsupported (64,128,256,512,1024)", (int)(C)); return 1; \
  }


// y = cast(x), y2 = cast(x + pos[row % period]): the encoder output when there is no final
// encoder LayerNorm (pre_norm=False, models/ConcatTransformer.py:24,105-106): the decoder then
// reads memory = x and memory + pos directly.  One thread per 4 consecutive columns.
template <typename T>
__global__ void add_pos_kernel(const float* x, long ldx, int M, int C, const float* pos,
                               int period, T* y, T* y2, long ldy) {
  const long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 4;
  if (i >= (long)M * C) return;
  const int row = (int)(i / C), c = (int)(i % C);
  const float4 v = *(const float4*)(x + (long)row * ldx + c);
  const float a[4] = {v.x, v.y, v.z, v.w};
  const float* pr = pos ? pos + (long)(row % period) * C + c : nullptr;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (y) y[(long)row * ldy + c + e] = from_f<T>(a[e]);
    if (y2) y2[(long)row * ldy + c + e] = from_f<T>(a[e] + (pr ? pr[e] : 0.f));
  }
}

// out (fp32) = a + b (either may be null): the gradient of add_pos w.r.t. x
template <typename T>
__global__ void sum2_kernel(const T* a, const T* b, long n, float* out) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (a ? to_f(a[i]) : 0.f) + (b ? to_f(b[i]) : 0.f);
}
}  // namespace

extern "C" {

int retr_layernorm_fwd(int dtype, const float* x, long ldx, const float* gamma,
                       const float* beta, float eps, int M, int C, void* y, long ldy, void* y2,
                       const float* pos, int period, float* mean, float* rstd, void* stream) {
  if (M == 0) return 0;
  RETR_REQUIRE(C % 64 == 0, "layernorm: C=%d must be a multiple of 64", C);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(cdiv(M, 4));
  const bool v4 = C % 256 == 0 && C <= 1024 && ldx % 4 == 0 && ldy % 4 == 0 &&
                  ((uintptr_t)x & 15) == 0 && (!y || ((uintptr_t)y & 7) == 0) &&
                  (!y2 || ((uintptr_t)y2 & 7) == 0) && (!pos || ((uintptr_t)pos & 15) == 0) &&
                  ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0;
  if (v4) {
#define LNF4(NC)                                                                                 \
    if (dtype == RETR_BF16)                                                                       \
      hipLaunchKernelGGL((ln_fwd4_kernel<bf16, NC>), grid, dim3(256), 0, st, x, ldx, gamma, beta, \
                         eps, M, (bf16*)y, ldy, (bf16*)y2, pos, period, mean, rstd);              \
    else                                                                                          \
      hipLaunchKernelGGL((ln_fwd4_kernel<float, NC>), grid, dim3(256), 0, st, x, ldx, gamma, beta,\
                         eps, M, (float*)y, ldy, (float*)y2, pos, period, mean, rstd);
    switch (C / 256) {
      case 1: LNF4(1); break;
      case 2: LNF4(2); break;
      default: LNF4(4); break;
    }
#undef LNF4
    return retr_check_launch("layernorm_fwd4");
  }
#define LNF(P)                                                                                   \
  if (dtype == RETR_BF16)                                                                         \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, P>), grid, dim3(256), 0, st, x, ldx, gamma, beta, eps, \
                       M, C, (bf16*)y, ldy, (bf16*)y2, pos, period, mean, rstd);                   \
  else                                                                                            \
    hipLaunchKernelGGL((ln_fwd_kernel<float, P>), grid, dim3(256), 0, st, x, ldx, gamma, beta, eps,\
                       M, C, (float*)y, ldy, (float*)y2, pos, period, mean, rstd);
  PER_SWITCH(C, LNF)
#undef LNF
  return retr_check_launch("layernorm_fwd");
}

int retr_layernorm_bwd(int dtype, const void* dy, const void* dy2, long lddy, const float* x,
                       long ldx, const float* gamma, const float* mean, const float* rstd, int M,
                       int C, float* dx, long lddx, const float* addend, float* dgamma,
                       float* dbeta, float* workspace, void* stream) {
  return retr_layernorm_bwd2(dtype, dy, dy2, lddy, x, ldx, gamma, mean, rstd, M, C, dx, lddx,
                             addend, dgamma, dbeta, workspace, nullptr, 0, 0.f, 0ull, nullptr,
                             stream);
}

int retr_layernorm_bwd2(int dtype, const void* dy, const void* dy2, long lddy, const float* x,
                        long ldx, const float* gamma, const float* mean, const float* rstd, int M,
                        int C, float* dx, long lddx, const float* addend, float* dgamma,
                        float* dbeta, float* workspace, void* dxd, long lddxd, float drop_p,
                        unsigned long long seed, int* nparts, void* stream) {
  if (nparts) *nparts = 0;
  if (M == 0) return 0;
  RETR_REQUIRE(!nparts || workspace, "layernorm_bwd: deferred parameter sums need a workspace");
  if (nparts) dgamma = dbeta = nullptr;
  RETR_REQUIRE(C % 64 == 0, "layernorm: C=%d must be a multiple of 64", C);
  RETR_REQUIRE(dy || dy2, "layernorm_bwd: no incoming gradient");
  RETR_REQUIRE(mean && rstd && gamma && dx, "layernorm_bwd: missing saved statistics");
  RETR_REQUIRE(!(dgamma || dbeta) || workspace, "layernorm_bwd: dgamma/dbeta need a workspace");
  hipStream_t st = (hipStream_t)stream;
  float* part = (dgamma || dbeta || nparts) ? workspace : nullptr;
  const DropoutParams dpd = make_dp(drop_p, seed);
  const bool v4 = C % 256 == 0 && C <= 512 && lddy % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 &&
                  (((uintptr_t)x | (uintptr_t)dx | (uintptr_t)gamma |
                    (uintptr_t)(addend ? addend : x)) & 15) == 0 &&
                  (((uintptr_t)(dy ? dy : dy2) | (uintptr_t)(dy2 ? dy2 : dy)) &
                   (dtype == RETR_BF16 ? 7 : 15)) == 0;
  if (v4) {
    // >= 4096 rows: 16 waves x 2 rows per block (1/4 the partial rows of 8-row blocks for the
    // parameter reduction); fewer rows: 4 waves x 2 rows (enough blocks to spread over the CUs)
    const bool big = M >= 4096;
    int rpb = big ? 32 : 8;
    int nw = big ? 16 : 4;
    // RETR_TUNE_LN_BWD (sweeps, tools/ln_micro.py): rows per block / waves per block
    switch (retr_tune_get(RETR_TUNE_LN_BWD)) {
      case 1: rpb = 32; nw = 16; break;
      case 2: rpb = 16; nw = 8; break;
      case 3: rpb = 8; nw = 4; break;
      case 4: rpb = 16; nw = 16; break;
      case 5: rpb = 64; nw = 16; break;
      case 6: rpb = 8; nw = 8; break;
      default: break;
    }
    dim3 grid(cdiv(M, rpb));
#define LNB4(NC, NW)                                                                               \
    if (dtype == RETR_BF16)                                                                        \
      hipLaunchKernelGGL((ln_bwd4_kernel<bf16, NC, NW>), grid, dim3(NW * 64), 0, st,               \
                         (const bf16*)dy, (const bf16*)dy2, lddy, x, ldx, gamma, mean, rstd, M,    \
                         dx, lddx, addend, part, rpb, (bf16*)dxd, lddxd, dpd);                     \
    else                                                                                           \
      hipLaunchKernelGGL((ln_bwd4_kernel<float, NC, NW>), grid, dim3(NW * 64), 0, st,              \
                         (const float*)dy, (const float*)dy2, lddy, x, ldx, gamma, mean, rstd, M,  \
                         dx, lddx, addend, part, rpb, (bf16*)dxd, lddxd, dpd);
    if (C == 256) {
      if (nw == 16) { LNB4(1, 16) } else if (nw == 8) { LNB4(1, 8) } else { LNB4(1, 4) }
    } else {
      if (nw == 16) { LNB4(2, 16) } else if (nw == 8) { LNB4(2, 8) } else { LNB4(2, 4) }
    }
#undef LNB4
    if (int e = retr_check_launch("layernorm_bwd4")) return e;
    if (!part) return 0;
    if (nparts) {   // the caller sums the partial rows (e.g. in its weight-gradient slab sum)
      *nparts = (int)grid.x;
      return 0;
    }
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(cdiv(2 * C, 64)), dim3(1024), 0, st, part,
                       (int)grid.x, C, dgamma, dbeta);
    return retr_check_launch("layernorm_param_reduce");
  }
  const int rpb = kLnBwdRows;  // 2 rows per wave: ~12 waves per CU at M = 6400
  dim3 grid(cdiv(M, rpb));
#define LNB(P)                                                                                     \
  if (dtype == RETR_BF16)                                                                          \
    hipLaunchKernelGGL((ln_bwd_kernel<bf16, P>), grid, dim3(256), 0, st, (const bf16*)dy,          \
                       (const bf16*)dy2, lddy, x, ldx, gamma, mean, rstd, M, C, dx, lddx, addend,  \
                       part, rpb);                                                                 \
  else                                                                                             \
    hipLaunchKernelGGL((ln_bwd_kernel<float, P>), grid, dim3(256), 0, st, (const float*)dy,        \
                       (const float*)dy2, lddy, x, ldx, gamma, mean, rstd, M, C, dx, lddx, addend, \
                       part, rpb);
  PER_SWITCH(C, LNB)
#undef LNB
  if (int e = retr_check_launch("layernorm_bwd")) return e;
  if (dxd && retr_dropout_apply(RETR_BF16, dx, lddx, dxd, lddxd, M, C, drop_p, seed, stream))
    return 1;
  if (!part) return 0;
  if (nparts) {
    *nparts = (int)grid.x;
    return 0;
  }
  hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(cdiv(2 * C, 64)), dim3(1024), 0, st, part,
                     (int)grid.x, C, dgamma, dbeta);
  return retr_check_launch("layernorm_param_reduce");
}

// retr_layernorm_bwd2 with the incoming gradient given as the fp32 split-K slabs of the bf16
// data-gradient GEMM that produces it (retr_linear_dgrad_slabs): dy = bf16(sum of ws[0..splits)
// in slice order), then the same backward -- bitwise the slab epilogue + retr_layernorm_bwd2
// path, without the epilogue launch and the dy round trip.  The vectorised layouts only (C 256
// or 512, 16-byte aligned rows, as the bf16 transformer blocks use).
int retr_layernorm_bwd_slabs(const float* ws, int splits, const float* x, long ldx,
                             const float* gamma, const float* mean, const float* rstd, int M,
                             int C, float* dx, long lddx, const float* addend, float* dgamma,
                             float* dbeta, float* workspace, void* dxd, long lddxd, float drop_p,
                             unsigned long long seed, int* nparts, void* stream) {
  if (nparts) *nparts = 0;
  if (M == 0) return 0;
  RETR_REQUIRE(ws && splits >= 1 && ((uintptr_t)ws & 15) == 0,
               "layernorm_bwd_slabs: slabs %p splits %d", (const void*)ws, splits);
  RETR_REQUIRE((C == 256 || C == 512) && ldx % 4 == 0 && lddx % 4 == 0 &&
                   (((uintptr_t)x | (uintptr_t)dx | (uintptr_t)gamma |
                     (uintptr_t)(addend ? addend : x)) & 15) == 0,
               "layernorm_bwd_slabs: C=%d (256 | 512, 16-byte aligned rows)", C);
  RETR_REQUIRE(mean && rstd && gamma && dx, "layernorm_bwd_slabs: missing saved statistics");
  RETR_REQUIRE(!nparts || workspace, "layernorm_bwd_slabs: deferred sums need a workspace");
  if (nparts) dgamma = dbeta = nullptr;
  RETR_REQUIRE(!(dgamma || dbeta) || workspace, "layernorm_bwd_slabs: dgamma/dbeta need a workspace");
  hipStream_t st = (hipStream_t)stream;
  float* part = (dgamma || dbeta || nparts) ? workspace : nullptr;
  const DropoutParams dpd = make_dp(drop_p, seed);
  const bool big = M >= 4096;                      // retr_layernorm_bwd2's choice
  const int rpb = big ? 32 : 8;
  const dim3 grid(cdiv(M, rpb));
#define LNBS(NC, NW)                                                                             \
  hipLaunchKernelGGL((ln_bwd4_kernel<bf16, NC, NW, true>), grid, dim3(NW * 64), 0, st,           \
                     (const bf16*)nullptr, (const bf16*)nullptr, 0L, x, ldx, gamma, mean, rstd, M, \
                     dx, lddx, addend, part, rpb, (bf16*)dxd, lddxd, dpd, ws, splits);
  if (C == 256) {
    if (big) { LNBS(1, 16) } else { LNBS(1, 4) }
  } else {
    if (big) { LNBS(2, 16) } else { LNBS(2, 4) }
  }
#undef LNBS
  if (int e = retr_check_launch("layernorm_bwd_slabs")) return e;
  if (!part) return 0;
  if (nparts) {
    *nparts = (int)grid.x;
    return 0;
  }
  hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(cdiv(2 * C, 64)), dim3(1024), 0, st, part,
                     (int)grid.x, C, dgamma, dbeta);
  return retr_check_launch("layernorm_param_reduce");
}

size_t retr_layernorm_bwd_workspace(int M, int C) {
  return sizeof(float) * 2 * (size_t)C * (size_t)cdiv(M, kLnBwdRows);
}

int retr_embed_ln_fwd(const long long* tokens, int B, int T, int C, const float* word,
                      const float* posw, const float* gamma, const float* beta, float eps,
                      float drop_p, unsigned long long seed, float* y, float* mean, float* rstd,
                      void* stream) {
  int M = B * T;
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  DropoutParams dp = make_dp(drop_p, seed);
  dim3 grid(cdiv(M, 4));
#define EF(P)                                                                                   \
  hipLaunchKernelGGL((embed_ln_fwd_kernel<P>), grid, dim3(256), 0, st, tokens, M, T, C, word, posw, \
                     gamma, beta, eps, dp, y, mean, rstd);
  PER_SWITCH(C, EF)
#undef EF
  return retr_check_launch("embed_ln_fwd");
}

size_t retr_embed_ln_bwd_workspace(int B, int T, int C) {
  const long M = (long)B * T;
  return sizeof(float) * ((size_t)M * C + 2 * (size_t)C * (size_t)cdiv(M, 32));
}

int retr_embed_ln_bwd(const long long* tokens, int B, int T, int C, const float* word,
                      const float* posw, const float* gamma, const float* mean, const float* rstd,
                      const float* dy, float drop_p, unsigned long long seed, float* dword,
                      float* dposw, float* dgamma, float* dbeta, int padding_idx,
                      void* workspace, void* stream) {
  int M = B * T;
  if (M == 0) return 0;
  RETR_REQUIRE(workspace != nullptr, "embed_ln_bwd: workspace required");
  RETR_REQUIRE(C <= 1024, "embed_ln_bwd: C=%d > 1024", C);
  hipStream_t st = (hipStream_t)stream;
  DropoutParams dp = make_dp(drop_p, seed);
  const int rpb = 32;
  const int nblk = cdiv(M, rpb);
  float* dsum = (float*)workspace;
  float* part = dsum + (size_t)M * C;
#define EB(P)                                                                                   \
  hipLaunchKernelGGL((embed_ln_bwd_kernel<P>), dim3(nblk), dim3(256), 0, st, tokens, M, T, C,   \
                     word, posw, gamma, mean, rstd, dy, dp, dsum, part, rpb);
  PER_SWITCH(C, EB)
#undef EB
  if (int e = retr_check_launch("embed_ln_bwd")) return e;
  if (dword) {
    hipLaunchKernelGGL(embed_word_scatter_kernel, dim3(M), dim3(256), 0, st, tokens, M, C, dsum,
                       dword, padding_idx);
    if (int e = retr_check_launch("embed_word_scatter")) return e;
  }
  if (dposw) {
    hipLaunchKernelGGL(embed_pos_reduce_kernel, dim3(cdiv((long)T * C, 256)), dim3(256), 0, st,
                       dsum, B, T, C, dposw);
    if (int e = retr_check_launch("embed_pos_reduce")) return e;
  }
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(cdiv(2 * C, 64)), dim3(1024), 0, st, part,
                       nblk, C, dgamma, dbeta);
    if (int e = retr_check_launch("embed_param_reduce")) return e;
  }
  return 0;
}

}  // extern "C"

extern "C" {

int retr_add_pos_fwd(int dtype, const float* x, long ldx, int M, int C, const float* pos,
                     int period, void* y, void* y2, long ldy, void* stream) {
  if (M == 0) return 0;
  RETR_REQUIRE(C % 4 == 0 && ldx % 4 == 0 && period > 0, "add_pos: C/ld must be %%4");
  const long n4 = (long)M * C / 4;
  dim3 grid(cdiv(n4, 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(add_pos_kernel<bf16>, grid, dim3(256), 0, st, x, ldx, M, C, pos, period,
                       (bf16*)y, (bf16*)y2, ldy);
  else
    hipLaunchKernelGGL(add_pos_kernel<float>, grid, dim3(256), 0, st, x, ldx, M, C, pos, period,
                       (float*)y, (float*)y2, ldy);
  return retr_check_launch("add_pos_fwd");
}

int retr_sum2(int dtype, const void* a, const void* b, long n, float* out, void* stream) {
  if (n == 0) return 0;
  dim3 grid(cdiv(n, 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(sum2_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)a, (const bf16*)b,
                       n, out);
  else
    hipLaunchKernelGGL(sum2_kernel<float>, grid, dim3(256), 0, st, (const float*)a,
                       (const float*)b, n, out);
  return retr_check_launch("sum2");
}

}  // extern "C"
