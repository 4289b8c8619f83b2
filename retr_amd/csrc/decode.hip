// Fused kernels of one incremental decode step (greedy / beam; eval_utils/decode.py:53-81 run as
// the KV-cache form).  A decode step has R = B*K query rows (one per caption /
// beam) of width C; each decoder layer (models/ConcatTransformer.py:187-214,
// models/transformer_modules.py:22-97, pre-norm) runs as five launches instead of thirteen:
//
//   dec_gemm         [q | k | v] = (LN1(x) (+pos)) W_in^T + b_in, k/v appended to the cache
//                    (also the head's first MLP layer)
//   dec_attn_row     per row: self-attention over the cache (beam ancestry), out-proj, residual,
//                    LN2 (+pos), cross-attention query projection
//   dec_attn_row     per row: cross-attention over the image memory, out-proj, residual, LN3
//   dec_ffn          FFN1 + ReLU + FFN2 split over the hidden units: partial slabs
//   dec_rows         x = x + b2 + sum of the slabs (fixed order), then the next LN1 (+pos)
//                    (the final decoder LN before the head)
//
// bf16 operands, fp32 accumulation and residual stream, exactly the roundings of the unfused
// path (bf16 GEMM inputs, bf16 q/k/v/attention output, fp32 residual).  Every kernel is
// latency-bound at R = 64: the point is fewer dependent launches per step.
#include <type_traits>

#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

RETR_DEVICE f4 mfma16(const u32x4& a, const u32x4& b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}

// Sum over aligned groups of G lanes (G = 4 or 8) by DPP: quad xor 1, quad xor 2 and, for 8,
// the half-row mirror (lane i <- 7 - i within 8).  Every lane of a group ends with the sum.
template <int CTRL>
RETR_DEVICE float dpp_mov(float s) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s),
                                                               CTRL, 0xF, 0xF, false));
}
template <int G>
RETR_DEVICE float group_sum(float s) {
  static_assert(G == 4 || G == 8, "group of 4 or 8 lanes");
  s += dpp_mov<0xB1>(s);
  s += dpp_mov<0x4E>(s);
  if constexpr (G == 8) s += dpp_mov<0x141>(s);
  return s;
}

// ---- dec_gemm ---------------------------------------------------------------------------------
// y = A W^T + b (opt. ReLU) over R rows, A bf16 [R][C] in global memory: segment s (output columns
// [s*segw, (s+1)*segw)) reads A = a_pos if seg_pos[s] else a_plain, and writes its rows to
// seg_base[s] + r * seg_rs[s] + (n - s*segw) (bf16).  Every operand fragment is loaded before the
// first MFMA (the kernel is latency-bound at R = 64).
struct Segs {
  bf16* base[3];
  long rs[3];
  int pos[3];
};

template <int PER>
__global__ void __launch_bounds__(256)
dec_gemm_kernel(const bf16* a_plain, const bf16* a_pos, int R, const bf16* w, const float* bias,
                int N, Segs segs, int segw, int relu) {
  constexpr int C = PER * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 32, r0 = blockIdx.y * 64;
  const int seg = n0 / segw;
  const bf16* A = segs.pos[seg] ? a_pos : a_plain;
  u32x4 bw[2][C / 32], af[C / 32];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < C / 32; ++ks)
      bw[j][ks] = n < N ? *(const u32x4*)(w + (long)n * C + 32 * ks + 8 * (lane >> 4))
                        : u32x4{0u, 0u, 0u, 0u};
  }
  const int ar = r0 + 16 * wave + (lane & 15);
#pragma unroll
  for (int ks = 0; ks < C / 32; ++ks)
    af[ks] = ar < R ? *(const u32x4*)(A + (long)ar * C + 32 * ks + 8 * (lane >> 4))
                    : u32x4{0u, 0u, 0u, 0u};
  float bn[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
    bn[j] = (bias && n < N) ? bias[n] : 0.f;
  }
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < C / 32; ++ks) {
    acc[0] = mfma16(af[ks], bw[0][ks], acc[0]);
    acc[1] = mfma16(af[ks], bw[1][ks], acc[1]);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
    if (n >= N) continue;
    const float b = bn[j];
    bf16* dst = segs.base[seg] + (n - seg * segw);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = r0 + 16 * wave + 4 * (lane >> 4) + e;
      if (r >= R) continue;
      float v = acc[j][e] + b;
      if (relu) v = fmaxf(v, 0.f);
      dst[(long)r * segs.rs[seg]] = (bf16)v;
    }
  }
}

// ---- dec_linear_f32: the fp32 parity-mode decode step's linears (M <= 64 rows) ---------------
// y[m][n] = x[m][:] . w[n][:] (+ b[n]) (ReLU) (+ res[m][n]) in exact fp32 (16x16x4 f32 MFMA).
// Block = one 16-column tile x ALL (up to four) 16-row tiles: its four waves split K in quarters
// (wave w: the 16-column blocks of K numbered w mod 4) and each wave runs the four row tiles off
// one weight load, so every weight byte is read once per launch (round 5's one-row-tile blocks
// re-read the 62.5 MB vocabulary projection from HBM once per row tile: 57 us of the 0.45 ms
// fused fp32 step).  Within a 16-column block lane group g feeds columns k0 + 4 g .. + 3 to the
// four MFMA steps (each step covers four distinct k, every k once), from one 16-byte load of x
// and of w per lane.  Each tile's wave partials are added in wave order (the same sums as the
// per-tile blocks).  The generic GEMM ran these as 8-block grids (12.7 us per call, 50 calls
// per step).
struct LinF32Seg {          // one linear of a grouped launch (blockIdx.z)
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  const float* res;
  long ldx, ldw, ldy, ldr;
  int N, relu;
};
struct LinF32Group {
  LinF32Seg s[3];
};

__global__ void __launch_bounds__(256)
dec_linear_f32_kernel(LinF32Group grp, int M, int K) {
  const LinF32Seg& sg = grp.s[blockIdx.z];
  const float* x = sg.x;
  const float* w = sg.w;
  const float* bias = sg.bias;
  float* y = sg.y;
  const float* res = sg.res;
  const long ldx = sg.ldx, ldw = sg.ldw, ldy = sg.ldy, ldr = sg.ldr;
  const int N = sg.N, relu = sg.relu;
  __shared__ f4 red[4][4][64];                    // [wave][row tile][lane]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n0 = 16 * blockIdx.x;
  if (n0 >= N) return;
  const int rr = lane & 15, g = lane >> 4;
  const int n = n0 + rr;
  const int MT = (M + 15) / 16;                   // row tiles (<= 4)
  const float* xr[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int m = 16 * t + rr;
    xr[t] = x + (long)(m < M ? m : M - 1) * ldx + 4 * g;
  }
  const float* wr = w + (long)(n < N ? n : N - 1) * ldw + 4 * g;
  f4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int nb = K / 16;                          // 16-column blocks of K
  constexpr int U = 4;                            // blocks per wave in flight
  for (int b0 = wv; b0 < nb; b0 += 4 * U) {
    f4 wa[U], xa[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + 4 * u;
      wa[u] = b < nb ? *(const f4*)(wr + 16 * b) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t)
        xa[u][t] = b < nb && t < MT ? *(const f4*)(xr[t] + 16 * b) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[u][t][s], wa[u][s], acc[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) red[wv][t][lane] = acc[t];
  __syncthreads();
  // wave t finalises row tile t
  const int t = wv;
  if (t >= MT) return;
  const f4 v4 = ((red[0][t][lane] + red[1][t][lane]) + red[2][t][lane]) + red[3][t][lane];
  const int col = n0 + (lane & 15);
  if (col >= N) return;
  const float bb = bias ? bias[col] : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = 16 * t + 4 * (lane >> 4) + e;
    if (row >= M) continue;
    float v = v4[e] + bb;
    if (relu) v = fmaxf(v, 0.f);
    if (res) v += res[(long)row * ldr + col];
    y[(long)row * ldy + col] = v;
  }
}

// ---- dec_linear_bf16: the greedy step's MLP-head linears (M <= 64 rows), same tiling -------
// y = bf16(relu(x W^T + b)), bf16 operands, one 16 x 16 tile per block, the 32-column blocks of
// K dealt to the four waves (16x16x32 bf16 MFMA), partial tiles added in wave order.
__global__ void __launch_bounds__(256)
dec_linear_bf16_kernel(const bf16* x, long ldx, const bf16* w, long ldw, const float* bias,
                       bf16* y, long ldy, int M, int N, int K, int relu) {
  __shared__ f4 red[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n0 = 16 * blockIdx.x, m0 = 16 * blockIdx.y;
  const int rr = lane & 15, g = lane >> 4;
  const int m = m0 + rr, n = n0 + rr;
  const bf16* xr = x + (long)(m < M ? m : M - 1) * ldx + 8 * g;
  const bf16* wr = w + (long)(n < N ? n : N - 1) * ldw + 8 * g;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  const int nb = K / 32;
  constexpr int U = 4;
  for (int b0 = wv; b0 < nb; b0 += 4 * U) {
    u32x4 xa[U], wa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + 4 * u;
      xa[u] = b < nb ? *(const u32x4*)(xr + 32 * b) : u32x4{0u, 0u, 0u, 0u};
      wa[u] = b < nb ? *(const u32x4*)(wr + 32 * b) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = mfma16(xa[u], wa[u], acc);
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv != 0) return;
  const f4 t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
  const int col = n0 + (lane & 15);
  if (col >= N) return;
  const float bb = bias ? bias[col] : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = m0 + 4 * (lane >> 4) + e;
    if (row >= M) continue;
    float v = t[e] + bb;
    if (relu) v = fmaxf(v, 0.f);
    y[(long)row * ldy + col] = (bf16)v;
  }
}

// ---- dec_rows: residual update + LayerNorm, one block per row ---------------------------------
// x = xin (+ b2 + sum_j slabs[j], slabs in order); xout = x (if given); n = LN(x) (bf16),
// npos = LN(x) + pos (bf16, if given).
// One 256-thread block per row: thread t owns columns t, t + 256 (C / 256 of them) and issues
// all of its slab loads at once (a wave-per-row layout ran only R / 4 blocks and walked the
// slabs in four dependent chunks); slabs are added in slab order per column.  The row's
// LayerNorm statistics come from a wave butterfly plus a 4-wave LDS sum.
template <int CPT>
__global__ void __launch_bounds__(256)
dec_rows_blk_kernel(const float* xin, const float* slabs, int nslab, const float* b2, int R,
                    float* xout, const float* gamma, const float* beta, float eps,
                    const float* pos, bf16* n, bf16* npos) {
  constexpr int C = CPT * 256, MAXS = 64 / CPT;
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blockIdx.x;
  const long RC = (long)R * C;
  float v[CPT], bb[CPT], gm[CPT], bt[CPT], ps[CPT];   // per-column operands, loaded up front
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = tid + 256 * i;
    v[i] = xin[(long)r * C + c];
    bb[i] = slabs ? b2[c] : 0.f;
    gm[i] = gamma[c];
    bt[i] = beta[c];
    ps[i] = npos ? pos[c] : 0.f;
  }
  if (slabs) {
    float s[CPT];
#pragma unroll
    for (int i = 0; i < CPT; ++i) s[i] = 0.f;
    for (int j0 = 0; j0 < nslab; j0 += MAXS) {
      float t[MAXS][CPT];
#pragma unroll
      for (int u = 0; u < MAXS; ++u)
#pragma unroll
        for (int i = 0; i < CPT; ++i)
          t[u][i] = j0 + u < nslab ? slabs[(long)(j0 + u) * RC + (long)r * C + tid + 256 * i] : 0.f;
#pragma unroll
      for (int u = 0; u < MAXS; ++u)
#pragma unroll
        for (int i = 0; i < CPT; ++i)
          if (j0 + u < nslab) s[i] += t[u][i];
    }
#pragma unroll
    for (int i = 0; i < CPT; ++i) v[i] = v[i] + (s[i] + bb[i]);
  }
  if (xout) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) xout[(long)r * C + tid + 256 * i] = v[i];
  }
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) sm += v[i];
  sm = wave_sum(sm);
  if (lane == 0) red[0][wave] = sm;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  q = wave_sum(q);
  if (lane == 0) red[1][wave] = q;
  __syncthreads();
  const float rstd = 1.0f / sqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / C + eps);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = tid + 256 * i;
    const float o = (v[i] - mean) * rstd * gm[i] + bt[i];
    n[(long)r * C + c] = (bf16)o;
    if (npos) npos[(long)r * C + c] = (bf16)(o + ps[i]);
  }
}

// ---- dec_embed_rows: token embedding + its LayerNorm, then the first decoder LN1 -----------
// Wave 0 computes LN_e(word[t] + qpos) with embed_ln_fwd_kernel's lane layout and reductions
// (norm.hip), the block then runs dec_rows_blk_kernel's LN on the result (same rounding as the
// two launches it replaces).
template <int CPT>
__global__ void __launch_bounds__(256)
dec_embed_rows_kernel(const long long* tok, const float* word, const float* qpos, const float* ge,
                      const float* be, float epse, float* xout, const float* g1, const float* b1,
                      float eps1, bf16* n, bf16* npos) {
  constexpr int C = CPT * 256, PER = C / 64;
  __shared__ float xs[C];
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blockIdx.x;
  float gm[CPT], bt[CPT], ps[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = tid + 256 * i;
    gm[i] = g1[c];
    bt[i] = b1[c];
    ps[i] = qpos[c];
  }
  if (wave == 0) {
    const long t = tok[r];
    float v[PER], s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      v[i] = word[t * C + c] + qpos[c];
      s += v[i];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float d = v[i] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + epse);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      const float o = (v[i] - mean) * rstd * ge[c] + be[c];
      xs[c] = o;
      xout[(long)r * C + c] = o;
    }
  }
  __syncthreads();
  float v[CPT];
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    v[i] = xs[tid + 256 * i];
    sm += v[i];
  }
  sm = wave_sum(sm);
  if (lane == 0) red[0][wave] = sm;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  q = wave_sum(q);
  if (lane == 0) red[1][wave] = q;
  __syncthreads();
  const float rstd = 1.0f / sqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / C + eps1);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = tid + 256 * i;
    const float o = (v[i] - mean) * rstd * gm[i] + bt[i];
    n[(long)r * C + c] = (bf16)o;
    npos[(long)r * C + c] = (bf16)(o + ps[i]);
  }
}

// Phase timestamps of block 0 / wave 0 for tools/dec_phase.py (a separate -DRETR_DEC_TIMING
// build of the library; compiled out of the product build).
#ifdef RETR_DEC_TIMING
__device__ long long g_dec_t[16];
#define DEC_T(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_dec_t[i] = wall_clock64();
#else
#define DEC_T(i)
#endif

// ---- dec_attn_row ----------------------------------------------------------------------------
// One block per query row r.  Multi-head attention of q[r] over Lk keys (self: cache rows
// (anc ? anc[r][j] : r) * Lmax + j; cross: rows (r / kv_group) * Lmax + j, masked by kpm),
// then xo = x + o W_o^T + b_o (fp32 row), then LN(xo) (+pos) -> either W_q2 (.) + b_q2 -> q2
// (bf16) or, without W_q2, the LN output itself -> q2 (bf16).
struct AttnRowArgs {
  const bf16* q;            // [R][C]
  const bf16* k;            // cache / memory rows [.][C]
  const bf16* v;
  int Lk, Lmax, kv_group;
  const int* anc;           // [R][Lmax] beam ancestry or null
  const unsigned char* kpm; // [R / kv_group][Lk] or null
  const float* x;           // residual in [R][C]
  const bf16* wo;           // [C][C]
  const float* bo;
  float* xo;                // residual out [R][C]
  const float* gamma;
  const float* beta;
  float eps;
  const float* pos;         // [C] or null
  const bf16* wq;           // [C][C] or null
  const float* bq;
  bf16* q2;                 // [R][C]
};

// out[n] = sum_k W[n][k] a[k] for n in [0, C): each half-wave dots one weight row per step
// (16-byte loads); U rows per half-wave are loaded before any is reduced (latency-bound at R=64)
template <int C, int NT>
RETR_DEVICE void gemv_rows(const bf16* W, const float* a, float* out, int tid) {
  constexpr int HW = NT / 32;                    // half-waves
  constexpr int CH = C / 8 / 32;                 // 16-byte chunks per lane per row
  constexpr int RPH = C / HW;                    // rows per half-wave
  constexpr int U = RPH < 8 ? RPH : 8;
  const int hw = tid >> 5, hl = tid & 31;
#pragma unroll
  for (int r0 = 0; r0 < RPH; r0 += U) {
    bf16x8 wv[U][CH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = hw + HW * (r0 + u);
#pragma unroll
      for (int c = 0; c < CH; ++c) wv[u][c] = *(const bf16x8*)(W + (long)n * C + 8 * (hl + 32 * c));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int k0 = 8 * (hl + 32 * c);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)wv[u][c][e] * a[k0 + e];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += xor_lane(s, o);
      if (hl == 0) out[hw + HW * (r0 + u)] = s;
    }
  }
}

// gemv split in two: load the half-wave's rows (C = 256: all 16 rows of a 512-thread block at
// once), then dot them
template <int C, int NT>
struct GemvFrag {
  static constexpr int HW = NT / 32, CH = C / 8 / 32, RPH = C / HW;
  bf16x8 wv[RPH][CH];
  RETR_DEVICE void load(const bf16* W, int tid) {
    const int hw = tid >> 5, hl = tid & 31;
#pragma unroll
    for (int u = 0; u < RPH; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c)
        wv[u][c] = *(const bf16x8*)(W + (long)(hw + HW * u) * C + 8 * (hl + 32 * c));
  }
  RETR_DEVICE void dot(const float* a, float* out, int tid) const {
    const int hw = tid >> 5, hl = tid & 31;
#pragma unroll
    for (int u = 0; u < RPH; ++u) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int k0 = 8 * (hl + 32 * c);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)wv[u][c][e] * a[k0 + e];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += xor_lane(s, o);
      if (hl == 0) out[hw + HW * u] = s;
    }
  }
};

// The residual + LayerNorm tail of dec_attn_row (the ln_fwd_kernel arithmetic), with every
// operand it reads from global memory (residual row, out-proj bias, LN parameters, position row)
// loaded at kernel start by wave 0: they do not depend on the attention, and loading them after
// it cost a dependent HBM round trip per launch.
template <int PER>
struct RowTail {
  static constexpr int C = PER * 64;
  // LDS-DMA (global_load_lds, 4 bytes per lane) of the tail operands into sm [5][C]: no
  // registers held while the attention loads are in flight; read after a __syncthreads (which
  // waits for vmcnt(0))
  RETR_DEVICE static void load(const AttnRowArgs& a, int r, int lane, float* sm) {
    auto g4 = [](const float* src, float* dst) {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 4, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      g4(a.x + (long)r * C + c, sm + 64 * i);
      g4(a.bo + c, sm + C + 64 * i);
      g4(a.gamma + c, sm + 2 * C + 64 * i);
      g4(a.beta + c, sm + 3 * C + 64 * i);
      if (a.pos) g4(a.pos + c, sm + 4 * C + 64 * i);
    }
  }
  // xo = x + (y + bo); t = bf16(LN(xo) (+pos)) -> ob (when a W_q2 follows) or q2
  RETR_DEVICE static void run(const AttnRowArgs& a, int r, int lane, const float* sm,
                              const float* yb, float* ob) {
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      v[i] = sm[c] + (yb[c] + sm[C + c]);
      a.xo[(long)r * C + c] = v[i];
      s += v[i];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float d = v[i] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + a.eps);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      const float o = (v[i] - mean) * rstd * sm[2 * C + c] + sm[3 * C + c];
      const float t = (float)(bf16)(a.pos ? o + sm[4 * C + c] : o);
      if (a.wq) ob[c] = t;
      else a.q2[(long)r * C + c] = (bf16)t;
    }
  }
};

// 1024-thread GEMV for C = 256, two passes of 128 outputs: thread t owns output
// n = 128 p + t / 8 and the 16-byte chunks sub, sub + 8, sub + 16, sub + 24 of its row
// (sub = t % 8): every load instruction reads 128 contiguous bytes per row; the 8 partial sums
// meet through three DPP adds (quad xor 1, quad xor 2, half-row mirror).  (One output row per
// half-wave needed five dependent cross-lane shuffles per row: 2-3 us per GEMV.)
struct Gemv256 {
  bf16x8 wv[2][4];
  RETR_DEVICE void load(const bf16* W, int tid) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const bf16* src = W + (long)(128 * p + (tid >> 3)) * 256 + 8 * (tid & 7);
#pragma unroll
      for (int c = 0; c < 4; ++c) wv[p][c] = *(const bf16x8*)(src + 64 * c);
    }
  }
  // out[n] = sum_k W[n][k] a[k]
  RETR_DEVICE void dot(const float* a, float* out, int tid) const {
    const float* av = a + 8 * (tid & 7);
    float s[2] = {0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f4 a0 = *(const f4*)(av + 64 * c), a1 = *(const f4*)(av + 64 * c + 4);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int e = 0; e < 4; ++e) s[p] += (float)wv[p][c][e] * a0[e];
#pragma unroll
        for (int e = 0; e < 4; ++e) s[p] += (float)wv[p][c][4 + e] * a1[e];
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float v = group_sum<8>(s[p]);
      if ((tid & 7) == 0) out[128 * p + (tid >> 3)] = v;
    }
  }
};

template <int PER, int HD, int MK>
__global__ void __launch_bounds__(512)
dec_attn_row_kernel(AttnRowArgs a, float scale) {
  constexpr int C = PER * 64, H = C / HD, NT = 512, NW = NT / 64;
  constexpr int HPW = (H + NW - 1) / NW;         // heads per wave
  __shared__ float qs[C];                        // scaled, rounded query
  __shared__ float ob[C];                        // attention output (bf16-rounded) / LN output
  __shared__ float yb[C];                        // GEMV result
  __shared__ float tsm[5 * C];                   // RowTail operands
  __shared__ float pb[NW][64 * MK];              // probabilities of the wave's current head
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blockIdx.x;
  constexpr bool kPre = C == 256;                // out-proj rows prefetched during attention
  GemvFrag<C, NT> wo;
  if constexpr (kPre) wo.load(a.wo, tid);
  if (wave == 0) RowTail<PER>::load(a, r, lane, tsm);
  float bq[(C + NT - 1) / NT];
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    bq[u] = (a.wq && c < C) ? a.bq[c] : 0.f;
  }
  for (int c = tid; c < C; c += NT) qs[c] = (float)(bf16)((float)a.q[(long)r * C + c] * scale);
  const int kvb = r / a.kv_group;
  const int* ar = a.anc ? a.anc + (long)r * a.Lmax : nullptr;
  const unsigned char* km = a.kpm ? a.kpm + (long)kvb * a.Lk : nullptr;
  const int Lk = a.Lk;
  long krow[MK];                                 // cache / memory row of key lane + 64 m
  bool kin[MK], kok[MK];                         // key exists / key exists and is not masked
#pragma unroll
  for (int m = 0; m < MK; ++m) {
    const int j = lane + 64 * m;
    kin[m] = j < Lk;
    kok[m] = kin[m] && !(km && km[j]);
    krow[m] = j < Lk ? (ar ? (long)ar[j] : (long)kvb) * a.Lmax + j : 0;
  }
  __syncthreads();
  float* p = pb[wave];
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    const int h = wave * HPW + hh;
    if (h >= H) break;
    bf16x8 kv[MK][HD / 8];
#pragma unroll
    for (int m = 0; m < MK; ++m)
#pragma unroll
      for (int d0 = 0; d0 < HD / 8; ++d0)
        kv[m][d0] = kin[m] ? *(const bf16x8*)(a.k + krow[m] * C + h * HD + 8 * d0) : bf16x8{};
    // first 8 value rows of this lane's PV share, loaded before the scores are reduced
    constexpr int NG = HD / 8, NPART = 64 / NG;
    const int g = lane % NG, part = lane / NG;
    bf16x8 vpre[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = part + NPART * u;
      const long row = j < Lk ? (ar ? (long)ar[j] : (long)kvb) * a.Lmax + j : 0;
      vpre[u] = j < Lk ? *(const bf16x8*)(a.v + row * C + h * HD + 8 * g) : bf16x8{};
    }
    float sc[MK];
    float mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < MK; ++m) {
      float s = -INFINITY;
      if (kok[m]) {
        s = 0.f;
#pragma unroll
        for (int d0 = 0; d0 < HD / 8; ++d0)
#pragma unroll
          for (int e = 0; e < 8; ++e) s += qs[h * HD + 8 * d0 + e] * (float)kv[m][d0][e];
      }
      sc[m] = s;
      mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int m = 0; m < MK; ++m) {
      const float e = (mx == -INFINITY || sc[m] == -INFINITY) ? 0.f : __expf(sc[m] - mx);
      p[lane + 64 * m] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
    // P V: lane = (dim group g of 8 dims, key part): keys j = part, part + NPART, ...
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j0 = part; j0 < Lk; j0 += NPART * 8) {
      bf16x8 vv[8];
      float pj[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + NPART * u;
        const bool ok = j < Lk;
        if (j0 == part) {
          vv[u] = vpre[u];
        } else {
          const long row = ok ? (ar ? (long)ar[j] : (long)kvb) * a.Lmax + j : 0;
          vv[u] = ok ? *(const bf16x8*)(a.v + row * C + h * HD + 8 * g) : bf16x8{};
        }
        pj[u] = ok ? p[j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += pj[u] * (float)vv[u][e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = NG; o < 64; o <<= 1) acc[e] += xor_lane(acc[e], o);
    if (part == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ob[h * HD + 8 * g + e] = (float)(bf16)(acc[e] * inv);
    }
  }
  __syncthreads();
  if constexpr (kPre) wo.dot(ob, yb, tid);
  else gemv_rows<C, NT>(a.wo, ob, yb, tid);
  GemvFrag<C, NT> wq;
  if (kPre && a.wq) wq.load(a.wq, tid);           // in flight across the residual + LN
  __syncthreads();
  // residual (fp32) and the next LayerNorm, one wave (the ln_fwd_kernel arithmetic)
  if (wave == 0) RowTail<PER>::run(a, r, lane, tsm, yb, ob);
  if (!a.wq) return;
  __syncthreads();
  if constexpr (kPre) wq.dot(ob, yb, tid);
  else gemv_rows<C, NT>(a.wq, ob, yb, tid);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    if (c < C) a.q2[(long)r * C + c] = (bf16)(yb[c] + bq[u]);
  }
}

// Two waves per head (1024 threads, H = 8): each wave scores and accumulates one half of the
// keys against its own running max; the halves merge through LDS (max, sum, 8 partial dims per
// lane group) -- the per-head dependency chain (key loads, scores, softmax, P V) is half as
// long as with one wave per head.  The out-projection / LayerNorm / next-query tail is the
// 512-thread kernel's, on 32 half-waves.
template <int PER, int HD, int MK>
__global__ void __launch_bounds__(1024)
dec_attn_row2_kernel(AttnRowArgs a, float scale) {
  constexpr int C = PER * 64, H = C / HD, NT = 1024;
  constexpr int NG = HD / 8, NPART = 64 / NG;
  constexpr int NU = 64 * MK / NPART;            // value rows per lane over all keys
  constexpr int NUH = NU / 2;                    // ... per half
  static_assert(H * 2 == NT / 64 && MK % 2 == 0, "two waves per head");
  __shared__ __attribute__((aligned(16))) float qs[C];
  __shared__ __attribute__((aligned(16))) float ob[C];
  __shared__ float yb[C];
  __shared__ float tsm[5 * C];                   // RowTail operands
  __shared__ float hmx[H][2], hsum[H][2];
  __shared__ float hacc[H][HD];                  // half 1's unnormalised P V
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = wave >> 1, half = wave & 1;
  const int r = blockIdx.x;
  DEC_T(0)
  constexpr bool kPre = C == 256;
  // C = 256: both GEMV weight slices (out-proj, next query) in flight from the start
  using Frag = std::conditional_t<kPre, Gemv256, GemvFrag<C, NT>>;
  constexpr bool kPreQ = kPre && MK <= 2;         // (MK = 4 would spill; cross has no W_q2)
  Frag wo, wq;
  float bq[(C + NT - 1) / NT];
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    bq[u] = (a.wq && c < C) ? a.bq[c] : 0.f;
  }
  bf16 qv[(C + NT - 1) / NT];
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    qv[u] = c < C ? a.q[(long)r * C + c] : bf16(0.f);
  }
  // (the tail's LDS-DMA is issued here: placed after the key / value loads it trips an
  // "incorrect register class" error in the gfx950 backend)
  if (wave == 0) RowTail<PER>::load(a, r, lane, tsm);
  const int kvb = r / a.kv_group;
  const int* ar = a.anc ? a.anc + (long)r * a.Lmax : nullptr;
  const unsigned char* km = a.kpm ? a.kpm + (long)kvb * a.Lk : nullptr;
  const int Lk = a.Lk;
  // lane = (dim group g of 8 dims, key part): keys j = part + NPART u (+ this half's offset);
  // every load instruction reads NPART rows x HD contiguous bytes pieces (the per-CU load
  // pipeline is the limit at one row per block), and the lane's scores are exactly the
  // probabilities its P V share needs (no LDS round trip for P)
  const int g = lane % NG, part = lane / NG;
  bool kok[NUH];
  bf16x8 kk[NUH], vv[NUH];
#pragma unroll
  for (int u = 0; u < NUH; ++u) {
    const int j = part + NPART * (u + half * NUH);
    const long row = j < Lk ? (ar ? (long)ar[j] : (long)kvb) * a.Lmax + j : 0;
    kk[u] = j < Lk ? *(const bf16x8*)(a.k + row * C + h * HD + 8 * g) : bf16x8{};
    kok[u] = j < Lk && !(km && km[j]);
  }
#pragma unroll
  for (int u = 0; u < NUH; ++u) {
    const int j = part + NPART * (u + half * NUH);
    const long row = j < Lk ? (ar ? (long)ar[j] : (long)kvb) * a.Lmax + j : 0;
    vv[u] = j < Lk ? *(const bf16x8*)(a.v + row * C + h * HD + 8 * g) : bf16x8{};
  }
  // load order = need order (the CU's load bandwidth is the limit at one row per block): query,
  // keys, values, then the GEMV weights, which stream in during the attention
  constexpr bool kEarlyWo = MK <= 2;             // (MK = 4: after the scores, or it spills)
  if constexpr (kPre && kEarlyWo) wo.load(a.wo, tid);
  if constexpr (kPreQ) {
    if (a.wq) wq.load(a.wq, tid);
  }
  // the query goes to LDS only after every key / value load has been issued (the store waits
  // for the query load)
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    if (c < C) qs[c] = (float)(bf16)((float)qv[u] * scale);
  }
  DEC_T(1)
  __syncthreads();
  DEC_T(2)
  float sc[NUH];
  float mx = -INFINITY;
  {
    const f4 q0 = *(const f4*)(qs + h * HD + 8 * g), q1 = *(const f4*)(qs + h * HD + 8 * g + 4);
#pragma unroll
    for (int u = 0; u < NUH; ++u) {
      float sv = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) sv += q0[e] * (float)kk[u][e];
#pragma unroll
      for (int e = 0; e < 4; ++e) sv += q1[e] * (float)kk[u][4 + e];
      sv = group_sum<NG>(sv);
      sc[u] = kok[u] ? sv : -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
  }
  if constexpr (kPre && !kEarlyWo) wo.load(a.wo, tid);
  mx = wave_max(mx);
  float sum = 0.f;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NUH; ++u) {
    const float e = (mx == -INFINITY || sc[u] == -INFINITY) ? 0.f : __expf(sc[u] - mx);
    sum += e;                                    // NG copies of every key: divided out below
#pragma unroll
    for (int d = 0; d < 8; ++d) acc[d] += e * (float)vv[u][d];
  }
  sum = wave_sum(sum) * (1.0f / NG);
  DEC_T(3)
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = NG; o < 64; o <<= 1) acc[e] += xor_lane(acc[e], o);
  if (lane == 0) {
    hmx[h][half] = mx;
    hsum[h][half] = sum;
  }
  if (half == 1 && part == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) hacc[h][8 * g + e] = acc[e];
  }
  DEC_T(4)
  __syncthreads();
  if (half == 0 && part == 0) {
    const float m0 = hmx[h][0], m1 = hmx[h][1];
    const float M = fmaxf(m0, m1);
    const float e0 = (m0 == -INFINITY) ? 0.f : __expf(m0 - M);
    const float e1 = (m1 == -INFINITY) ? 0.f : __expf(m1 - M);
    const float inv = 1.f / (hsum[h][0] * e0 + hsum[h][1] * e1);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      ob[h * HD + 8 * g + e] = (float)(bf16)((acc[e] * e0 + hacc[h][8 * g + e] * e1) * inv);
  }
  __syncthreads();
  DEC_T(5)
  if constexpr (kPre) wo.dot(ob, yb, tid);
  else gemv_rows<C, NT>(a.wo, ob, yb, tid);
  if constexpr (kPre && !kPreQ) {
    if (a.wq) wq.load(a.wq, tid);                // in flight across the residual + LN
  }
  __syncthreads();
  DEC_T(6)
  if (wave == 0) RowTail<PER>::run(a, r, lane, tsm, yb, ob);
  DEC_T(7)
  if (!a.wq) return;
  __syncthreads();
  if constexpr (kPre) wq.dot(ob, yb, tid);
  else gemv_rows<C, NT>(a.wq, ob, yb, tid);
  DEC_T(8)
  __syncthreads();
  DEC_T(9)
#pragma unroll
  for (int u = 0; u < (C + NT - 1) / NT; ++u) {
    const int c = tid + NT * u;
    if (c < C) a.q2[(long)r * C + c] = (bf16)(yb[c] + bq[u]);
  }
  DEC_T(10)
}

// ---- dec_ffn: FFN1 + ReLU + FFN2 over hidden units [32 j, 32 j + 32) -> slab j -----------------
template <int PER>
__global__ void __launch_bounds__(64)
dec_ffn_kernel(const bf16* n3, int R, const bf16* w1, const float* b1, const bf16* w2, int F,
               float* slabs) {
  // one wave = 16 rows per block: every wave loads its own weight fragments anyway, so
  // single-wave blocks cost no extra traffic and put 4x the blocks on the GPU at R = 64
  constexpr int C = PER * 64;
  constexpr int HS = 32 + 8;
  __shared__ __attribute__((aligned(16))) bf16 Hs[16 * HS];     // relu(h) [16 rows][32 units]
  const int tid = threadIdx.x, lane = tid & 63, wave = 0;
  const int j0 = blockIdx.x * 32, r0 = blockIdx.y * 16;
  constexpr int NT = C / 16;                     // output column tiles of FFN2
  // every fragment of both weight slices and of the wave's 16 input rows, before any MFMA
  u32x4 w1f[2][C / 32], af[C / 32], w2f[NT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < C / 32; ++ks)
      w1f[t][ks] = *(const u32x4*)(w1 + (long)(j0 + 16 * t + (lane & 15)) * C + 32 * ks +
                                   8 * (lane >> 4));
#pragma unroll
  for (int t = 0; t < NT; ++t)
    w2f[t] = *(const u32x4*)(w2 + (long)(16 * t + (lane & 15)) * F + j0 + 8 * (lane >> 4));
  const int ar = r0 + 16 * wave + (lane & 15);
#pragma unroll
  for (int ks = 0; ks < C / 32; ++ks)
    af[ks] = ar < R ? *(const u32x4*)(n3 + (long)ar * C + 32 * ks + 8 * (lane >> 4))
                    : u32x4{0u, 0u, 0u, 0u};
  const float b1v[2] = {b1[j0 + (lane & 15)], b1[j0 + 16 + (lane & 15)]};
  f4 h[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < C / 32; ++ks) {
    h[0] = mfma16(af[ks], w1f[0][ks], h[0]);
    h[1] = mfma16(af[ks], w1f[1][ks], h[1]);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int jj = 16 * t + (lane & 15);
    const float b = b1v[t];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      Hs[(16 * wave + 4 * (lane >> 4) + e) * HS + jj] = (bf16)fmaxf(h[t][e] + b, 0.f);
  }
  __syncthreads();
  // partial[r][n] = sum_{jj < 32} H[r][jj] W2[n][j0 + jj]; wave = 16 rows x all C columns
  const u32x4 a0 = *(const u32x4*)(Hs + (16 * wave + (lane & 15)) * HS + 8 * (lane >> 4));
  float* slab = slabs + (long)blockIdx.x * R * C;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = 16 * t + (lane & 15);
    const f4 acc = mfma16(a0, w2f[t], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = r0 + 16 * wave + 4 * (lane >> 4) + e;
      if (r < R) slab[(long)r * C + n] = acc[e];
    }
  }
}

// ---- dec_ffn_ln: dec_ffn with the FFN's input LayerNorm in its prologue -----------------------
// Block = 4 waves over the same 16 rows x 32 hidden units as dec_ffn.  Wave w: rows 4w..4w+3 of
// x = xin + (sum_j hslab[j] + bo) (slabs in order; hidden chunk 0's blocks write x to xout) and
// n3 = bf16(LN3(x)) into LDS; waves 0 / 1 then the FFN1 column tile w (16 hidden units), and every
// wave 4 of the 16 FFN2 column tiles -- instead of a retr_dec_rows launch between the per-head
// cross-attention partials (csrc/decode_heads.hip) and the FFN.
template <int PER, int MAXS, int HB, int NWV = 4>
__global__ void __launch_bounds__(64 * NWV)
dec_ffn_ln_kernel(const float* xin, const float* hslab, int nslab, const float* bo,
                  const float* gamma, const float* beta, float eps, float* xout, int R,
                  const bf16* w1, const float* b1, const bf16* w2, int F, float* slabs) {
  constexpr int C = PER * 64;
  constexpr int HS = HB + 8, AS = C + 8;
  constexpr int CPL = C / 64;                     // consecutive columns per lane
  constexpr int NT = C / 16, NTW = NT / NWV;      // FFN2 column tiles, per wave
  constexpr int RPW = 16 / NWV;                   // LayerNorm rows per wave
  constexpr int T1 = HB / 16;                     // FFN1 column tiles (waves 0 .. T1-1)
  constexpr int K2 = HB / 32;                     // FFN2 K-steps
  typedef __attribute__((ext_vector_type(4))) float f4v;
  __shared__ __attribute__((aligned(16))) bf16 Hs[16 * HS];     // relu(h) [16 rows][HB units]
  __shared__ __attribute__((aligned(16))) bf16 As[16 * AS];     // LN3 rows [16][C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.x * HB, r0 = blockIdx.y * 16;
  // weights first: FFN1 column tile w (waves 0 .. T1-1), FFN2 column tiles 4w .. 4w + 3
  u32x4 w1f[C / 32], w2f[NTW][K2];
  if (w < T1) {
#pragma unroll
    for (int ks = 0; ks < C / 32; ++ks)
      w1f[ks] = *(const u32x4*)(w1 + (long)(j0 + 16 * w + (lane & 15)) * C + 32 * ks +
                                8 * (lane >> 4));
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int k2 = 0; k2 < K2; ++k2)
      w2f[t][k2] = *(const u32x4*)(w2 + (long)(16 * (NTW * w + t) + (lane & 15)) * F + j0 +
                                   32 * k2 + 8 * (lane >> 4));
  const float b1v = w < T1 ? b1[j0 + 16 * w + (lane & 15)] : 0.f;
  const long RC = (long)R * C;
  const int c0 = CPL * lane;
  float bb[CPL], gm[CPL], bt[CPL];
#pragma unroll
  for (int e = 0; e < CPL; e += 4) {
    *(f4v*)(bb + e) = *(const f4v*)(bo + c0 + e);
    *(f4v*)(gm + e) = *(const f4v*)(gamma + c0 + e);
    *(f4v*)(bt + e) = *(const f4v*)(beta + c0 + e);
  }
  // the wave's RPW rows: slab loads in flight SCH slabs at a time (every one of them when the
  // registers allow: 64 floats per lane), summed per column in slab order
  constexpr int SCH0 = 64 / (RPW * CPL) < 1 ? 1 : 64 / (RPW * CPL);
  constexpr int SCH = SCH0 < MAXS ? SCH0 : MAXS;
  float sacc[RPW][CPL], xv[RPW][CPL];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int r = r0 + RPW * w + q;
    const int rr = r < R ? r : R - 1;
#pragma unroll
    for (int e = 0; e < CPL; e += 4) *(f4v*)(&xv[q][e]) = *(const f4v*)(xin + (long)rr * C + c0 + e);
#pragma unroll
    for (int e = 0; e < CPL; ++e) sacc[q][e] = 0.f;
  }
#pragma unroll
  for (int j0 = 0; j0 < MAXS; j0 += SCH) {
    float t[RPW][SCH][CPL];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int r = r0 + RPW * w + q;
      const int rr = r < R ? r : R - 1;
#pragma unroll
      for (int j = 0; j < SCH; ++j)
#pragma unroll
        for (int e = 0; e < CPL; e += 4)
          *(f4v*)(&t[q][j][e]) = j0 + j < nslab
                                     ? *(const f4v*)(hslab + (j0 + j) * RC + (long)rr * C + c0 + e)
                                     : f4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q)
#pragma unroll
      for (int e = 0; e < CPL; ++e)
#pragma unroll
        for (int j = 0; j < SCH; ++j)
          if (j0 + j < nslab) sacc[q][e] += t[q][j][e];
  }
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int r = r0 + RPW * w + q;
    float v[CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) v[e] = xv[q][e] + (sacc[q][e] + bb[e]);
    float sm = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) sm += v[e];
    const float mean = wave_sum(sm) / C;
    float qq = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const float d = v[e] - mean;
      qq += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(qq) / C + eps);
#pragma unroll
    for (int e = 0; e < CPL; ++e)
      As[(RPW * w + q) * AS + c0 + e] = (bf16)((v[e] - mean) * rstd * gm[e] + bt[e]);
    if (blockIdx.x == 0 && r < R) {
#pragma unroll
      for (int e = 0; e < CPL; e += 4) *(f4v*)(xout + (long)r * C + c0 + e) = *(f4v*)(v + e);
    }
  }
  __syncthreads();
  if (w < T1) {
    f4 h = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C / 32; ++ks) {
      const u32x4 af = *(const u32x4*)(As + (lane & 15) * AS + 32 * ks + 8 * (lane >> 4));
      h = mfma16(af, w1f[ks], h);
    }
    const int jj = 16 * w + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      Hs[(4 * (lane >> 4) + e) * HS + jj] = (bf16)fmaxf(h[e] + b1v, 0.f);
  }
  __syncthreads();
  u32x4 a0[K2];
#pragma unroll
  for (int k2 = 0; k2 < K2; ++k2)
    a0[k2] = *(const u32x4*)(Hs + (lane & 15) * HS + 32 * k2 + 8 * (lane >> 4));
  float* slab = slabs + (long)blockIdx.x * R * C;
#pragma unroll
  for (int t2 = 0; t2 < NTW; ++t2) {
    const int n = 16 * (NTW * w + t2) + (lane & 15);
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k2 = 0; k2 < K2; ++k2) acc = mfma16(a0[k2], w2f[t2][k2], acc);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = r0 + 4 * (lane >> 4) + e;
      if (r < R) slab[(long)r * C + n] = acc[e];
    }
  }
}

template <typename K>
void set_lds(K kern, size_t bytes) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    done = true;
  }
}

// eight heads: two waves per head (1024 threads); otherwise one wave per head
template <int P, int HDV, int MKV>
void launch_attn_row(const AttnRowArgs& a, float scale, int R, hipStream_t st) {
  if constexpr (P * 64 / HDV == 8)
    hipLaunchKernelGGL((dec_attn_row2_kernel<P, HDV, MKV>), dim3(R), dim3(1024), 0, st, a, scale);
  else
    hipLaunchKernelGGL((dec_attn_row_kernel<P, HDV, MKV>), dim3(R), dim3(512), 0, st, a, scale);
}

}  // namespace

extern "C" {

int retr_dec_gemm(const void* a_plain, const void* a_pos, int R, int C, const void* w,
                  const float* bias, int N, void* d0, long rs0, int pos0, void* d1, long rs1,
                  int pos1, void* d2, long rs2, int pos2, int segw, int relu, void* stream) {
  RETR_REQUIRE(C == 256 || C == 512, "dec_gemm: C=%d (256 | 512)", C);
  RETR_REQUIRE(segw % 32 == 0 && N <= 3 * segw && N % 32 == 0, "dec_gemm: N=%d segw=%d", N,
               segw);
  if (R == 0) return 0;
  Segs s{{(bf16*)d0, (bf16*)d1, (bf16*)d2}, {rs0, rs1, rs2}, {pos0, pos1, pos2}};
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(N / 32, cdiv(R, 64));
  if (C == 256)
    hipLaunchKernelGGL(dec_gemm_kernel<4>, grid, dim3(256), 0, st, (const bf16*)a_plain,
                       (const bf16*)a_pos, R, (const bf16*)w, bias, N, s, segw, relu);
  else
    hipLaunchKernelGGL(dec_gemm_kernel<8>, grid, dim3(256), 0, st, (const bf16*)a_plain,
                       (const bf16*)a_pos, R, (const bf16*)w, bias, N, s, segw, relu);
  return retr_check_launch("dec_gemm");
}

int retr_dec_rows(const float* xin, const float* slabs, int nslab, const float* b2, int R, int C,
                  float* xout, const float* gamma, const float* beta, float eps, const float* pos,
                  void* n, void* npos, void* stream) {
  RETR_REQUIRE(C == 256 || C == 512, "dec_rows: C=%d (256 | 512)", C);
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (C == 256)
    hipLaunchKernelGGL(dec_rows_blk_kernel<1>, dim3(R), dim3(256), 0, st, xin, slabs, nslab, b2,
                       R, xout, gamma, beta, eps, pos, (bf16*)n, (bf16*)npos);
  else
    hipLaunchKernelGGL(dec_rows_blk_kernel<2>, dim3(R), dim3(256), 0, st, xin, slabs, nslab, b2,
                       R, xout, gamma, beta, eps, pos, (bf16*)n, (bf16*)npos);
  return retr_check_launch("dec_rows");
}

int retr_dec_embed_rows(const long long* tok, int R, int C, const float* word, const float* qpos,
                        const float* ge, const float* be, float epse, float* x, const float* g1,
                        const float* b1, float eps1, void* n, void* npos, void* stream) {
  RETR_REQUIRE(C == 256 || C == 512, "dec_embed_rows: C=%d (256 | 512)", C);
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (C == 256)
    hipLaunchKernelGGL(dec_embed_rows_kernel<1>, dim3(R), dim3(256), 0, st, tok, word, qpos, ge,
                       be, epse, x, g1, b1, eps1, (bf16*)n, (bf16*)npos);
  else
    hipLaunchKernelGGL(dec_embed_rows_kernel<2>, dim3(R), dim3(256), 0, st, tok, word, qpos, ge,
                       be, epse, x, g1, b1, eps1, (bf16*)n, (bf16*)npos);
  return retr_check_launch("dec_embed_rows");
}

int retr_dec_attn_row(const void* q, const void* k, const void* v, int R, int C, int H, int Lk,
                      int Lmax, int kv_group, const int* anc, const unsigned char* kpm,
                      const float* x, const void* wo, const float* bo, float* xo,
                      const float* gamma, const float* beta, float eps, const float* pos,
                      const void* wq, const float* bq, void* q2, void* stream) {
  const int hd = C / H;
  RETR_REQUIRE((C == 256 || C == 512) && (hd == 32 || hd == 64) && H % 4 == 0,
               "dec_attn_row: C=%d H=%d unsupported", C, H);
  RETR_REQUIRE(Lk > 0 && Lk <= 512, "dec_attn_row: Lk=%d (1..512)", Lk);
  if (R == 0) return 0;
  AttnRowArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, Lk, Lmax, kv_group, anc, kpm, x,
                (const bf16*)wo, bo, xo, gamma, beta, eps, pos, (const bf16*)wq, bq, (bf16*)q2};
  const float scale = 1.0f / sqrtf((float)hd);
  hipStream_t st = (hipStream_t)stream;
#define ATT(P, HDV, MKV) launch_attn_row<P, HDV, MKV>(a, scale, R, st)
#define ATT_MK(P, HDV)                 \
  if (Lk <= 128) ATT(P, HDV, 2);       \
  else if (Lk <= 256) ATT(P, HDV, 4);  \
  else ATT(P, HDV, 8);
  if (C == 256 && hd == 32) { ATT_MK(4, 32) }
  else if (C == 256) { ATT_MK(4, 64) }
  else if (hd == 32) { ATT_MK(8, 32) }
  else { ATT_MK(8, 64) }
#undef ATT_MK
#undef ATT
  return retr_check_launch("dec_attn_row");
}

int retr_dec_ffn(const void* n3, int R, int C, const void* w1, const float* b1, const void* w2,
                 int F, float* slabs, void* stream) {
  RETR_REQUIRE((C == 256 || C == 512) && F % 32 == 0, "dec_ffn: C=%d F=%d", C, F);
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(F / 32, cdiv(R, 16));
  if (C == 256)
    hipLaunchKernelGGL(dec_ffn_kernel<4>, grid, dim3(64), 0, st, (const bf16*)n3, R,
                       (const bf16*)w1, b1, (const bf16*)w2, F, slabs);
  else
    hipLaunchKernelGGL(dec_ffn_kernel<8>, grid, dim3(64), 0, st, (const bf16*)n3, R,
                       (const bf16*)w1, b1, (const bf16*)w2, F, slabs);
  return retr_check_launch("dec_ffn");
}

int retr_dec_ffn_ln(const float* xin, const float* hslab, int nslab, const float* bo,
                    const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                    const void* w1, const float* b1, const void* w2, int F, float* slabs,
                    void* stream) {
  RETR_REQUIRE((C == 256 || C == 512) && F % 32 == 0 && nslab >= 0 && nslab <= 16,
               "dec_ffn_ln: C=%d F=%d nslab=%d (<= 16)", C, F, nslab);
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(F / 32, cdiv(R, 16));
#define FL(P, MS) hipLaunchKernelGGL((dec_ffn_ln_kernel<P, MS, 32>), grid, dim3(256), 0, st, xin, \
                                     hslab, nslab, bo, gamma, beta, eps, xout, R,                  \
                                     (const bf16*)w1, b1, (const bf16*)w2, F, slabs)
  if (C == 256) { if (nslab <= 8) FL(4, 8); else FL(4, 16); }
  else { if (nslab <= 8) FL(8, 8); else FL(8, 16); }
#undef FL
  return retr_check_launch("dec_ffn_ln");
}

int retr_dec_ffn_ln64(const float* xin, const float* hslab, int nslab, const float* bo,
                      const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                      const void* w1, const float* b1, const void* w2, int F, float* slabs,
                      void* stream) {
  RETR_REQUIRE((C == 256 || C == 512) && F % 64 == 0 && nslab >= 0 && nslab <= 16,
               "dec_ffn_ln64: C=%d F=%d nslab=%d (<= 16)", C, F, nslab);
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(F / 64, cdiv(R, 16));
  // 8 waves (2 LayerNorm rows, 2 FFN2 column tiles each) unless RETR_TUNE_DEC_WAVES asks for 4
  const int kn = retr_tune_get(RETR_TUNE_DEC_WAVES);
  const bool w8 = C == 256 && nslab <= 8 && kn != 1 && kn != 2;
  // 16 waves (one LayerNorm row, one FFN2 column tile each) by default: greedy 0.227 -> 0.223
  // ms/step; RETR_TUNE_DEC_WAVES 4 keeps 8
  if (w8 && kn != 4) {
    hipLaunchKernelGGL((dec_ffn_ln_kernel<4, 8, 64, 16>), grid, dim3(1024), 0, st, xin, hslab,
                       nslab, bo, gamma, beta, eps, xout, R, (const bf16*)w1, b1,
                       (const bf16*)w2, F, slabs);
    return retr_check_launch("dec_ffn_ln64");
  }
#define FL(P, MS) hipLaunchKernelGGL((dec_ffn_ln_kernel<P, MS, 64>), grid, dim3(256), 0, st, xin, \
                                     hslab, nslab, bo, gamma, beta, eps, xout, R,                  \
                                     (const bf16*)w1, b1, (const bf16*)w2, F, slabs)
  if (w8)
    hipLaunchKernelGGL((dec_ffn_ln_kernel<4, 8, 64, 8>), grid, dim3(512), 0, st, xin, hslab, nslab,
                       bo, gamma, beta, eps, xout, R, (const bf16*)w1, b1, (const bf16*)w2, F,
                       slabs);
  else if (C == 256) { if (nslab <= 8) FL(4, 8); else FL(4, 16); }
  else { if (nslab <= 8) FL(8, 8); else FL(8, 16); }
#undef FL
  return retr_check_launch("dec_ffn_ln64");
}

int retr_dec_ffn_ln128(const float* xin, const float* hslab, int nslab, const float* bo,
                       const float* gamma, const float* beta, float eps, float* xout, int R,
                       int C, const void* w1, const float* b1, const void* w2, int F,
                       float* slabs, void* stream) {
  RETR_REQUIRE(C == 256 && F % 128 == 0 && nslab >= 0 && nslab <= 8,
               "dec_ffn_ln128: C=%d F=%d nslab=%d (C 256, nslab <= 8)", C, F, nslab);
  if (R == 0) return 0;
  // 8 waves: FFN1 column tile w (16 hidden units) each, 2 FFN2 column tiles x 4 K-steps each
  // (RETR_TUNE_DEC_WAVES 3, sweeps: 16 waves, one LayerNorm row / FFN2 tile each)
  if (retr_tune_get(RETR_TUNE_DEC_WAVES) == 3)
    hipLaunchKernelGGL((dec_ffn_ln_kernel<4, 8, 128, 16>), dim3(F / 128, cdiv(R, 16)), dim3(1024),
                       0, (hipStream_t)stream, xin, hslab, nslab, bo, gamma, beta, eps, xout, R,
                       (const bf16*)w1, b1, (const bf16*)w2, F, slabs);
  else
    hipLaunchKernelGGL((dec_ffn_ln_kernel<4, 8, 128, 8>), dim3(F / 128, cdiv(R, 16)), dim3(512), 0,
                       (hipStream_t)stream, xin, hslab, nslab, bo, gamma, beta, eps, xout, R,
                       (const bf16*)w1, b1, (const bf16*)w2, F, slabs);
  return retr_check_launch("dec_ffn_ln128");
}

int retr_dec_linear_bf16(const void* x, long ldx, const void* w, long ldw, const float* bias,
                         void* y, long ldy, int M, int N, int K, int relu, void* stream) {
  RETR_REQUIRE(M >= 0 && M <= 4096 && N > 0 && K > 0 && K % 32 == 0 && ldx % 8 == 0 &&
                   ldw % 8 == 0 && (((uintptr_t)x | (uintptr_t)w) & 15) == 0,
               "dec_linear_bf16: M=%d N=%d K=%d (M <= 4096, K %% 32, 16-byte rows)", M, N, K);
  if (M == 0) return 0;
  hipLaunchKernelGGL(dec_linear_bf16_kernel, dim3(cdiv(N, 16), cdiv(M, 16)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)x, ldx, (const bf16*)w, ldw, bias,
                     (bf16*)y, ldy, M, N, K, relu);
  return retr_check_launch("dec_linear_bf16");
}

int retr_dec_linear_f32(const float* x, long ldx, const float* w, long ldw, const float* bias,
                        float* y, long ldy, int M, int N, int K, int relu, const float* res,
                        long ldr, void* stream) {
  return retr_dec_linear3_f32(1, x, ldx, w, ldw, bias, y, ldy, N, relu, res, ldr, nullptr, 0,
                              nullptr, 0, nullptr, nullptr, 0, 0, 0, nullptr, 0, nullptr, 0,
                              nullptr, 0, nullptr, nullptr, 0, 0, 0, nullptr, 0, M, K, stream);
}

int retr_dec_linear3_f32(int n, const float* x0, long ldx0, const float* w0, long ldw0,
                         const float* b0, float* y0, long ldy0, int N0, int relu0,
                         const float* r0, long ldr0, const float* x1, long ldx1, const float* w1,
                         long ldw1, const float* b1, float* y1, long ldy1, int N1, int relu1,
                         const float* r1, long ldr1, const float* x2, long ldx2, const float* w2,
                         long ldw2, const float* b2, float* y2, long ldy2, int N2, int relu2,
                         const float* r2, long ldr2, int M, int K, void* stream) {
  RETR_REQUIRE(n >= 1 && n <= 3 && M >= 0 && M <= 64 && K > 0 && K % 16 == 0,
               "dec_linear3_f32: n=%d M=%d K=%d (M <= 64, K %% 16)", n, M, K);
  LinF32Group g{{{x0, w0, b0, y0, r0, ldx0, ldw0, ldy0, ldr0, N0, relu0},
                 {x1, w1, b1, y1, r1, ldx1, ldw1, ldy1, ldr1, N1, relu1},
                 {x2, w2, b2, y2, r2, ldx2, ldw2, ldy2, ldr2, N2, relu2}}};
  int nmax = 0;
  for (int q = 0; q < n; ++q) {
    const LinF32Seg& sg = g.s[q];
    RETR_REQUIRE(sg.N > 0 && sg.ldx % 4 == 0 && sg.ldw % 4 == 0 &&
                     (((uintptr_t)sg.x | (uintptr_t)sg.w) & 15) == 0,
                 "dec_linear3_f32[%d]: N=%d, 16-byte rows", q, sg.N);
    nmax = sg.N > nmax ? sg.N : nmax;
  }
  if (M == 0) return 0;
  hipLaunchKernelGGL(dec_linear_f32_kernel, dim3(cdiv(nmax, 16), 1, n), dim3(256), 0,
                     (hipStream_t)stream, g, M, K);
  return retr_check_launch("dec_linear_f32");
}

#ifdef RETR_DEC_TIMING
int retr_dec_timing_read(long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dec_t), sizeof(long long) * 16);
}
#endif

}  // extern "C"
