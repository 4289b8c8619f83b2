// Linear layers (nn.Linear / MHA projections / MLP head) on the MFMA GEMM core.
//   forward : Y = epi(X W^T + b)           X [M][K], W [N][K]
//   dgrad   : dX = gate(dY W [+ addend])   dY [M][N]
//   wgrad   : dW += dY^T X                 (fp32, split-K + atomics)
//   bias    : db += colsum(dY)
#include "gemm2.hpp"
#include "splitk_fused.hpp"
#include "panel.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

using namespace retr;

namespace retr {
static __device__ int g_splitk_tickets[1 << 16];   // zero at load; every last arriver re-zeroes
static int g_splitk_cursor = 0;
int* splitk_tickets(int n) {
  static int* base = nullptr;
  if (!base) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_splitk_tickets)) != hipSuccess) return nullptr;
    base = (int*)a;
  }
  if (n > (1 << 16)) return nullptr;
  if (g_splitk_cursor + n > (1 << 16)) g_splitk_cursor = 0;
  int* p = base + g_splitk_cursor;
  g_splitk_cursor += (n + 63) / 64 * 64;
  return p;
}
}  // namespace retr

namespace {

// bf16 forward / data-gradient GEMMs with enough 128x128 tiles to fill the GPU (MLP head, FFN
// expansions) go to the LDS-DMA kernels of gemm2.hpp; the rest keep the occupancy-sized
// register-staged kernel.
template <int FAM, typename T, class LA, class LB, class EP>
int launch_linear(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, hipStream_t st,
                  const char* what) {
  if constexpr (sizeof(T) == 2) {
    // sweep override (tools/linear_micro.py): every bf16 linear through launch_big's tile
    if (retr_tune_get(RETR_TUNE_BIG_TILE) != 0)
      return launch_big<FAM>(la, lb, ep, M, N, K, 1, st, what);
    // RETR_TUNE_LIN_SMALL = 2 (sweeps; not the default, see retr_linear_splits): few output
    // tiles on the 32x64 LDS-DMA tile (4 waves side by side over 64 columns, S2 ring)
    {
      const long b128 = (long)cdiv(M, 128) * cdiv(N, 128), b64 = (long)cdiv(M, 64) * cdiv(N, 64);
      if (b128 < 160 && K >= 128 && (K >= 1024 || b64 < 192) &&
          retr_tune_get(RETR_TUNE_LIN_SMALL) == 2)
        return launch_gemm2<FAM, 32, 64, 1, 4, 2>(la, lb, ep, M, N, K, 1, st, what);
    }
    // short reductions into wide outputs (the FFN expansions and their gated data gradients):
    // the A panel resident in LDS, B streamed over a run of column tiles (panel.hpp) -- opt-in
    // only: measured slower than the 64x64 tile's wider grid (profiles/r4_ab_panel_rejected.txt)
    if (K <= 256 && K % 64 == 0 && N >= 1024 && M >= 64 && retr_tune_get(RETR_TUNE_PANEL) == 1)
      return launch_panel<FAM>(la, lb, ep, M, N, K, st, what);
    // short reductions (K <= 256: the FFN expansions) run 15-20 % faster on the 64x64
    // two-stage tile than on 128x128 (tools/linear_micro.py, profiles/r2_linear_tiles.txt)
    if ((long)cdiv(M, 128) * cdiv(N, 128) >= 160 && K >= 128)
      return launch_big<FAM>(la, lb, ep, M, N, K, 1, st, what,
                             K <= 256 && N <= 4096 && retr_tune_get(RETR_TUNE_BIG_TILE) == 0);
    // K = 256 on few output tiles (the d_model-256 projections): every K-step fetched at once
    // (same bits as the double-buffered loop; graphed cfg2 step 9.405 -> 9.344 ms,
    // profiles/r6_ab_lin_k256.txt); knob 1 keeps the loop
    if (K == 256 && (long)cdiv(M, 128) * cdiv(N, 128) < 240 &&
        retr_tune_get(RETR_TUNE_LIN_K256) != 1) {
      if ((long)cdiv(M, 64) * cdiv(N, 64) >= 192 || N < 64)
        return launch_short<FAM, 64, 64>(la, lb, ep, M, N, K, st, what);
      return launch_short<FAM, 32, 64>(la, lb, ep, M, N, K, st, what);
    }
  }
  return launch_sized<FAM, T>(la, lb, ep, M, N, K, st, what);
}

template <typename T, typename TO>
int linear_fwd_t(const void* x, long ldx, const void* w, long ldw, const float* bias, void* y,
                 long ldy, int M, int N, int K, int relu, const float* res, long ldr, float p,
                 unsigned long long seed, hipStream_t st) {
  DenseK<T> la{(const T*)x, ldx, M, K};
  DenseK<T> lb{(const T*)w, ldw, N, K};
  DropoutParams dp = make_dp(p, seed);
  EpiFwd<TO, float> ep{(TO*)y, ldy, bias, res, ldr, relu, dp, (long)N};
  ep.set_vec();
  return launch_linear<kFamLinearFwd, T>(la, lb, ep, M, N, K, st, "linear_fwd");
}

template <typename T, typename TO, typename TA>
int linear_dgrad_t(const void* dy, long lddy, const void* w, long ldw, void* dx, long lddx,
                   int M, int N, int K, const void* addend, long lda, const void* gate, long ldg,
                   int w_trans, hipStream_t st) {
  // dX[m][k] = sum_n dY[m][n] W[n][k]:  A = dY (K-dim = N), B(k, n) = W[n][k].
  // w_trans: the caller passes W^T stored [K][N] (K-contiguous B operand, no LDS transpose).
  DenseK<T> la{(const T*)dy, lddy, M, N};
  EpiDgrad<TO, TA, T> ep{(TO*)dx, lddx, (const TA*)addend, lda, (const T*)gate, ldg};
  ep.set_vec();
  if (w_trans) {
    DenseK<T> lb{(const T*)w, ldw, K, N};
    return launch_linear<kFamLinearDgrad, T>(la, lb, ep, M, K, N, st, "linear_dgrad");
  }
  DenseT<T> lb{(const T*)w, ldw, K, N};
  return launch_linear<kFamLinearDgrad, T>(la, lb, ep, M, K, N, st, "linear_dgrad");
}

// Split-K linears (few output tiles, long reduction: the FFN down-projections at d_model 256,
// the FFN up-projections' data gradients, the vocabulary head's data gradient): the slices
// write fp32 slabs ws[s][M][N] with plain stores; slab_epilogue_kernel adds them in slice order
// (deterministic) and runs the GEMM's own epilogue (bias / ReLU / dropout / residual, or addend
// / ReLU gate) on the sum.
template <class EP>
__global__ void slab_epilogue_kernel(const float* ws, int splits, int M, int N, EP ep) {
  const int CH = (N + 7) / 8;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)M * CH) return;
  const int m = (int)(i / CH), n = (int)(i % CH) * 8;
  const long MN = (long)M * N;
  const float* p = ws + (long)m * N + n;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n + 8 <= N && N % 4 == 0) {
    // the epilogue's operands (residual / addend / gate) in flight with the slabs
    typename PreOf<EP>::type pre;
    if constexpr (has_prefetch<EP>::value) ep.fetch8(m, n, pre);
    int s = 0;
    for (; s + 3 < splits; s += 4) {
      f32x4 a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = *(const f32x4*)(p + (s + u) * MN);
        b[u] = *(const f32x4*)(p + (s + u) * MN + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += a[u][e], v[e + 4] += b[u][e];
    }
    for (; s < splits; ++s) {
      const f32x4 a = *(const f32x4*)(p + s * MN), b = *(const f32x4*)(p + s * MN + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += a[e], v[e + 4] += b[e];
    }
    if constexpr (has_prefetch<EP>::value) ep.apply8p(m, n, v, pre);
    else ep.apply8(m, n, v);
    return;
  }
  for (int e = 0; e < 8 && n + e < N; ++e) {
    float t = 0.f;
    for (int s = 0; s < splits; ++s) t += p[s * MN + e];
    ep.apply(m, n + e, t);
  }
}

// the K-slice count launch_big / launch_gemm will actually use for `splits` requested
int norm_splits_k(int K, int BK, int splits) {
  const int ksteps = cdiv(K, BK);
  if (splits > ksteps) splits = ksteps;
  if (splits < 1) splits = 1;
  return cdiv(K, cdiv(ksteps, splits) * BK);
}


// The split-K slices alone (fp32 slabs ws[s][M][N]); the caller runs the slab epilogue.
template <typename T, class LA, class LB>
int splitk_slabs(const LA& la, const LB& lb, int M, int N, int K, float* ws, int splits,
                 int fam_dgrad, hipStream_t st, const char* what) {
  EpiAccF32 acc{ws, (long)N, 0, 0, 1, nullptr};
  acc.split_stride = (long)M * N;
  acc.set_vec();
  if constexpr (sizeof(T) == 2) {
    return fam_dgrad ? launch_big<kFamLinearDgrad>(la, lb, acc, M, N, K, splits, st, what)
                     : launch_big<kFamLinearFwd>(la, lb, acc, M, N, K, splits, st, what);
  } else {
    return fam_dgrad ? launch_gemm<kFamLinearDgrad, T, 64, 64>(la, lb, acc, M, N, K, splits, st, what)
                     : launch_gemm<kFamLinearFwd, T, 64, 64>(la, lb, acc, M, N, K, splits, st, what);
  }
}

// Slab epilogue of a residual-stream linear (fp32 out, N = 256 NCH) fused with the LayerNorm
// that reads its output next (the following pre-norm block's, or the stack's final norm): one
// wave per row, a lane owns 4 consecutive columns per 256-column chunk.  The slab sum (slice
// order), the EpiFwd arithmetic (bias, ReLU, dropout, residual) and the LayerNorm (ln_fwd4's
// statistics and output expressions, norm.hip) are each the unfused kernels' own, so out, LN(out),
// LN(out) + pos, mean and rstd equal the slab_epilogue_kernel + retr_layernorm_fwd path bitwise;
// the LayerNorm launch and its re-read of out are gone.
template <int NCH>
__global__ void __launch_bounds__(256)
slab_epilogue_ln_kernel(const float* ws, int splits, int M, EpiFwd<float, float> ep,
                        retr_ln_out ln) {
  constexpr int N = 256 * NCH;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const long MN = (long)M * N;
  const float* p = ws + (long)row * N + 4 * lane;
  f32x4 v[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the epilogue's and the LayerNorm's row operands (bias, residual, gamma, beta, position row)
  // issued up front with the slabs: one memory round trip, not one per operand behind the slab
  // sum.  No branch around a load (a conditional load drains the load counter at the join): an
  // absent operand reads the row's first slab instead and is not used.
  const float* bp = ep.bias ? ep.bias + 4 * lane : p;
  const float* rp = ep.res ? ep.res + (long)row * ep.ldr + 4 * lane : p;
  const float* pr = (ln.y2 && ln.pos) ? ln.pos + (long)(row % ln.period) * N + 4 * lane : p;
  f32x4 ob[NCH], orr[NCH], og[NCH], obe[NCH], opos[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    ob[j] = *(const f32x4*)(bp + 256 * j);
    orr[j] = *(const f32x4*)(rp + 256 * j);
    og[j] = *(const f32x4*)(ln.gamma + 4 * lane + 256 * j);
    obe[j] = *(const f32x4*)(ln.beta + 4 * lane + 256 * j);
    opos[j] = *(const f32x4*)(pr + 256 * j);
  }
  // every load of a group of four slices in flight before the adds (slice order kept)
  int s0 = 0;
  for (; s0 + 3 < splits; s0 += 4) {
    f32x4 a[4][NCH];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < NCH; ++j) a[u][j] = *(const f32x4*)(p + (s0 + u) * MN + 256 * j);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] += a[u][j][e];
  }
  for (; s0 < splits; ++s0)
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const f32x4 a = *(const f32x4*)(p + s0 * MN + 256 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] += a[e];
    }
  const uint32_t rk = ep.dp.thresh ? drop_row_key(dp_seed(ep.dp), (uint32_t)row) : 0u;
  const uint32_t th = drop_th16(ep.dp.thresh);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * lane + 256 * j;
    if (ep.bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] += ob[j][e];
    }
    if (ep.relu == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = fmaxf(v[j][e], 0.f);
    }
    if (ep.dp.thresh) {
      const uint32_t km = drop_keep4(rk, (uint32_t)c, th);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = ((km >> e) & 1u) ? v[j][e] * ep.dp.scale : 0.f;
    }
    if (ep.res) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] += orr[j][e];
    }
    if (ep.relu == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = fmaxf(v[j][e], 0.f);
    }
    *(f32x4*)(ep.out + (long)row * ep.ldo + c) = v[j];
    s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  }
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[j][e] - mean;
      q += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / N + ln.eps);
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * lane + 256 * j;
    const f32x4 g = og[j], b = obe[j];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mean) * rstd * g[e] + b[e];
    if (ln.y)
      *(bf16x4*)((bf16*)ln.y + (long)row * ln.ldy + c) =
          bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
    if (ln.y2) {
      const f32x4 o2 = o + opos[j];
      *(bf16x4*)((bf16*)ln.y2 + (long)row * ln.ldy + c) =
          bf16x4{(bf16)o2[0], (bf16)o2[1], (bf16)o2[2], (bf16)o2[3]};
    }
  }
  if (lane == 0) {
    if (ln.mean) ln.mean[row] = mean;
    if (ln.rstd) ln.rstd[row] = rstd;
  }
}

// Row-complete forward linear with the next LayerNorm in its epilogue (round 6): the GEMM tile
// spans all N = 256 output columns (gemm2_tile BM x 256, the whole K in one pass), so its
// epilogue owns complete rows -- EpiFwd's bias / dropout / residual arithmetic and the
// LayerNorm outputs of slab_epilogue_ln_kernel, from the fp32 tile in LDS instead of summed
// split-K slabs: no slab round trip through HBM, no second launch.  (One fp32 MFMA chain over K
// per output instead of four slab chains summed: the same values to fp32 reassociation.)
struct EpiRowLN {
  static constexpr bool kRows = true;
  EpiFwd<float, float> ep;
  retr_ln_out ln;
  RETR_DEVICE void rows(const float* ct, int ld, int m0, int nrows, int tid, int nthreads) const {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    constexpr int N = 256;
    const int lane = tid & 63, nw = nthreads >> 6;
    const int c = 4 * lane;
    const uint32_t th = drop_th16(ep.dp.thresh);
    for (int r = tid >> 6; r < nrows; r += nw) {
      const int row = m0 + r;
      f32x4 v = *(const f32x4*)(ct + r * ld + c);
      const uint32_t rk = ep.dp.thresh ? drop_row_key(dp_seed(ep.dp), (uint32_t)row) : 0u;
      if (ep.bias) {
        const f32x4 b = *(const f32x4*)(ep.bias + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += b[e];
      }
      if (ep.relu == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (ep.dp.thresh) {
        const uint32_t km = drop_keep4(rk, (uint32_t)c, th);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ((km >> e) & 1u) ? v[e] * ep.dp.scale : 0.f;
      }
      if (ep.res) {
        const f32x4 rr = *(const f32x4*)(ep.res + (long)row * ep.ldr + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += rr[e];
      }
      if (ep.relu == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      *(f32x4*)(ep.out + (long)row * ep.ldo + c) = v;
      const float mean = wave_sum((v[0] + v[1]) + (v[2] + v[3])) / N;
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[e] - mean;
        q += d * d;
      }
      const float rstd = 1.0f / sqrtf(wave_sum(q) / N + ln.eps);
      const f32x4 g = *(const f32x4*)(ln.gamma + c), b = *(const f32x4*)(ln.beta + c);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[e] - mean) * rstd * g[e] + b[e];
      if (ln.y)
        *(bf16x4*)((bf16*)ln.y + (long)row * ln.ldy + c) =
            bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      if (ln.y2) {
        const f32x4 o2 = o + *(const f32x4*)(ln.pos + (long)(row % ln.period) * N + c);
        *(bf16x4*)((bf16*)ln.y2 + (long)row * ln.ldy + c) =
            bf16x4{(bf16)o2[0], (bf16)o2[1], (bf16)o2[2], (bf16)o2[3]};
      }
      if (lane == 0) {
        if (ln.mean) ln.mean[row] = mean;
        if (ln.rstd) ln.rstd[row] = rstd;
      }
    }
  }
  // (the per-chunk epilogue interface gemm2_tile instantiates but never calls with kRows)
  RETR_DEVICE bool lane_contiguous() const { return false; }
  RETR_DEVICE void apply(int, int, float) const {}
  RETR_DEVICE void apply8(int, int, float (&)[8]) const {}
  RETR_DEVICE void empty_split(int, int) const {}
};

int launch_rowln(int variant, const DenseK<bf16>& la, const DenseK<bf16>& lb, const EpiRowLN& ep,
                 int M, int K, hipStream_t st) {
  constexpr const char* what = "linear_fwd_rowln";
  switch (variant) {
    case 2: return launch_gemm2<kFamLinearFwd, 32, 256, 1, 4, 2, 1>(la, lb, ep, M, 256, K, 1, st, what);
    case 4: return launch_gemm2<kFamLinearFwd, 32, 256, 1, 4, 4, 1>(la, lb, ep, M, 256, K, 1, st, what);
    case 5: return launch_gemm2<kFamLinearFwd, 64, 256, 2, 4, 3, 1>(la, lb, ep, M, 256, K, 1, st, what);
    default: return launch_gemm2<kFamLinearFwd, 32, 256, 1, 4, 3, 1>(la, lb, ep, M, 256, K, 1, st, what);
  }
}

template <typename T, class LA, class LB, class EP>
int splitk_run(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, float* ws,
               int splits, int fam_dgrad, hipStream_t st, const char* what) {
  constexpr int BK = Elem<T>::BK;
  splits = norm_splits_k(K, BK, splits);
  if constexpr (sizeof(T) == 2) {
    // slice reduction + epilogue by each tile's last-arriving block (splitk_fused.hpp)
    if (retr_tune_get(RETR_TUNE_SPLITK_FUSED) == 1 && N % 8 == 0 && splits > 1) {
      const long t128 = (long)cdiv(M, 128) * cdiv(N, 128) * splits;
      if (t128 >= 160)
        return fam_dgrad
                   ? launch_splitk_fused<kFamLinearDgrad, 128, 128, 4, 2, 2>(la, lb, ep, ws, M, N, K, splits, st, what)
                   : launch_splitk_fused<kFamLinearFwd, 128, 128, 4, 2, 2>(la, lb, ep, ws, M, N, K, splits, st, what);
      return fam_dgrad
                 ? launch_splitk_fused<kFamLinearDgrad, 64, 64, 2, 2, 2>(la, lb, ep, ws, M, N, K, splits, st, what)
                 : launch_splitk_fused<kFamLinearFwd, 64, 64, 2, 2, 2>(la, lb, ep, ws, M, N, K, splits, st, what);
    }
  }
  if (int e = splitk_slabs<T>(la, lb, M, N, K, ws, splits, fam_dgrad, st, what)) return e;
  const long chunks = (long)M * ((N + 7) / 8);
  hipLaunchKernelGGL((slab_epilogue_kernel<EP>), dim3((unsigned)cdiv(chunks, 256)), dim3(256), 0,
                     st, ws, splits, M, N, ep);
  return retr_check_launch(what);
}

template <typename T, typename TO>
int linear_fwd_splitk_t(const void* x, long ldx, const void* w, long ldw, const float* bias,
                        void* y, long ldy, int M, int N, int K, int relu, const float* res,
                        long ldr, float p, unsigned long long seed, float* ws, int splits,
                        hipStream_t st) {
  DenseK<T> la{(const T*)x, ldx, M, K};
  DenseK<T> lb{(const T*)w, ldw, N, K};
  EpiFwd<TO, float> ep{(TO*)y, ldy, bias, res, ldr, relu, make_dp(p, seed), (long)N};
  ep.set_vec();
  return splitk_run<T>(la, lb, ep, M, N, K, ws, splits, 0, st, "linear_fwd_splitk");
}

template <typename T, typename TO, typename TA>
int linear_dgrad_splitk_t(const void* dy, long lddy, const void* w, long ldw, void* dx, long lddx,
                          int M, int N, int K, const void* addend, long lda, const void* gate,
                          long ldg, int w_trans, float* ws, int splits, hipStream_t st) {
  DenseK<T> la{(const T*)dy, lddy, M, N};
  EpiDgrad<TO, TA, T> ep{(TO*)dx, lddx, (const TA*)addend, lda, (const T*)gate, ldg};
  ep.set_vec();
  if (w_trans) {
    DenseK<T> lb{(const T*)w, ldw, K, N};
    return splitk_run<T>(la, lb, ep, M, K, N, ws, splits, 1, st, "linear_dgrad_splitk");
  }
  DenseT<T> lb{(const T*)w, ldw, K, N};
  return splitk_run<T>(la, lb, ep, M, K, N, ws, splits, 1, st, "linear_dgrad_splitk");
}

// zero an fp32 [rows][cols] region with row stride ld (stream-ordered, graph-capturable)
int zero_f32(float* p, long ld, int rows, int cols, hipStream_t st) {
  hipError_t e = (ld == cols) ? hipMemsetAsync(p, 0, sizeof(float) * (size_t)rows * cols, st)
                              : hipMemset2DAsync(p, sizeof(float) * ld, 0, sizeof(float) * cols,
                                                 rows, st);
  if (e != hipSuccess) {
    retr_set_error("memset: %s", hipGetErrorString(e));
    return 1;
  }
  return 0;
}

// Deterministic column sums db[n] (=|+=) sum_m dY[m][n]: one 1024-thread block per 64 columns,
// wave w sums rows w, w+16, ... in order, the 16 wave partials are added in wave order.
template <typename T>
__global__ void __launch_bounds__(1024)
colsum_det_kernel(const T* dy, long ld, int M, int N, float* db, int accumulate) {
  __shared__ float part[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (n < N) {
#pragma unroll 8
    for (int m = wave; m < M; m += 16) s += to_f(dy[(long)m * ld + n]);
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += part[w][lane];
    db[n] = accumulate ? db[n] + t : t;
  }
}

template <typename T>
int colsum_det(const void* dy, long ld, int M, int N, float* db, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(colsum_det_kernel<T>, dim3(cdiv(N, 64)), dim3(1024), 0, st, (const T*)dy, ld,
                     M, N, db, accumulate);
  return retr_check_launch("bias_grad_det");
}

template <typename T>
int linear_wgrad_t(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw,
                   int M, int N, int K, float* db, int accumulate, hipStream_t st) {
  // dW[n][k] = sum_m dY[m][n] X[m][k]: A(n, m) = dY[m][n], B(k, m) = X[m][k]  (both [m][.])
  DenseT<T> la{(const T*)dy, lddy, N, M};
  DenseT<T> lb{(const T*)x, ldx, K, M};
  constexpr int BK = Elem<T>::BK;
  const bool big = N >= 512 && K >= 128;
  int s = big ? pick_splits(N, K, M, 128, 128, BK) : pick_splits(N, K, M, 64, 64, BK);
  if (retr_deterministic()) {
    // no split-K atomics, no fused (LDS-atomic) row sums: ordered column sums instead
    s = 1;
    if (db && colsum_det<T>(dy, lddy, M, N, db, accumulate, st)) return 1;
    db = nullptr;
  }
  if (!accumulate) {
    if (s > 1 && zero_f32(dw, lddw, N, K, st)) return 1;
    if (db && zero_f32(db, N, 1, N, st)) return 1;
  }
  EpiAccF32 ep{dw, lddw, s > 1, 0, !accumulate && s == 1, db};
  ep.set_vec();
  if constexpr (sizeof(T) == 2) {
    // LDS-DMA kernels for the bf16 weight gradients with enough tiles (the vocabulary head's
    // 30522 x 512: 956 tiles); RETR_TUNE_LIN_WGRAD 1 = the register-staged kernel
    const int tk = retr_tune_get(RETR_TUNE_LIN_WGRAD);
    if (big && tk != 1 && (long)cdiv(N, 128) * cdiv(K, 128) * s >= 256) {
      // no fused row sums in the LDS-DMA kernels: the bias gradient is an ordered column sum
      if (db) {
        if (colsum_det<T>(dy, lddy, M, N, db, accumulate, st)) return 1;
        ep.rowsum = nullptr;
      }
      // tools/wgrad_micro.py (profiles/r3_wgrad_micro.txt): vocabulary head 118 us register-
      // staged -> 99 us on the 4-wave 128x128 LDS-DMA tile (+ the column sum)
      if (tk == 2) return launch_gemm2<kFamLinearWgrad, 256, 256, 2, 4, 2>(la, lb, ep, N, K, M, s, st, "linear_wgrad");
      if (tk == 4) return launch_gemm2<kFamLinearWgrad, 128, 128, 4, 2, 2>(la, lb, ep, N, K, M, s, st, "linear_wgrad");
      return launch_gemm2<kFamLinearWgrad, 128, 128, 2, 2, 2>(la, lb, ep, N, K, M, s, st, "linear_wgrad");
    }
  }
  if (big) return launch_gemm<kFamLinearWgrad, T, 128, 128>(la, lb, ep, N, K, M, s, st, "linear_wgrad");
  return launch_gemm<kFamLinearWgrad, T, 64, 64>(la, lb, ep, N, K, M, s, st, "linear_wgrad");
}

// db[n] += sum_m dY[m][n]; one thread per column-pair, blocks stride over rows.
template <typename T>
__global__ void colsum_kernel(const T* dy, long ld, int M, int N, float* db, int rows_per_blk) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  int r0 = blockIdx.y * rows_per_blk, r1 = min(M, r0 + rows_per_blk);
  float s = 0.f;
  for (int m = r0; m < r1; ++m) s += to_f(dy[(long)m * ld + n]);
  atomicAdd(db + n, s);
}

}  // namespace

extern "C" {

int retr_linear_fwd(int dtype, const void* x, long ldx, const void* w, long ldw,
                    const float* bias, void* y, long ldy, int y_f32, int M, int N, int K, int relu,
                    const float* residual, long ldr, float drop_p, unsigned long long seed,
                    void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(M >= 0 && N > 0 && K > 0, "linear_fwd: bad shape M=%d N=%d K=%d", M, N, K);
  if (M == 0) return 0;
  if (dtype == RETR_BF16) {
    RETR_REQUIRE(K % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0, "linear_fwd: K/ld must be %%8");
    return y_f32 ? linear_fwd_t<bf16, float>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual, ldr, drop_p, seed, st)
                 : linear_fwd_t<bf16, bf16>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual, ldr, drop_p, seed, st);
  }
  RETR_REQUIRE(K % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0, "linear_fwd: K/ld must be %%4");
  return linear_fwd_t<float, float>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual, ldr,
                                    drop_p, seed, st);
}

int retr_linear_dgrad(int dtype, const void* dy, long lddy, const void* w, long ldw, void* dx,
                      long lddx, int dx_f32, int M, int N, int K, const void* addend,
                      int addend_f32, long lda, const void* gate, long ldg, int w_trans,
                      void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  if (dtype == RETR_BF16) {
    RETR_REQUIRE(N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0 && ldw % 8 == 0,
                 "linear_dgrad: N/K/ld must be %%8");
    if (dx_f32) {
      return addend_f32 ? linear_dgrad_t<bf16, float, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, st)
                        : linear_dgrad_t<bf16, float, bf16>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, st);
    }
    return addend_f32 ? linear_dgrad_t<bf16, bf16, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, st)
                      : linear_dgrad_t<bf16, bf16, bf16>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, st);
  }
  RETR_REQUIRE(N % 4 == 0 && K % 4 == 0 && lddy % 4 == 0 && ldw % 4 == 0,
               "linear_dgrad: N/K/ld must be %%4");
  return linear_dgrad_t<float, float, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda,
                                             gate, ldg, w_trans, st);
}

int retr_linear_splits(int dtype, int M, int N, int K) {
  // few 128x128 output tiles and a long reduction: split toward two blocks per CU, >= 8
  // K-steps per slice, at most 8 slices (bf16; fp32 keeps single-pass GEMMs).
  // tools/splitk_micro.py (profiles/r2_splitk_micro.txt): the vocabulary head's dgrad 276 us
  // single-pass -> 84 us at 8 slices; the FFN shapes gain little beyond 4
  // RETR_TUNE_LIN_SMALL = 2: K <= 2048 single-pass on the 32x64 LDS-DMA tile instead
  // (launch_linear) -- faster in isolation (tools/linear_micro.py splitk,
  // profiles/r3_linear_splitk.txt: M2048 14.7 -> 11.1 us fwd) but 0.1 ms/step slower in the
  // graphed step (profiles/r3_ab_lin_small.txt), so not the default
  if (dtype != RETR_BF16 || M <= 0) return 1;
  const long tiles = (long)cdiv(M, 128) * cdiv(N, 128);
  const int ksteps = cdiv(K, 64);
  if (tiles >= 160 || ksteps < 16) return 1;
  if (ksteps <= 32 && retr_tune_get(RETR_TUNE_LIN_SMALL) == 2) return 1;
  long s = (512 + tiles - 1) / tiles;
  if (s > ksteps / 8) s = ksteps / 8;
  if (s > 8) s = 8;
  return s < 2 ? 1 : norm_splits_k(K, 64, (int)s);
}

int retr_linear_fwd_splitk(int dtype, const void* x, long ldx, const void* w, long ldw,
                           const float* bias, void* y, long ldy, int y_f32, int M, int N, int K,
                           int relu, const float* residual, long ldr, float drop_p,
                           unsigned long long seed, float* ws, int splits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(splits >= 1 && ws != nullptr, "linear_fwd_splitk: splits=%d", splits);
  if (dtype == RETR_BF16) {
    RETR_REQUIRE(K % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0, "linear_fwd_splitk: K/ld must be %%8");
    return y_f32 ? linear_fwd_splitk_t<bf16, float>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual, ldr, drop_p, seed, ws, splits, st)
                 : linear_fwd_splitk_t<bf16, bf16>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual, ldr, drop_p, seed, ws, splits, st);
  }
  RETR_REQUIRE(K % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0, "linear_fwd_splitk: K/ld must be %%4");
  return linear_fwd_splitk_t<float, float>(x, ldx, w, ldw, bias, y, ldy, M, N, K, relu, residual,
                                           ldr, drop_p, seed, ws, splits, st);
}

int retr_linear_fwd_splitk_ln(int dtype, const void* x, long ldx, const void* w, long ldw,
                              const float* bias, float* y, long ldy, int M, int N, int K, int relu,
                              const float* residual, long ldr, float drop_p,
                              unsigned long long seed, float* ws, int splits,
                              const retr_ln_out* ln, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(splits >= 1 && ln != nullptr, "linear_fwd_splitk_ln: splits=%d", splits);
  auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  auto a8 = [](const void* q) { return ((uintptr_t)q & 7) == 0; };
  const bool fused = dtype == RETR_BF16 && ln->y_bf16 && N % 256 == 0 && N <= 512 &&
                     K % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldy % 4 == 0 &&
                     ldr % 4 == 0 && ln->ldy % 4 == 0 && a16(y) && a16(bias) && a16(residual) &&
                     a16(ws) && a16(ln->gamma) && a16(ln->beta) && a16(ln->pos) && a8(ln->y) &&
                     a8(ln->y2) && (ln->pos == nullptr || ln->period > 0) &&
                     ln->gamma != nullptr && ln->beta != nullptr;
  if (!fused) {
    // two launches with the same results: the (split-K) linear, then the LayerNorm
    if (int e = ws ? retr_linear_fwd_splitk(dtype, x, ldx, w, ldw, bias, y, ldy, 1, M, N, K,
                                            relu, residual, ldr, drop_p, seed, ws, splits, stream)
                   : retr_linear_fwd(dtype, x, ldx, w, ldw, bias, y, ldy, 1, M, N, K, relu,
                                     residual, ldr, drop_p, seed, stream))
      return e;
    return retr_layernorm_fwd(ln->y_bf16 ? RETR_BF16 : RETR_F32, y, ldy, ln->gamma, ln->beta,
                              ln->eps, M, N, ln->y, ln->ldy, ln->y2, ln->pos, ln->period,
                              ln->mean, ln->rstd, stream);
  }
  DenseK<bf16> la{(const bf16*)x, ldx, M, K};
  DenseK<bf16> lb{(const bf16*)w, ldw, N, K};
  // the row-complete tile with the LayerNorm in its epilogue (N = 256): by default for short
  // reductions (K <= 512: the attention out-projections, 4-8 K-steps), where the whole-K tile
  // costs no latency; long ones keep the split-K slabs (profiles/r6_ab_rowln_rejected.txt).
  // RETR_TUNE_ROWLN: 1 slabs always, 2-5 a row-complete variant always
  int rv = retr_tune_get(RETR_TUNE_ROWLN);
  if (rv == 0) rv = K <= 512 ? 2 : 1;
  if (N == 256 && rv >= 2) {
    EpiRowLN ep{EpiFwd<float, float>{y, ldy, bias, residual, ldr, relu, make_dp(drop_p, seed),
                                     (long)N},
                *ln};
    return launch_rowln(rv, la, lb, ep, M, K, st);
  }
  RETR_REQUIRE(ws != nullptr, "linear_fwd_splitk_ln: the split-K path needs a workspace");
  splits = norm_splits_k(K, Elem<bf16>::BK, splits);
  if (int e = splitk_slabs<bf16>(la, lb, M, N, K, ws, splits, 0, st, "linear_fwd_splitk_ln"))
    return e;
  EpiFwd<float, float> ep{y, ldy, bias, residual, ldr, relu, make_dp(drop_p, seed), (long)N};
  const dim3 grid((unsigned)cdiv(M, 4));
  if (N == 256)
    hipLaunchKernelGGL(slab_epilogue_ln_kernel<1>, grid, dim3(256), 0, st, ws, splits, M, ep, *ln);
  else
    hipLaunchKernelGGL(slab_epilogue_ln_kernel<2>, grid, dim3(256), 0, st, ws, splits, M, ep, *ln);
  return retr_check_launch("linear_fwd_splitk_ln");
}

int retr_linear_dgrad_splitk(int dtype, const void* dy, long lddy, const void* w, long ldw,
                             void* dx, long lddx, int dx_f32, int M, int N, int K,
                             const void* addend, int addend_f32, long lda, const void* gate,
                             long ldg, int w_trans, float* ws, int splits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(splits >= 1 && ws != nullptr, "linear_dgrad_splitk: splits=%d", splits);
  if (dtype == RETR_BF16) {
    RETR_REQUIRE(N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0 && ldw % 8 == 0,
                 "linear_dgrad_splitk: N/K/ld must be %%8");
    if (dx_f32)
      return addend_f32 ? linear_dgrad_splitk_t<bf16, float, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, ws, splits, st)
                        : linear_dgrad_splitk_t<bf16, float, bf16>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, ws, splits, st);
    return addend_f32 ? linear_dgrad_splitk_t<bf16, bf16, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, ws, splits, st)
                      : linear_dgrad_splitk_t<bf16, bf16, bf16>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend, lda, gate, ldg, w_trans, ws, splits, st);
  }
  RETR_REQUIRE(N % 4 == 0 && K % 4 == 0 && lddy % 4 == 0 && ldw % 4 == 0,
               "linear_dgrad_splitk: N/K/ld must be %%4");
  return linear_dgrad_splitk_t<float, float, float>(dy, lddy, w, ldw, dx, lddx, M, N, K, addend,
                                                    lda, gate, ldg, w_trans, ws, splits, st);
}

// the split-K data gradient's slices only: ws[splits][M][K] = partial dY[:, slice] W[slice, :]
// (fp32, plain stores) for a consumer that sums them itself (retr_layernorm_bwd_slabs); splits
// must already be a normalised slice count (retr_linear_splits' result)
int retr_linear_dgrad_slabs(int dtype, const void* dy, long lddy, const void* w, long ldw, int M,
                            int N, int K, int w_trans, float* ws, int splits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(dtype == RETR_BF16, "linear_dgrad_slabs: bf16 only");
  RETR_REQUIRE(N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0 && ldw % 8 == 0 && ws != nullptr,
               "linear_dgrad_slabs: N/K/ld must be %%8");
  RETR_REQUIRE(splits >= 1 && norm_splits_k(N, 64, splits) == splits,
               "linear_dgrad_slabs: splits=%d is not a normalised slice count for N=%d", splits, N);
  DenseK<bf16> la{(const bf16*)dy, lddy, M, N};
  if (w_trans) {
    DenseK<bf16> lb{(const bf16*)w, ldw, K, N};
    return splitk_slabs<bf16>(la, lb, M, K, N, ws, splits, 1, st, "linear_dgrad_slabs");
  }
  DenseT<bf16> lb{(const bf16*)w, ldw, K, N};
  return splitk_slabs<bf16>(la, lb, M, K, N, ws, splits, 1, st, "linear_dgrad_slabs");
}

int retr_linear_wgrad(int dtype, const void* dy, long lddy, const void* x, long ldx, float* dw,
                      long lddw, int M, int N, int K, float* db, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  if (dtype == RETR_BF16) {
    // a ragged N reads the 16-byte group past row N-1 of dY: the row stride must cover it
    RETR_REQUIRE(lddy >= (N + 7) / 8 * 8 && K % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0,
                 "linear_wgrad: K/ld must be %%8 and ld(dy) >= N rounded up to 8");
    return linear_wgrad_t<bf16>(dy, lddy, x, ldx, dw, lddw, M, N, K, db, accumulate, st);
  }
  RETR_REQUIRE(lddy >= (N + 3) / 4 * 4 && K % 4 == 0 && lddy % 4 == 0 && ldx % 4 == 0,
               "linear_wgrad: K/ld must be %%4 and ld(dy) >= N rounded up to 4");
  return linear_wgrad_t<float>(dy, lddy, x, ldx, dw, lddw, M, N, K, db, accumulate, st);
}

int retr_bias_grad(int dtype, const void* dy, long lddy, int M, int N, float* db, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  if (retr_deterministic()) {
    return dtype == RETR_BF16 ? colsum_det<bf16>(dy, lddy, M, N, db, 1, st)
                              : colsum_det<float>(dy, lddy, M, N, db, 1, st);
  }
  int rows = 64;
  dim3 grid(cdiv(N, 256), cdiv(M, rows));
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)dy, lddy, M, N, db, rows);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, (const float*)dy, lddy, M, N, db, rows);
  return retr_check_launch("bias_grad");
}

}  // extern "C"
