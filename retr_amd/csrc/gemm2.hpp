// Large-tile bf16 MFMA GEMM for gfx950 with LDS-DMA (global_load_lds_dwordx4) staging.
//
//   C[m][n] = sum_k A(m,k) * B(n,k), same loader / epilogue contracts as gemm.hpp.
//
//  * Operand tiles go straight from global memory into LDS (no VGPR round trip, no ds_write
//    pass): a wave-instruction writes 1 KiB, lane-linear, at a wave-uniform LDS base.  The
//    LDS images are the ones gemm.hpp's fragment reads expect (XOR-swizzled [rows][8 chunks]
//    for k-contiguous operands, the k-major [BK][rows] image read with ds_read_b64_tr_b16 for
//    row-contiguous ones); the swizzle is applied on the SOURCE side: each lane loads the
//    logical chunk that belongs at its linear slot.  For every tile shape used here that
//    logical chunk column is a per-thread constant, so the loaders keep their k cursors.
//  * Chunks outside the operand (conv padding, ragged M/N/K edges) are read from a zero page.
//  * S-stage LDS ring, one raw s_barrier per K-step: tile t+S-1 is issued right after the
//    barrier that retires tile t, so S-2 tiles stay in flight across it (counted vmcnt, never
//    a vmcnt(0) in the steady state: __syncthreads() would drain the DMA queue).
//  * BM x BN block tile over (BM/WM) x (BN/WN) waves, 16x16x32 bf16 MFMA, fp32 accumulation;
//    epilogue through LDS (8 consecutive columns per thread, 16-byte global accesses).
//  * XCD-aware block order and split-K over blockIdx.y as in gemm.hpp.
#pragma once
#include <type_traits>
#include <utility>

#include "gemm.hpp"
#include "../../include/retr_hip.h"

namespace retr {

static __device__ __attribute__((aligned(64))) unsigned int g_zero_page[64];  // 256 B of zeros

RETR_DEVICE void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                   0, 0);
}

template <int N>
RETR_DEVICE void wait_vmcnt_lgkm0() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

RETR_DEVICE void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Loaders with kUniformK = true keep the K cursor wave-uniform (it only depends on the block's
// K range, so the compiler holds it in SGPRs): the per-thread 16-byte chunk offset goes into
// the row context instead (row_ctx_c(r, coff)), and kcur(kb) takes the block's K start.
template <class L, class = void>
struct uniform_k : std::false_type {};
template <class L>
struct uniform_k<L, std::void_t<decltype(L::kUniformK)>> : std::integral_constant<bool, L::kUniformK> {};

// Loaders with addr_or(ctx, cursor, fallback) return `fallback` (the zero page) themselves for
// a chunk outside the operand: one select instead of a null result re-tested by the stager.
template <class L, class = void>
struct has_addr_or : std::false_type {};
template <class L>
struct has_addr_or<L, std::void_t<decltype(std::declval<const L&>().addr_or(
                          std::declval<const typename L::Ctx&>(),
                          std::declval<const typename L::KCur&>(), (const void*)nullptr))>>
    : std::true_type {};

template <class L>
RETR_DEVICE const void* chunk_src(const L& l, const typename L::Ctx& c, const typename L::KCur& k) {
  if constexpr (has_addr_or<L>::value) {
    return l.addr_or(c, k, (const void*)g_zero_page);
  } else {
    const void* p = l.addr(c, k);
    return p ? p : (const void*)g_zero_page;
  }
}

// LDS-DMA stager of one ROWS x BK operand tile (bf16) for an NT-thread block.
template <int ROWS, int NT, class L>
struct GStager {
  static constexpr int EPC = 8, BK = 64;
  static constexpr int CPR = ROWS / 8;          // 16-byte slots per k-row of the k-major image
  static constexpr int NCH = ROWS * 8 / NT;     // chunks per thread per tile
  static_assert(NCH >= 1 && (ROWS * 8) % NT == 0, "tile too small for the block");
  // (uniform-K loaders keep one row context per chunk, so each chunk may take its own swizzle
  // column; the per-chunk-cursor form needs one column for all of a thread's k rows)
  static_assert(L::kContig || (NT % CPR == 0 &&
                               (uniform_k<L>::value || (8 * NT / ROWS) % 16 == 0)),
                "k-major image: thread's k rows must share one swizzle phase");
  static constexpr bool kU = uniform_k<L>::value;
  typename L::Ctx ctx[(L::kContig || kU) ? NCH : 1];
  typename L::KCur kc[(L::kContig || kU) ? 1 : NCH];

  RETR_DEVICE void init(const L& l, int row0, int tid, int kb) {
    if constexpr (L::kContig) {
      // linear slot (row r = tid/8 + (NT/8) i, slot tid%8) holds chunk slot ^ ((r>>1)&7)
      const int c = (tid & 7) ^ ((tid >> 4) & 7);
      if constexpr (uniform_k<L>::value) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) ctx[i] = l.row_ctx_c(row0 + (tid >> 3) + (NT / 8) * i, c * EPC);
        kc[0] = l.kcur(kb);
      } else {
#pragma unroll
        for (int i = 0; i < NCH; ++i) ctx[i] = l.row_ctx(row0 + (tid >> 3) + (NT / 8) * i);
        kc[0] = l.kcur(kb + c * EPC);
      }
    } else {
      // linear slot (k = tid/CPR + (NT/CPR) i, slot tid%CPR) holds row-chunk slot ^ (f(k)/2)
      const int k0 = tid / CPR, slot = tid % CPR;
      auto phase = [](int k) {
        if constexpr (ROWS >= 128) return 4 * ((k & 3) | (((k >> 3) & 1) << 2));
        else return 4 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
      };
      const int c = slot ^ (phase(k0) >> 1);
      if constexpr (uniform_k<L>::value) {
        // one row context per k row of the thread (its k offset and swizzle column baked in),
        // one block cursor
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
          const int k = k0 + (NT / CPR) * i;
          ctx[i] = l.row_ctx_c(row0 + (slot ^ (phase(k) >> 1)) * EPC, k);
        }
        kc[0] = l.kcur(kb);
      } else {
        ctx[0] = l.row_ctx(row0 + c * EPC);
#pragma unroll
        for (int i = 0; i < NCH; ++i) kc[i] = l.kcur(kb + k0 + (NT / CPR) * i);
      }
    }
  }
  // issue the tile at the cursors into the image at `lds`, then advance the cursors
  RETR_DEVICE void issue(const L& l, char* lds, int wave) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const void* p = (L::kContig || kU) ? chunk_src(l, ctx[i], kc[0]) : chunk_src(l, ctx[0], kc[i]);
      glds16(p, lds + (NT * i + wave * 64) * 16);
      if constexpr (!L::kContig && !kU) l.advance(kc[i], BK);
    }
    if constexpr (L::kContig || kU) l.advance(kc[0], BK);
  }
};

template <int BM, int BN, int EPB>
constexpr int epi_bands() {
  return EPB > 0 ? EPB : ((size_t)BM * (BN + 4) * 4 > 160 * 1024 ? 2 : 1);
}

template <int BM, int BN, int S, int EPB>
constexpr size_t gemm2_lds_bytes() {
  constexpr size_t stage = (size_t)S * (BM + BN) * kBKBytes;
  constexpr size_t epi = (size_t)BM * (BN + 4) * 4 / epi_bands<BM, BN, EPB>();
  return stage > epi ? stage : epi;
}

// EPB: epilogue row bands (0 = as few as fit in LDS); S = 1: single-buffered (small-K GEMMs,
// where the LDS footprint, not the pipeline depth, limits the blocks per CU)
template <class E, class = void>
struct has_prefetch : std::false_type {};
template <class E>
struct has_prefetch<E, std::void_t<typename E::Pre>> : std::true_type {};
template <class E, class = void>
struct PreOf {
  struct type {};
};
template <class E>
struct PreOf<E, std::void_t<typename E::Pre>> {
  using type = typename E::Pre;
};

// XCD-aware block order: hardware dispatches block b to XCD b % 8; consecutive logical
// blocks (neighbouring tiles sharing operand rows) land on one XCD and share its L2
RETR_DEVICE int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// Epilogues with kOnesBias = true also want the row sums of A over the tile's K range (the
// bias gradient colsum(dY) of a weight-gradient GEMM): the waves of the first column tile
// (wn == 0, when ep.bias_here(tile column)) run one more MFMA per A fragment against a
// constant all-ones B fragment and hand the sums to ep.bias_apply(row, sum) -- no ones-vector
// GEMM problem, no extra operand traffic.
template <class E, class = void>
struct has_ones_bias : std::false_type {};
template <class E>
struct has_ones_bias<E, std::void_t<decltype(E::kOnesBias)>>
    : std::integral_constant<bool, E::kOnesBias> {};

// Epilogues with kRows = true take whole output ROWS: the fp32 tile goes to LDS once and
// ep.rows(ct, ld, m0, rows, tid, nthreads) runs per row (a LayerNorm over a row the tile holds
// completely: BN = N).
template <class E, class = void>
struct has_rows_epi : std::false_type {};
template <class E>
struct has_rows_epi<E, std::void_t<decltype(E::kRows)>> : std::integral_constant<bool, E::kRows> {};

// One BM x BN output tile (index `tile` in row-major tile order), K range
// [split * kchunk, (split + 1) * kchunk).
template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB, class LA, class LB, class EP>
RETR_DEVICE __attribute__((always_inline)) void gemm2_tile(const LA& la, const LB& lb,
                                                           const EP& ep, int M, int N, int K,
                                                           int kchunk, int tiles_n, int tile,
                                                           int split) {
  using T = bf16;
  constexpr int NT = WM * WN * 64;
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int kStage = (BM + BN) * kBKBytes;
  constexpr bool kBias = has_ones_bias<EP>::value;
  using SA = GStager<BM, NT, LA>;
  using SB = GStager<BN, NT, LB>;
  constexpr int LPT = SA::NCH + SB::NCH;        // DMA instructions per wave per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // the wave id through readfirstlane: the compiler then knows every LDS-DMA destination
  // (wave-uniform base, M0) is uniform and sets M0 from an SGPR instead of one
  // v_readfirstlane per DMA instruction
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  bool bias_wave = false;
  if constexpr (kBias) bias_wave = wn == 0 && ep.bias_here(tile % tiles_n);
  const int kb = split * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke && K > 0) {
    ep.empty_split(m0, n0);
    return;
  }
  const int nk = K > 0 ? (ke - kb + BK - 1) / BK : 0;

  SA sa;
  SB sb;
  sa.init(la, m0, tid, kb);
  sb.init(lb, n0, tid, kb);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[kBias ? TM : 1];
#pragma unroll
  for (int i = 0; i < (kBias ? TM : 1); ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr unsigned kOne2 = 0x3F803F80u;       // two bf16 1.0
  const u32x4 ones{kOne2, kOne2, kOne2, kOne2};

#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    if (s < nk) {
      sa.issue(la, smem + s * kStage, wave);
      sb.issue(lb, smem + s * kStage + BM * kBKBytes, wave);
    }
  }

  for (int t = 0; t < nk; ++t) {
    if constexpr (S == 1) {
      if (t > 0) raw_barrier();          // every wave is done reading the previous tile
      sa.issue(la, smem, wave);
      sb.issue(lb, smem + BM * kBKBytes, wave);
      wait_vmcnt_lgkm0<0>();
    } else if constexpr (S > 2) {
      if (t + S - 2 < nk) wait_vmcnt_lgkm0<LPT * (S - 2)>();
      else wait_vmcnt_lgkm0<0>();
    } else {
      wait_vmcnt_lgkm0<0>();
    }
    raw_barrier();
    if (S > 1 && t + S - 1 < nk) {
      char* st = smem + ((t + S - 1) % S) * kStage;
      sa.issue(la, st, wave);
      sb.issue(lb, st + BM * kBKBytes, wave);
    }
    const char* A = smem + (t % S) * kStage;
    const char* B = A + BM * kBKBytes;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = Stager<T, BM, LA>::frag(A, wm * WTM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = Stager<T, BN, LB>::frag(B, wn * WTN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_step<T>(acc[i][j], af[i], bfr[j]);
      if constexpr (kBias) {
        if (bias_wave) {
#pragma unroll
          for (int i = 0; i < TM; ++i) mfma_step<T>(accb[i], af[i], ones);
        }
      }
    }
  }
  if constexpr (kBias) {
    // D = A * ones: every column of the 16x16 block holds the row sums; lanes 0/16/32/48 own
    // column 0 of rows 4 (lane / 16) + e
    if (bias_wave && (lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wm * WTM + 16 * i + 4 * (lane >> 4) + e;
          if (m < M) ep.bias_apply(m, accb[i][e]);
        }
    }
  }
  (void)ones;
  __syncthreads();
  if constexpr (has_rows_epi<EP>::value) {
    static_assert(epi_bands<BM, BN, EPB>() == 1, "row epilogue: the fp32 tile must fit in LDS");
    float* ct = (float*)smem;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ct[(wm * WTM + 16 * i + 4 * (lane >> 4) + e) * (BN + 4) + wn * WTN + 16 * j +
             (lane & 15)] = acc[i][j][e];
    __syncthreads();
    ep.rows(ct, BN + 4, m0, min(BM, M - m0), tid, NT);
    return;
  }

  // ---- epilogue through LDS (see gemm.hpp), in EP_PASSES row bands when the fp32 tile does
  // not fit in LDS (wave rows wm belong to band wm / (WM / EP_PASSES))
  constexpr int CS = BN + 4;
  constexpr int EP_PASSES = epi_bands<BM, BN, EPB>();
  constexpr int BAND = BM / EP_PASSES;
  constexpr int CH = BN / 8;
  constexpr int IT = BAND * CH / NT;            // 8-column chunks per thread per band
  constexpr bool kPre = has_prefetch<EP>::value && (BAND * CH) % NT == 0 && IT <= 4;
  float* ct = (float*)smem;
#pragma unroll
  for (int pass = 0; pass < EP_PASSES; ++pass) {
    if (pass > 0) __syncthreads();
    if constexpr (kPre) {
      // the band's epilogue operands (residual / addend / gate): all loads in flight while the
      // accumulators go through LDS
      typename PreOf<EP>::type pre[IT];
      const int mb = m0 + pass * BAND;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int q = tid + it * NT;
        const int r = q / CH, c = (q % CH) * 8;
        const int m = mb + r, n = n0 + c;
        if (m < M && n + 8 <= N) ep.fetch8(m, n, pre[it]);
      }
      if (wm / (WM / EP_PASSES) == pass) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              ct[(wm * WTM - pass * BAND + 16 * i + 4 * (lane >> 4) + e) * CS + wn * WTN +
                 16 * j + (lane & 15)] = acc[i][j][e];
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int q = tid + it * NT;
        const int r = q / CH, c = (q % CH) * 8;
        const int m = mb + r, n = n0 + c;
        if (m >= M || n >= N) continue;
        const f32x4 lo = *(const f32x4*)(ct + r * CS + c);
        const f32x4 hi = *(const f32x4*)(ct + r * CS + c + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (n + 8 <= N) {
          ep.apply8p(m, n, v, pre[it]);
        } else {
          for (int e = 0; e < 8 && n + e < N; ++e) ep.apply(m, n + e, v[e]);
        }
      }
      continue;
    }
    if (wm / (WM / EP_PASSES) == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            ct[(wm * WTM - pass * BAND + 16 * i + 4 * (lane >> 4) + e) * CS + wn * WTN + 16 * j +
               (lane & 15)] = acc[i][j][e];
    }
    __syncthreads();
    const int mb = m0 + pass * BAND;
    if (ep.lane_contiguous()) {
      for (int q = tid; q < BAND * BN; q += NT) {
        const int r = q / BN, c = q % BN;
        const int m = mb + r, n = n0 + c;
        if (m < M && n < N) ep.apply(m, n, ct[r * CS + c]);
      }
      continue;
    }
#pragma unroll 2
    for (int q = tid; q < BAND * CH; q += NT) {
      const int r = q / CH, c = (q % CH) * 8;
      const int m = mb + r, n = n0 + c;
      if (m >= M || n >= N) continue;
      const f32x4 lo = *(const f32x4*)(ct + r * CS + c);
      const f32x4 hi = *(const f32x4*)(ct + r * CS + c + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (n + 8 <= N) {
        ep.apply8(m, n, v);
      } else {
        for (int e = 0; e < 8 && n + e < N; ++e) ep.apply(m, n + e, v[e]);
      }
    }
  }
}

template <class E, class = void>
struct has_split_slot : std::false_type {};
template <class E>
struct has_split_slot<E, std::void_t<decltype(std::declval<E&>().split)>> : std::true_type {};

// Split-K grids (weight gradients) are remapped split-major over the whole grid: every tile of
// one K-slice lands on the same XCD, so the slice's operand rows are fetched into that XCD's L2
// once and shared by all its tiles (a tile-only remap spread each slice over all eight L2s).
template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB, class LA, class LB, class EP>
__global__ void __launch_bounds__(WM * WN * 64)
gemm2_kernel(LA la, LB lb, EP ep, int M, int N, int K, int kchunk, int tiles_n) {
  const int tiles = gridDim.x;
  const int r = xcd_remap(blockIdx.y * tiles + blockIdx.x, tiles * gridDim.y);
  const int split = r / tiles, tile = r - split * tiles;
  if constexpr (has_split_slot<EP>::value) ep.split = split;
  gemm2_tile<FAM, BM, BN, WM, WN, S, EPB>(la, lb, ep, M, N, K, kchunk, tiles_n, tile, split);
}

// ---- grouped launch: up to G independent GEMMs with the same operand/epilogue types (the
// projections of one attention block, the weight gradients of one layer, ...) in one grid.
// Problem i owns blocks [blk0, blk0 + tiles * splits) of the (XCD-remapped) block order,
// split-major so the blocks of one K-slice of one problem are neighbours.
template <class LA, class LB, class EP>
struct GProb {
  LA la;
  LB lb;
  EP ep;
  int M, N, K, kchunk, tiles_n, tiles, blk0, nblk;
};

template <class LA, class LB, class EP, int G>
struct GGroup {
  GProb<LA, LB, EP> p[G];
  int n;
};

template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB, class LA, class LB, class EP,
          int G>
__global__ void __launch_bounds__(WM * WN * 64)
gemm2_group_kernel(GGroup<LA, LB, EP, G> g) {
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  int p = 0;
#pragma unroll
  for (int i = 1; i < G; ++i)
    if (i < g.n && bid >= g.p[i].blk0) p = i;
  const GProb<LA, LB, EP>& d = g.p[p];
  const int local = bid - d.blk0;
  if (local >= d.nblk) return;
  const int split = local / d.tiles, tile = local - split * d.tiles;
  if constexpr (has_split_slot<EP>::value) {
    EP ep = d.ep;
    ep.split = split;
    gemm2_tile<FAM, BM, BN, WM, WN, S, EPB>(d.la, d.lb, ep, d.M, d.N, d.K, d.kchunk, d.tiles_n,
                                            tile, split);
  } else {
    gemm2_tile<FAM, BM, BN, WM, WN, S, EPB>(d.la, d.lb, d.ep, d.M, d.N, d.K, d.kchunk,
                                            d.tiles_n, tile, split);
  }
}

// Host side of a grouped launch: fill problems with add(), then launch().
template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB, class LA, class LB, class EP,
          int G>
struct Group2 {
  GGroup<LA, LB, EP, G> g{};
  int blocks = 0;
  int add(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits) {
    if (g.n >= G) return 1;
    constexpr int BK = 64;
    GProb<LA, LB, EP>& d = g.p[g.n];
    d.la = la;
    d.lb = lb;
    d.ep = ep;
    d.M = M;
    d.N = N;
    d.K = K;
    d.tiles_n = cdiv(N, BN);
    d.tiles = cdiv(M, BM) * d.tiles_n;
    if (splits < 1) splits = 1;
    const int ksteps = cdiv(K, BK);
    d.kchunk = BK;
    if (K > 0) {
      if (splits > ksteps) splits = ksteps;
      d.kchunk = cdiv(ksteps, splits) * BK;
      splits = cdiv(K, d.kchunk);
    } else {
      splits = 1;
    }
    d.blk0 = blocks;
    d.nblk = d.tiles * splits;
    blocks += d.nblk;
    ++g.n;
    return 0;
  }
  int launch(hipStream_t st, const char* what) {
    if (blocks == 0) return 0;
    constexpr size_t lds = gemm2_lds_bytes<BM, BN, S, EPB>();
    auto kern = gemm2_group_kernel<FAM, BM, BN, WM, WN, S, EPB, LA, LB, EP, G>;
    if constexpr (lds > 65536) {
      static bool attr_set = false;
      if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr_set = true;
      }
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(WM * WN * 64), lds, st, g);
    return retr_check_launch(what);
  }
};


template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB = 0, class LA, class LB,
          class EP>
int launch_gemm2(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits,
                 hipStream_t st, const char* what) {
  constexpr int BK = 64;
  const int tm = cdiv(M, BM), tn = cdiv(N, BN);
  if (splits < 1) splits = 1;
  const int ksteps = cdiv(K, BK);
  int kchunk = BK;
  if (K > 0) {
    if (splits > ksteps) splits = ksteps;
    kchunk = cdiv(ksteps, splits) * BK;
    splits = cdiv(K, kchunk);
  } else {
    splits = 1;
  }
  dim3 grid(tm * tn, splits);
  constexpr size_t lds = gemm2_lds_bytes<BM, BN, S, EPB>();
  auto kern = gemm2_kernel<FAM, BM, BN, WM, WN, S, EPB, LA, LB, EP>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, grid, dim3(WM * WN * 64), lds, st, la, lb, ep, M, N, K, kchunk, tn);
  return retr_check_launch(what);
}

// Short-reduction GEMMs (K = NKS x 64, no split: the d_model-256 projections of the
// transformer at M 2048 / 6400 and N 256, whose few tiles leave the chip latency-bound).
// gemm_kernel's register-staged loop pays one memory round trip per 64-deep K-step (fetch the
// next step, compute this one, store, barrier); here every K-step of the A / B tiles is fetched
// at once, together with the epilogue operands (residual / addend / gate), then stored to LDS
// behind one barrier: one round trip per tile.  The MFMA chain (K ascending in 32-deep steps,
// 2 x 2 waves of TM x TN 16x16 sub-tiles) and the epilogue are gemm_kernel's, so the output is
// the same bits.
template <int BM, int BN, int NKS, class LA, class LB, class EP>
RETR_DEVICE __attribute__((always_inline)) void short_tile(const LA& la, const LB& lb,
                                                           const EP& ep, int M, int N,
                                                           int tiles_n, int tile) {
  using T = bf16;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int kBuf = (BM + BN) * kBKBytes;
  using SA = Stager<T, BM, LA>;
  using SB = Stager<T, BN, LB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;

  SA sa;
  SB sb;
  sa.init(la, m0, tid, 0);
  sb.init(lb, n0, tid, 0);
  u32x4 ra[NKS][SA::NCH], rb[NKS][SB::NCH];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    sa.fetch(la);
    sb.fetch(lb);
#pragma unroll
    for (int i = 0; i < SA::NCH; ++i) ra[s][i] = sa.reg[i];
#pragma unroll
    for (int i = 0; i < SB::NCH; ++i) rb[s][i] = sb.reg[i];
  }
  constexpr int CH = BN / 8;
  constexpr int IT = BM * CH / 256;             // 8-column epilogue chunks per thread
  static_assert(BM * CH % 256 == 0, "short GEMM epilogue chunks");
  constexpr bool kPre = has_prefetch<EP>::value;
  typename PreOf<EP>::type pre[IT];
  if constexpr (kPre) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int q = tid + it * 256;
      const int m = m0 + q / CH, n = n0 + (q % CH) * 8;
      if (m < M && n + 8 <= N) ep.fetch8(m, n, pre[it]);
    }
  }
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
#pragma unroll
    for (int i = 0; i < SA::NCH; ++i) sa.reg[i] = ra[s][i];
#pragma unroll
    for (int i = 0; i < SB::NCH; ++i) sb.reg[i] = rb[s][i];
    sa.store(smem + s * kBuf, tid);
    sb.store(smem + s * kBuf + BM * kBKBytes, tid);
  }
  __syncthreads();

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const char* A = smem + s * kBuf;
    const char* B = A + BM * kBKBytes;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = SA::frag(A, wm * (BM / 2) + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = SB::frag(B, wn * (BN / 2) + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_step<T>(acc[i][j], af[i], bfr[j]);
    }
  }
  __syncthreads();
  // epilogue through LDS as gemm_kernel's: fp32 [BM][BN + 4], 8 consecutive columns per thread
  constexpr int CS = BN + 4;
  float* ct = (float*)smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ct[(wm * (BM / 2) + 16 * i + 4 * (lane >> 4) + e) * CS + wn * (BN / 2) + 16 * j +
           (lane & 15)] = acc[i][j][e];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int q = tid + it * 256;
    const int r = q / CH, c = (q % CH) * 8;
    const int m = m0 + r, n = n0 + c;
    if (m >= M || n >= N) continue;
    const f32x4 lo = *(const f32x4*)(ct + r * CS + c);
    const f32x4 hi = *(const f32x4*)(ct + r * CS + c + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (n + 8 <= N) {
      if constexpr (kPre) ep.apply8p(m, n, v, pre[it]);
      else ep.apply8(m, n, v);
    } else {
      for (int e = 0; e < 8 && n + e < N; ++e) ep.apply(m, n + e, v[e]);
    }
  }
}

template <int FAM, int BM, int BN, int NKS, class LA, class LB, class EP>
__global__ void __launch_bounds__(256)
gemm_short_kernel(LA la, LB lb, EP ep, int M, int N, int tiles_n) {
  short_tile<BM, BN, NKS>(la, lb, ep, M, N, tiles_n, xcd_remap(blockIdx.x, gridDim.x));
}

template <int BM, int BN, int NKS>
constexpr size_t short_lds_bytes() {
  constexpr size_t stage = (size_t)NKS * (BM + BN) * kBKBytes, epi = (size_t)BM * (BN + 4) * 4;
  return stage > epi ? stage : epi;
}

template <int FAM, int BM, int BN, class LA, class LB, class EP>
int launch_short(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, hipStream_t st,
                 const char* what) {
  constexpr int NKS = 4;
  RETR_REQUIRE(K == NKS * 64, "%s: short-K GEMM needs K = %d (K = %d)", what, NKS * 64, K);
  const int tn = cdiv(N, BN), tiles = cdiv(M, BM) * tn;
  constexpr size_t lds = short_lds_bytes<BM, BN, NKS>();
  static_assert(lds <= 65536, "short GEMM LDS");
  hipLaunchKernelGGL((gemm_short_kernel<FAM, BM, BN, NKS, LA, LB, EP>), dim3(tiles), dim3(256), lds,
                     st, la, lb, ep, M, N, tn);
  return retr_check_launch(what);
}

// Tile choice for the large bf16 GEMMs (convolutions, big linears), from the tools/gemm_tune
// sweep on MI355X (profiles/r2_gemm_tune.txt): the 4-wave 128x128 LDS-DMA tile with a 2-stage
// ring (2 blocks per CU) is the fastest on every conv-shaped GEMM; 128x64 (3 stages) for N=64;
// the 8-wave 256x256 tile only for very wide outputs (the 30522-word head); small grids fall
// back to the register-staged 64x64 kernel of gemm.hpp.  ``splits`` > 1 only for
// weight-gradient GEMMs (split over the pixel / token reduction).
template <int FAM, class LA, class LB, class EP>
int launch_big(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits,
               hipStream_t st, const char* what, bool prefer64 = false) {
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256) * splits;
  const long t128 = (long)cdiv(M, 128) * cdiv(N, 128) * splits;
  const long t12864 = (long)cdiv(M, 128) * cdiv(N, 64) * splits;
  switch (retr_tune_get(RETR_TUNE_BIG_TILE)) {   // sweep override (tools/conv_micro.py)
    case 1: return launch_gemm2<FAM, 128, 128, 2, 2, 1, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 2: return launch_gemm2<FAM, 128, 128, 2, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 3: return launch_gemm2<FAM, 256, 256, 2, 4, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 4: return launch_gemm2<FAM, 128, 64, 2, 2, 3>(la, lb, ep, M, N, K, splits, st, what);
    case 5: return launch_gemm<FAM, bf16, 64, 64>(la, lb, ep, M, N, K, splits, st, what);
    case 6: return launch_gemm2<FAM, 64, 64, 2, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 7: return launch_gemm2<FAM, 128, 128, 2, 2, 1, 1>(la, lb, ep, M, N, K, splits, st, what);
    case 8: return launch_gemm2<FAM, 64, 64, 2, 2, 4>(la, lb, ep, M, N, K, splits, st, what);
    case 9: return launch_gemm2<FAM, 64, 128, 2, 2, 3>(la, lb, ep, M, N, K, splits, st, what);
    case 10: return launch_gemm2<FAM, 32, 64, 1, 4, 4>(la, lb, ep, M, N, K, splits, st, what);
    case 11: return launch_gemm2<FAM, 32, 64, 1, 4, 3>(la, lb, ep, M, N, K, splits, st, what);
    case 12: return launch_gemm2<FAM, 32, 64, 1, 4, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 13: return launch_gemm2<FAM, 64, 64, 2, 2, 1>(la, lb, ep, M, N, K, splits, st, what);
    case 14: return launch_gemm2<FAM, 64, 128, 2, 2, 1>(la, lb, ep, M, N, K, splits, st, what);
    case 15: return launch_gemm2<FAM, 128, 64, 2, 2, 1>(la, lb, ep, M, N, K, splits, st, what);
    // 8 waves of 64x64 (one block per CU): half the LDS fragment bytes per MFMA of the 32x64
    // wave tile, 1.33x fewer loader chunks per MFMA than 2 x 128x128
    case 16: return launch_gemm2<FAM, 256, 128, 4, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 17: return launch_gemm2<FAM, 128, 256, 2, 4, 2>(la, lb, ep, M, N, K, splits, st, what);
    case 18: return launch_gemm2<FAM, 256, 128, 4, 2, 3>(la, lb, ep, M, N, K, splits, st, what);
    default: break;
  }
  // skinny GEMMs over a wide N (the decode step's vocabulary projection, M = 64 caption rows /
  // 320 beam rows, N = 30528): weight streaming is the cost -- 64x64 with a 4-deep ring at
  // M <= 64 (12.4 -> 8.7 us), single-stage 128x128 up to 512 rows (30.3 -> 26.1 us;
  // tools/head_micro.py, profiles/r2_head_tiles.txt)
  if (M <= 64 && N >= 4096)
    return launch_gemm2<FAM, 64, 64, 2, 2, 4>(la, lb, ep, M, N, K, splits, st, what);
  if (M <= 512 && N >= 4096 && K >= 256)
    return launch_gemm2<FAM, 128, 128, 2, 2, 1, 2>(la, lb, ep, M, N, K, splits, st, what);
  // short reductions over wide outputs (1x1 convs with K <= 256 into >= 256 channels and their
  // data gradients, the FFN expansions): HBM / latency-bound, so blocks in flight beat ring
  // depth -- the single-stage 64x64 tile (17 KB of LDS: 8 blocks = 32 waves per CU) over the
  // 2-stage 64x64 / single-stage 128x128 ones (tools/conv_micro.py r50 with RETR_SWEEP_S1,
  // profiles/r3_shortk_s1.txt: 80x80x128->512 + residual 50.9 -> 42.7 us, its data gradient
  // 80x80x512<-128 45.4 -> 36.3 us, 160x160x256<-128 116 -> 103 us; FFN 6400x2048x256
  // 20.5 -> 19.4 us)
  if (K <= 256 && N >= 256 && splits == 1 && retr_tune_get(RETR_TUNE_SHORTK) != 1)
    return launch_gemm2<FAM, 64, 64, 2, 2, 1>(la, lb, ep, M, N, K, splits, st, what);
  // caller's choice of the 64x64 two-stage tile (conv shapes where 4x the blocks win: the
  // 20x20 maps of layer 4 and the 1x1 convolutions to / from 1024 channels at 40x40)
  if (prefer64) return launch_gemm2<FAM, 64, 64, 2, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
  // small K (<= 4 K-steps): single-stage 128x128, 4 blocks per CU (tools/conv_micro.py:
  // 1x1 convs with 256 input channels 46 -> 38 us); N = 64: the 64x64 two-stage tile (the stem
  // 325 -> 280 us, 3x3 64-channel convs 82 -> 64 us)
  if (K <= 256 && splits == 1 && N > 64 && t128 >= 160)
    return launch_gemm2<FAM, 128, 128, 2, 2, 1, 2>(la, lb, ep, M, N, K, splits, st, what);
  if (N >= 4096 && t256 >= 256)
    return launch_gemm2<FAM, 256, 256, 2, 4, 2>(la, lb, ep, M, N, K, splits, st, what);
  // 128x128 over 8 waves (4 x 2, 32x64 per wave), two blocks per CU: 4 waves per SIMD hide the
  // per-K-step load latency better than 4 waves of 64x64 (tools/gemm_tune deep,
  // profiles/r3_gemm_depth.txt: conv-shaped GEMMs 3-8 % faster; deeper rings at 1 block/CU lose)
  if (N > 64 && t128 >= 160)
    return launch_gemm2<FAM, 128, 128, 4, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
  if (N <= 64 && t12864 >= 160)
    return launch_gemm2<FAM, 64, 64, 2, 2, 2>(la, lb, ep, M, N, K, splits, st, what);
  return launch_gemm<FAM, bf16, 64, 64>(la, lb, ep, M, N, K, splits, st, what);
}

}  // namespace retr
