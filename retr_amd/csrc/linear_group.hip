// Grouped linear GEMMs: the independent projections of one transformer block in ONE launch.
//
// At d_model 256 a single projection (e.g. M 2048-6400 tokens x N 256 x K 256) is a few
// hundred MFMA tiles of work: alone it cannot fill 256 CUs and its runtime is pipeline fill and
// drain.  The attention block's q|k and v projections (models/transformer_modules.py:38,66 ->
// torch/nn/functional.py:5785-5850), the cross-attention's q, k and v, the data gradients of
// the same, and the weight gradients of every projection of a block are independent GEMMs:
// gemm2.hpp's grouped kernel runs up to kMaxGroup of them in one grid (per-problem operands,
// shapes and epilogues; blocks partitioned by a prefix over the problems).
//
// Weight gradients (dW += dY^T X, db += colsum dY) are split over the token dimension into
// fp32 slabs written with plain stores; the bias gradient is one more GEMM problem against a
// ones vector (dY^T 1); a second launch adds every problem's slabs in slice order into dW / db.
// Deterministic by construction, no float atomics.
#include <cstring>
#include <vector>

#include "gemm2.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

using namespace retr;

namespace {

constexpr int kMaxGroup = 16;
constexpr int kMaxWgrad = 8;   // weight-gradient problems per group (x2 with the bias rows)

static __device__ __attribute__((aligned(16))) unsigned short g_ones_bf16[8] = {
    0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

const bf16* ones_ptr() {
  static const bf16* p = nullptr;
  if (!p) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_ones_bf16)) == hipSuccess) p = (const bf16*)a;
  }
  return p;
}

// the K-slice count the launcher will actually use for `splits` requested slices (whole K-steps)
int norm_splits(int K, int splits) {
  constexpr int BK = 64;
  if (K <= 0) return 1;
  const int ksteps = cdiv(K, BK);
  if (splits < 1) splits = 1;
  if (splits > ksteps) splits = ksteps;
  return cdiv(K, cdiv(ksteps, splits) * BK);
}

// ---- forward / data-gradient groups: tile by the group's total tile count
template <int FAM, int BM, int BN, int WM, int WN, int S, int EPB, class LA, class LB, class EP>
int run_group(int n, const LA* la, const LB* lb, const EP* ep, const int* M, const int* N,
              const int* K, hipStream_t st, const char* what) {
  Group2<FAM, BM, BN, WM, WN, S, EPB, LA, LB, EP, kMaxGroup> g;
  for (int i = 0; i < n; ++i)
    if (M[i] > 0 && g.add(la[i], lb[i], ep[i], M[i], N[i], K[i], 1)) return 1;
  return g.launch(st, what);
}

template <int FAM, class LA, class LB, class EP>
int launch_group(int n, const LA* la, const LB* lb, const EP* ep, const int* M, const int* N,
                 const int* K, hipStream_t st, const char* what) {
  long t128 = 0;
  int kmax = 0;
  for (int i = 0; i < n; ++i) {
    t128 += (long)cdiv(M[i], 128) * cdiv(N[i], 128);
    kmax = K[i] > kmax ? K[i] : kmax;
  }
  int tile = retr_tune_get(RETR_TUNE_GROUP_TILE);
  int stages = retr_tune_get(RETR_TUNE_GROUP_STAGES);
  // tools/group_micro.py (profiles/r2_group_micro.txt): the 64x64 two-stage tile wins on every
  // block-sized group at d_model 256 (more blocks in flight beat the larger tile's reuse)
  if (tile != 64 && tile != 128) tile = t128 >= 400 ? 128 : 64;
  if (tile == 128) {
    if (stages == 0) stages = kmax <= 128 ? 1 : 2;
    if (stages == 1)
      return run_group<FAM, 128, 128, 2, 2, 1, 2>(n, la, lb, ep, M, N, K, st, what);
    if (stages == 3)
      return run_group<FAM, 128, 128, 2, 2, 3, 0>(n, la, lb, ep, M, N, K, st, what);
    return run_group<FAM, 128, 128, 2, 2, 2, 0>(n, la, lb, ep, M, N, K, st, what);
  }
  if (stages == 4) return run_group<FAM, 64, 64, 2, 2, 4, 0>(n, la, lb, ep, M, N, K, st, what);
  if (stages == 1) return run_group<FAM, 64, 64, 2, 2, 1, 0>(n, la, lb, ep, M, N, K, st, what);
  return run_group<FAM, 64, 64, 2, 2, 2, 0>(n, la, lb, ep, M, N, K, st, what);
}

template <typename TO>
int fwd_group_t(int n, const retr_linear_fwd_desc* d, hipStream_t st) {
  DenseK<bf16> la[kMaxGroup], lb[kMaxGroup];
  EpiFwd<TO, float> ep[kMaxGroup];
  int M[kMaxGroup], N[kMaxGroup], K[kMaxGroup];
  for (int i = 0; i < n; ++i) {
    const retr_linear_fwd_desc& q = d[i];
    la[i] = DenseK<bf16>{(const bf16*)q.x, q.ldx, q.M, q.K};
    lb[i] = DenseK<bf16>{(const bf16*)q.w, q.ldw, q.N, q.K};
    ep[i] = EpiFwd<TO, float>{(TO*)q.y, q.ldy, q.bias, q.residual, q.ldr, q.relu,
                              make_dp(q.drop_p, q.seed), (long)q.N};
    ep[i].set_vec();
    M[i] = q.M;
    N[i] = q.N;
    K[i] = q.K;
  }
  return launch_group<kFamLinearFwd>(n, la, lb, ep, M, N, K, st, "linear_fwd_group");
}

template <typename TO, typename TA, class LB>
int dgrad_group_t(int n, const retr_linear_dgrad_desc* d, hipStream_t st) {
  DenseK<bf16> la[kMaxGroup];
  LB lb[kMaxGroup];
  EpiDgrad<TO, TA, bf16> ep[kMaxGroup];
  int M[kMaxGroup], N[kMaxGroup], K[kMaxGroup];
  for (int i = 0; i < n; ++i) {
    const retr_linear_dgrad_desc& q = d[i];
    // dX[m][k] = sum_n dY[m][n] W[n][k]: A = dY (reduction over N), B(k, n) = W[n][k]
    la[i] = DenseK<bf16>{(const bf16*)q.dy, q.lddy, q.M, q.N};
    lb[i] = LB{(const bf16*)q.w, q.ldw, q.K, q.N};
    ep[i] = EpiDgrad<TO, TA, bf16>{(TO*)q.dx, q.lddx, (const TA*)q.addend, q.lda,
                                   (const bf16*)q.gate, q.ldg};
    ep[i].set_vec();
    M[i] = q.M;
    N[i] = q.K;
    K[i] = q.N;
  }
  return launch_group<kFamLinearDgrad>(n, la, lb, ep, M, N, K, st, "linear_dgrad_group");
}

// ---- weight-gradient groups
struct WPlan {
  int tile;                   // 128 or 64
  int stages;                 // LDS ring depth
  int n;                      // GEMM problems (dW problems + bias problems)
  int src[2 * kMaxWgrad];     // descriptor index of each problem
  int bias[2 * kMaxWgrad];    // 1: the problem is the bias-gradient column of src
  int splits[2 * kMaxWgrad];
  long ws_off[2 * kMaxWgrad]; // float offset of the problem's slabs
  long ws_floats;
};

WPlan wgrad_plan(int n, const retr_linear_wgrad_desc* d) {
  WPlan p{};
  long t128 = 0;
  for (int i = 0; i < n; ++i)
    if (d[i].M > 0) t128 += (long)cdiv(d[i].N, 128) * cdiv(d[i].K, 128);
  // 128x128 tiles only for token-heavy groups (the encoder FFN: 64 tiles x 6400 tokens);
  // 64x64 with 512-1024-token slices elsewhere (tools/group_micro.py sweep; a 120k threshold,
  // which moves the decoder FFN to 128x128, did not reproduce in-step: r3_ab_wgrad_tile.txt)
  long tok128 = 0;
  for (int i = 0; i < n; ++i)
    if (d[i].M > 0) tok128 += (long)cdiv(d[i].N, 128) * cdiv(d[i].K, 128) * d[i].M;
  p.tile = tok128 >= 400000 ? 128 : 64;
  (void)t128;
  const int tt = retr_tune_get(RETR_TUNE_WGRAD_TILE);
  if (tt == 64 || tt == 128) p.tile = tt;
  if (tt > 128) p.tile = tok128 >= tt ? 128 : 64;   // A/B: another threshold
  p.stages = retr_tune_get(RETR_TUNE_WGRAD_STAGES);
  if (p.stages == 0) p.stages = 2;
  // one K-slice length (in tokens) for the whole group: about two blocks per CU over the
  // group's tiles, at least 4 K-steps per slice
  long tok_tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (d[i].M <= 0) continue;
    long tiles = (long)cdiv(d[i].N, p.tile) * cdiv(d[i].K, p.tile);
    if (d[i].db) tiles += cdiv(d[i].N, p.tile);
    tok_tiles += tiles * d[i].M;
  }
  const long target = 512;   // blocks
  long kc = (tok_tiles + target - 1) / target;
  kc = (kc + 63) / 64 * 64;
  if (kc < (p.tile == 128 ? 256 : 512)) kc = p.tile == 128 ? 256 : 512;
  if (retr_tune_get(RETR_TUNE_WGRAD_KC) > 0) kc = retr_tune_get(RETR_TUNE_WGRAD_KC);
  for (int i = 0; i < n; ++i) {
    if (d[i].M <= 0) continue;
    const int s = norm_splits(d[i].M, cdiv(d[i].M, (int)kc));
    for (int b = 0; b < (d[i].db ? 2 : 1); ++b) {
      const int j = p.n++;
      p.src[j] = i;
      p.bias[j] = b;
      p.splits[j] = s;
      p.ws_off[j] = p.ws_floats;
      p.ws_floats += (long)s * d[i].N * (b ? 1 : d[i].K);
      p.ws_floats = (p.ws_floats + 3) / 4 * 4;   // 16-byte aligned slabs
    }
  }
  return p;
}

struct SlabSum {
  const float* ws;
  float* dst;
  long ld;        // dst row stride
  long slab;      // floats per slab (rows * cols)
  long sstride;   // floats between consecutive slabs (>= slab)
  int rows, cols, splits, accumulate, blk0, nblk, vec;
  int rowpar;     // many short slabs (LayerNorm partial rows): 64 columns per block, the four
                  // waves take every fourth slab, 8 loads in flight, summed in wave order
};

constexpr int kMaxExtra = 4;   // extra partial-row sums per launch (two LayerNorms' dgamma/dbeta)

struct SlabGroup {
  SlabSum p[2 * kMaxWgrad + kMaxExtra];
  int n;
};

constexpr int kSlabPerThread = 4;

// dst (=|+=) sum_s ws[s] in slice order; 4 consecutive elements per thread
__global__ void __launch_bounds__(256) slab_sum_group_kernel(SlabGroup g) {
  const int bid = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int i = 1; i < 2 * kMaxWgrad + kMaxExtra; ++i)
    if (i < g.n && bid >= g.p[i].blk0) p = i;
  const SlabSum& d = g.p[p];
  if (d.rowpar) {
    __shared__ float red[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = (bid - d.blk0) * 64 + lane;
    float v = 0.f;
    if (c < d.cols) {
      const float* src = d.ws + c;
      int s = w;
      for (; s + 28 < d.splits; s += 32) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = src[(long)(s + 4 * u) * d.sstride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += t[u];
      }
      for (; s < d.splits; s += 4) v += src[(long)s * d.sstride];
    }
    red[w][lane] = v;
    __syncthreads();
    if (w == 0 && c < d.cols) {
      const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
      d.dst[c] = d.accumulate ? d.dst[c] + t : t;
    }
    return;
  }
  const long e0 = ((long)(bid - d.blk0) * 256 + threadIdx.x) * kSlabPerThread;
  if (e0 >= d.slab) return;
  float v[kSlabPerThread] = {0.f, 0.f, 0.f, 0.f};
  if (d.vec) {
    int s = 0;
    for (; s + 3 < d.splits; s += 4) {
      f32x4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = *(const f32x4*)(d.ws + (long)(s + u) * d.sstride + e0);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += t[u][e];
    }
    for (; s < d.splits; ++s) {
      const f32x4 t = *(const f32x4*)(d.ws + (long)s * d.sstride + e0);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += t[e];
    }
    const long r = e0 / d.cols, c = e0 - r * d.cols;
    float* o = d.dst + r * d.ld + c;
    if (d.accumulate) {
      const f32x4 a = *(const f32x4*)o;
      *(f32x4*)o = f32x4{a[0] + v[0], a[1] + v[1], a[2] + v[2], a[3] + v[3]};
    } else {
      *(f32x4*)o = f32x4{v[0], v[1], v[2], v[3]};
    }
    return;
  }
  for (int e = 0; e < kSlabPerThread; ++e) {
    const long i = e0 + e;
    if (i >= d.slab) break;
    float t = 0.f;
    for (int s = 0; s < d.splits; ++s) t += d.ws[(long)s * d.sstride + i];
    const long r = i / d.cols, c = i - r * d.cols;
    float* o = d.dst + r * d.ld + c;
    *o = d.accumulate ? *o + t : t;
  }
}

template <int BM, int S>
int wgrad_group_gemm(const WPlan& p, const retr_linear_wgrad_desc* d, float* ws, hipStream_t st) {
  using L = DenseT<bf16>;
  Group2<kFamLinearWgrad, BM, BM, 2, 2, S, 0, L, L, EpiAccF32, 2 * kMaxWgrad> g;
  const bf16* ones = ones_ptr();
  if (!ones) {
    retr_set_error("linear_wgrad_group: ones vector unavailable");
    return 1;
  }
  for (int j = 0; j < p.n; ++j) {
    const retr_linear_wgrad_desc& q = d[p.src[j]];
    // dW[n][k] = sum_m dY[m][n] X[m][k]: A(n, m) = dY[m][n], B(k, m) = X[m][k]
    L la{(const bf16*)q.dy, q.lddy, q.N, q.M};
    const int cols = p.bias[j] ? 1 : q.K;
    // the bias column: B(0, m) = 1 (a 16-byte ones chunk re-read for every token, ld 0)
    L lb = p.bias[j] ? L{ones, 0, 1, q.M} : L{(const bf16*)q.x, q.ldx, q.K, q.M};
    EpiAccF32 ep{ws + p.ws_off[j], (long)cols, 0, 0, 1, nullptr};
    ep.split_stride = (long)q.N * cols;
    ep.set_vec();
    if (g.add(la, lb, ep, q.N, cols, q.M, p.splits[j])) return 1;
  }
  return g.launch(st, "linear_wgrad_group");
}

// ---- weight gradients with the split-K reduction inside the GEMM launch -----------------------
// (RETR_TUNE_WGRAD_FUSED = 1; measured slower than slabs + slab_sum_group, kept for A/B.)
// Every (tile, K-slice) block writes its fp32 slab with write-through stores (EpiSlab); the block that
// arrives LAST at its tile's ticket (agent-scope release / acquire, cdna_hip_programming.md §5
// "Projection GEMM at M = 256" item 2 and §6 Guideline 16) adds all slices' slabs in SLICE
// order -- whoever arrives last, the sum is the same, and the same as slab_sum_group's -- and
// writes (or accumulates into) dW / db.  The slabs are re-read while L2 / Infinity-Cache
// resident, no second launch.  Blocks past the GEMM blocks sum the extra partial rows
// (LayerNorm dgamma / dbeta from retr_layernorm_bwd2) in the same launch.
struct EpiSlab {
  float* ws;              // slab of slice 0 (row-major [rows][cols])
  long ld;                // = cols
  long split_stride;      // floats between consecutive slices' slabs
  int split = 0;          // set per block
  float* dst;             // dW ([rows][lddw]) or db
  long lddw;
  int rows, cols, splits, accumulate, vec;
  int* tickets;           // one counter per output tile (zero between launches)
  static constexpr bool kRowSum = false;
  // write-through (sc1) stores: the slab reaches memory without an L2 write-back, so the
  // publish needs no release fence (Guideline 16 R1: plain stores + agent release made every
  // block flush its XCD's dirty L2 -- +19 us per launch, measured)
  RETR_DEVICE __amdgpu_buffer_rsrc_t rsrc() const {
    return __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  }
  RETR_DEVICE unsigned off(int m, int n) const {
    return (unsigned)(((long)split * split_stride + (long)m * ld + n) * 4);
  }
  RETR_DEVICE void apply(int m, int n, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc(), off(m, n), 0,
                                          16);
  }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const {
    if (vec) {
      const auto r = rsrc();
      const unsigned o = off(m, n);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__builtin_bit_cast(unsigned, v[0]),
                                                   __builtin_bit_cast(unsigned, v[1]),
                                                   __builtin_bit_cast(unsigned, v[2]),
                                                   __builtin_bit_cast(unsigned, v[3])},
                                             r, o, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__builtin_bit_cast(unsigned, v[4]),
                                                   __builtin_bit_cast(unsigned, v[5]),
                                                   __builtin_bit_cast(unsigned, v[6]),
                                                   __builtin_bit_cast(unsigned, v[7])},
                                             r, o + 16, 0, 16);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) apply(m, n + e, v[e]);
    }
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return false; }
};

constexpr int kTickets = 1 << 18;
static __device__ int g_wgrad_tickets[kTickets];   // zero at load; every last arriver re-zeroes

struct RowParJob {          // dst[c] (=|+=) sum_s parts[s * stride + c], 64 columns per block
  const float* parts;
  float* dst;
  long stride;
  int nparts, cols, accumulate, blk0;
};

struct WgradSide {
  RowParJob job[kMaxExtra];
  int njobs, gemm_blocks;
};

// dst rows [m0, m0 + BM) x cols [n0, n0 + BN) of problem ep: sum of the slabs in slice order
template <int BM, int BN, int NT>
RETR_DEVICE void slab_tile_sum(const EpiSlab& ep, int m0, int n0) {
  const int tid = threadIdx.x;
  const int r1 = min(ep.rows, m0 + BM), c1 = min(ep.cols, n0 + BN);
  if (ep.vec) {
    constexpr int Q = BN / 4;
    for (int q = tid; q < BM * Q; q += NT) {
      const int r = m0 + q / Q, c = n0 + 4 * (q % Q);
      if (r >= r1 || c >= c1) continue;
      const float* src = ep.ws + (long)r * ep.ld + c;
      f32x4 v = *(const f32x4*)src;
      int s = 1;
      for (; s + 3 < ep.splits; s += 4) {
        f32x4 t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = *(const f32x4*)(src + (long)(s + u) * ep.split_stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) v = v + t[u];
      }
      for (; s < ep.splits; ++s) v = v + *(const f32x4*)(src + (long)s * ep.split_stride);
      float* o = ep.dst + (long)r * ep.lddw + c;
      if (ep.accumulate) {
        const f32x4 a = *(const f32x4*)o;
        v = a + v;
      }
      *(f32x4*)o = v;
    }
    return;
  }
  for (int q = tid; q < BM * BN; q += NT) {
    const int r = m0 + q / BN, c = n0 + q % BN;
    if (r >= r1 || c >= c1) continue;
    const float* src = ep.ws + (long)r * ep.ld + c;
    float v = src[0];
    for (int s = 1; s < ep.splits; ++s) v += src[(long)s * ep.split_stride];
    float* o = ep.dst + (long)r * ep.lddw + c;
    *o = ep.accumulate ? *o + v : v;
  }
}

template <int BM, int S>
__global__ void __launch_bounds__(256)
wgrad_fused_kernel(GGroup<DenseT<bf16>, DenseT<bf16>, EpiSlab, 2 * kMaxWgrad> g, WgradSide side) {
  constexpr int NT = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  if (bid >= side.gemm_blocks) {
    // partial-row sums: four waves take every fourth partial row, 8 loads in flight, summed in
    // wave order (slab_sum_group's rowpar arithmetic)
    int j = 0;
#pragma unroll
    for (int i = 1; i < kMaxExtra; ++i)
      if (i < side.njobs && bid - side.gemm_blocks >= side.job[i].blk0) j = i;
    const RowParJob& d = side.job[j];
    float* red = (float*)smem;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = (bid - side.gemm_blocks - d.blk0) * 64 + lane;
    float v = 0.f;
    if (c < d.cols) {
      const float* src = d.parts + c;
      int s = w;
      for (; s + 28 < d.nparts; s += 32) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = src[(long)(s + 4 * u) * d.stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += t[u];
      }
      for (; s < d.nparts; s += 4) v += src[(long)s * d.stride];
    }
    red[w * 64 + lane] = v;
    __syncthreads();
    if (w == 0 && c < d.cols) {
      const float t = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
      d.dst[c] = d.accumulate ? d.dst[c] + t : t;
    }
    return;
  }
  int p = 0;
#pragma unroll
  for (int i = 1; i < 2 * kMaxWgrad; ++i)
    if (i < g.n && bid >= g.p[i].blk0) p = i;
  const auto& d = g.p[p];
  const int local = bid - d.blk0;
  if (local >= d.nblk) return;
  const int split = local / d.tiles, tile = local - split * d.tiles;
  EpiSlab ep = d.ep;
  ep.split = split;
  gemm2_tile<kFamLinearWgrad, BM, BM, 2, 2, S, 0>(d.la, d.lb, ep, d.M, d.N, d.K, d.kchunk,
                                                  d.tiles_n, tile, split);
  // publish this slice's slab (every storing wave drains its write-through stores, then the
  // barrier), draw the tile's ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = (int*)smem;
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ep.tickets + tile, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == ep.splits - 1;
    if (last) {
      // re-arm the counter for the next launch (a memory-side atomic, like the adds)
      __hip_atomic_exchange(ep.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  const int m0 = (tile / d.tiles_n) * BM, n0 = (tile % d.tiles_n) * BM;
  slab_tile_sum<BM, BM, NT>(ep, m0, n0);
}

int g_ticket_cursor = 0;

int* take_tickets(int n) {
  static int* base = nullptr;
  if (!base) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_wgrad_tickets)) != hipSuccess) return nullptr;
    base = (int*)a;
  }
  if (n > kTickets) return nullptr;
  if (g_ticket_cursor + n > kTickets) g_ticket_cursor = 0;
  int* p = base + g_ticket_cursor;
  g_ticket_cursor += (n + 63) / 64 * 64;
  return p;
}

template <int BM, int S>
int wgrad_fused_launch(const WPlan& p, const retr_linear_wgrad_desc* d, float* ws, int nx,
                       const retr_slab_sum_desc* x, hipStream_t st) {
  using L = DenseT<bf16>;
  Group2<kFamLinearWgrad, BM, BM, 2, 2, S, 0, L, L, EpiSlab, 2 * kMaxWgrad> g;
  const bf16* ones = ones_ptr();
  RETR_REQUIRE(ones != nullptr, "linear_wgrad_group: ones vector unavailable");
  for (int j = 0; j < p.n; ++j) {
    const retr_linear_wgrad_desc& q = d[p.src[j]];
    L la{(const bf16*)q.dy, q.lddy, q.N, q.M};
    const int cols = p.bias[j] ? 1 : q.K;
    L lb = p.bias[j] ? L{ones, 0, 1, q.M} : L{(const bf16*)q.x, q.ldx, q.K, q.M};
    EpiSlab ep{};
    ep.ws = ws + p.ws_off[j];
    ep.ld = cols;
    ep.split_stride = (long)q.N * cols;
    ep.dst = p.bias[j] ? q.db : q.dw;
    ep.lddw = p.bias[j] ? 1 : q.lddw;
    ep.rows = q.N;
    ep.cols = cols;
    ep.splits = p.splits[j];
    ep.accumulate = q.accumulate;
    ep.vec = cols % 8 == 0 && ((uintptr_t)ep.ws & 15) == 0 && ep.lddw % 4 == 0 &&
             ((uintptr_t)ep.dst & 15) == 0 && ep.split_stride % 4 == 0;
    if (g.add(la, lb, ep, q.N, cols, q.M, p.splits[j])) return 1;
    auto& pr = g.g.p[g.g.n - 1];
    pr.ep.tickets = take_tickets(pr.tiles);
    RETR_REQUIRE(pr.ep.tickets != nullptr, "linear_wgrad_group: ticket array unavailable");
  }
  WgradSide side{};
  side.gemm_blocks = g.blocks;
  int extra = 0;
  for (int i = 0; i < nx; ++i) {
    const retr_slab_sum_desc& q = x[i];
    if (!q.dst || q.nparts <= 0 || q.cols <= 0) continue;
    RowParJob& r = side.job[side.njobs++];
    r.parts = q.parts;
    r.dst = q.dst;
    r.stride = q.stride;
    r.nparts = q.nparts;
    r.cols = q.cols;
    r.accumulate = q.accumulate;
    r.blk0 = extra;
    extra += (int)cdiv(q.cols, 64);
  }
  const int blocks = g.blocks + extra;
  if (blocks == 0) return 0;
  constexpr size_t lds = gemm2_lds_bytes<BM, BM, S, 0>();
  auto kern = wgrad_fused_kernel<BM, S>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, st, g.g, side);
  return retr_check_launch("linear_wgrad_fused");
}

// ---- deferred weight-gradient batch (retr_linear_wgrad_batch) -------------------------------
// The weight gradients of many blocks (a whole transformer backward) in ONE launch, one K-slice
// per tile: with ~1000 128x128 tiles there is no reason to split the token reduction, so there
// are no fp32 slabs and no slab-sum launch.  The bias gradients ride along as one extra MFMA
// per A fragment against an all-ones fragment in the first column tile (gemm2.hpp
// has_ones_bias); the LayerNorm dgamma / dbeta partial rows are summed by extra blocks.  The
// problem table lives in device memory (written by table_put_kernel launches in stream order),
// so the problem count is not bounded by the kernel-argument size.  Each output element is one
// fp32 MFMA chain over all tokens in order: the bits do not depend on how problems are batched.
struct EpiWB : EpiAccF32 {
  float* db;
  int bias_on;
  static constexpr bool kOnesBias = true;
  RETR_DEVICE bool bias_here(int tile_col) const { return bias_on && tile_col == 0; }
  RETR_DEVICE void bias_apply(int m, float v) const { db[m] = overwrite ? v : db[m] + v; }
};

struct WBProb {               // dW[N][K] (=|+=) dY[M][N]^T X[M][K], db[N] (=|+=) colsum dY
  const bf16* dy;
  const bf16* x;
  float* dw;
  float* db;                  // or null
  int lddy, ldx, lddw, M, N, K, blk0, flags;   // flags: accumulate | vec << 1 | tiles_n << 2
};
struct WBRow {                // dst[c] (=|+=) sum_s parts[s * stride + c]
  const float* parts;
  float* dst;
  int stride, nparts, cols, accumulate, blk0, pad;
};
// Block order: logical blocks (problems longest-reduction first, then the partial-row sums) go
// to the XCDs in runs of kWBChunk (RETR_TUNE_WB_CHUNK > 0: runs of that many), the XCDs taking
// turns.  (Round 5's problem-affine order -- every tile of a problem on one XCD, from a host-built
// piece table -- was measured 0.05 ms/step slower and has been removed: DESIGN.md §4.)
struct WBHead {
  int nprob, nrow, gemm_blocks, total;
};
static_assert(sizeof(WBProb) == 64 && sizeof(WBRow) == 40 && sizeof(WBHead) == 16, "table");

constexpr int kWBChunk = 4;        // consecutive logical blocks per XCD turn

size_t wb_table_bytes(int n, int nx) {
  return sizeof(WBHead) + (size_t)n * sizeof(WBProb) + (size_t)nx * sizeof(WBRow);
}

template <int BM, int S>
__global__ void __launch_bounds__(256) wgrad_batch_kernel(const char* __restrict__ table,
                                                          int chunk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WBHead& h = *(const WBHead*)table;
  const WBProb* P = (const WBProb*)(table + sizeof(WBHead));
  const WBRow* R = (const WBRow*)(table + sizeof(WBHead) + (size_t)h.nprob * sizeof(WBProb));
  // hardware block b runs on XCD b % 8: logical blocks in `chunk` runs, the XCDs taking turns
  const int hw = blockIdx.x, x = hw & 7, q = hw >> 3;
  const int L = (q / chunk) * (8 * chunk) + x * chunk + q % chunk;
  if (L >= h.total) return;
  int lo = 0, tile = 0, rb = -1;
  if (L >= h.gemm_blocks) {
    rb = L - h.gemm_blocks;
  } else {
    int hi = h.nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (P[mid].blk0 <= L) lo = mid;
      else hi = mid - 1;
    }
    tile = L - P[lo].blk0;
  }
  if (rb >= 0) {
    int j = 0;
    for (int i = 1; i < h.nrow; ++i)
      if (rb >= R[i].blk0) j = i;
    const WBRow d = R[j];
    float* red = (float*)smem;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = (rb - d.blk0) * 64 + lane;
    float v = 0.f;
    if (c < d.cols) {
      const float* src = d.parts + c;
      int s = w;
      for (; s + 28 < d.nparts; s += 32) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = src[(long)(s + 4 * u) * d.stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += t[u];
      }
      for (; s < d.nparts; s += 4) v += src[(long)s * d.stride];
    }
    red[w * 64 + lane] = v;
    __syncthreads();
    if (w == 0 && c < d.cols) {
      const float t = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
      d.dst[c] = d.accumulate ? d.dst[c] + t : t;
    }
    return;
  }
  if (lo >= h.nprob) return;                    // table guard
  const WBProb d = P[lo];
  const int tiles_n = d.flags >> 2;
  if (tile >= tiles_n * ((d.N + BM - 1) / BM)) return;
  using Ld = DenseT<bf16>;
  // dW[n][k] = sum_m dY[m][n] X[m][k]: A(n, m) = dY[m][n], B(k, m) = X[m][k]
  const Ld la{d.dy, d.lddy, d.N, d.M};
  const Ld lb{d.x, d.ldx, d.K, d.M};
  EpiWB ep{};
  ep.out = d.dw;
  ep.ldo = d.lddw;
  ep.atomic = 0;
  ep.vec = (d.flags >> 1) & 1;
  ep.overwrite = !(d.flags & 1);
  ep.rowsum = nullptr;
  ep.split_stride = 0;
  ep.split = 0;
  ep.db = d.db;
  ep.bias_on = d.db != nullptr;
  const int kchunk = (d.M + 63) / 64 * 64;
  gemm2_tile<kFamLinearWgrad, BM, BM, 2, 2, S, 0>(la, lb, ep, d.N, d.K, d.M, kchunk, tiles_n,
                                                  tile, 0);
}

struct PutChunk {
  unsigned w[640];            // 2.5 KiB of the table per launch (kernel-argument payload)
  int off, n;                 // word offset, words
};

__global__ void __launch_bounds__(256) table_put_kernel(PutChunk c, unsigned* dst) {
  for (int i = threadIdx.x; i < c.n; i += 256) dst[c.off + i] = c.w[i];
}

template <int BM, int S>
int wgrad_batch_launch(const char* table, int total, hipStream_t st) {
  constexpr size_t lds = gemm2_lds_bytes<BM, BM, S, 0>();
  auto kern = wgrad_batch_kernel<BM, S>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  // RETR_TUNE_WB_CHUNK > 0: runs of that many blocks per XCD turn (sweeps); else kWBChunk
  const int knob = retr_tune_get(RETR_TUNE_WB_CHUNK);
  const int chunk = knob > 0 ? knob : kWBChunk;
  const int grid = cdiv(total, 8 * chunk) * 8 * chunk;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, table, chunk);
  return retr_check_launch("linear_wgrad_batch");
}

}  // namespace

extern "C" {

int retr_linear_fwd_group(int dtype, int y_f32, int n, const retr_linear_fwd_desc* d,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && n <= kMaxGroup, "linear_fwd_group: n=%d (max %d)", n, kMaxGroup);
  if (dtype != RETR_BF16) {
    for (int i = 0; i < n; ++i) {
      const retr_linear_fwd_desc& q = d[i];
      int e = retr_linear_fwd(dtype, q.x, q.ldx, q.w, q.ldw, q.bias, q.y, q.ldy, y_f32, q.M, q.N,
                              q.K, q.relu, q.residual, q.ldr, q.drop_p, q.seed, stream);
      if (e) return e;
    }
    return 0;
  }
  for (int i = 0; i < n; ++i)
    RETR_REQUIRE(d[i].M >= 0 && d[i].N > 0 && d[i].K > 0 && d[i].K % 8 == 0 &&
                     d[i].ldx % 8 == 0 && d[i].ldw % 8 == 0,
                 "linear_fwd_group[%d]: bad shape M=%d N=%d K=%d", i, d[i].M, d[i].N, d[i].K);
  return y_f32 ? fwd_group_t<float>(n, d, st) : fwd_group_t<bf16>(n, d, st);
}

int retr_linear_dgrad_group(int dtype, int dx_f32, int addend_f32, int w_trans, int n,
                            const retr_linear_dgrad_desc* d, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && n <= kMaxGroup, "linear_dgrad_group: n=%d (max %d)", n, kMaxGroup);
  if (dtype != RETR_BF16) {
    for (int i = 0; i < n; ++i) {
      const retr_linear_dgrad_desc& q = d[i];
      int e = retr_linear_dgrad(dtype, q.dy, q.lddy, q.w, q.ldw, q.dx, q.lddx, dx_f32, q.M, q.N,
                                q.K, q.addend, addend_f32, q.lda, q.gate, q.ldg, w_trans, stream);
      if (e) return e;
    }
    return 0;
  }
  for (int i = 0; i < n; ++i)
    RETR_REQUIRE(d[i].M >= 0 && d[i].N > 0 && d[i].K > 0 && d[i].N % 8 == 0 &&
                     d[i].lddy % 8 == 0 && d[i].ldw % 8 == 0,
                 "linear_dgrad_group[%d]: bad shape M=%d N=%d K=%d", i, d[i].M, d[i].N, d[i].K);
  if (w_trans) {
    if (dx_f32) return addend_f32 ? dgrad_group_t<float, float, DenseK<bf16>>(n, d, st)
                                  : dgrad_group_t<float, bf16, DenseK<bf16>>(n, d, st);
    return addend_f32 ? dgrad_group_t<bf16, float, DenseK<bf16>>(n, d, st)
                      : dgrad_group_t<bf16, bf16, DenseK<bf16>>(n, d, st);
  }
  if (dx_f32) return addend_f32 ? dgrad_group_t<float, float, DenseT<bf16>>(n, d, st)
                                : dgrad_group_t<float, bf16, DenseT<bf16>>(n, d, st);
  return addend_f32 ? dgrad_group_t<bf16, float, DenseT<bf16>>(n, d, st)
                    : dgrad_group_t<bf16, bf16, DenseT<bf16>>(n, d, st);
}

size_t retr_linear_wgrad_group_workspace(int n, const retr_linear_wgrad_desc* d) {
  if (n <= 0 || n > kMaxWgrad) return 0;
  return (size_t)wgrad_plan(n, d).ws_floats * sizeof(float);
}

int retr_linear_wgrad_group(int dtype, int n, const retr_linear_wgrad_desc* d, void* workspace,
                            void* stream) {
  return retr_linear_wgrad_group2(dtype, n, d, workspace, 0, nullptr, stream);
}

int retr_linear_wgrad_group2(int dtype, int n, const retr_linear_wgrad_desc* d, void* workspace,
                             int nx, const retr_slab_sum_desc* x, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && n <= kMaxWgrad, "linear_wgrad_group: n=%d (max %d)", n, kMaxWgrad);
  RETR_REQUIRE(nx >= 0 && nx <= kMaxExtra && (nx == 0 || x), "linear_wgrad_group: nx=%d", nx);
  SlabGroup sg{};
  int blocks = 0;
  auto push = [&](SlabSum& s) {
    s.blk0 = blocks;
    s.nblk = s.rowpar ? (int)cdiv(s.cols, 64) : (int)cdiv(s.slab, 256L * kSlabPerThread);
    blocks += s.nblk;
  };
  if (dtype != RETR_BF16) {
    for (int i = 0; i < n; ++i) {
      const retr_linear_wgrad_desc& q = d[i];
      int e = retr_linear_wgrad(dtype, q.dy, q.lddy, q.x, q.ldx, q.dw, q.lddw, q.M, q.N, q.K,
                                q.db, q.accumulate, stream);
      if (e) return e;
    }
  } else {
    for (int i = 0; i < n; ++i)
      RETR_REQUIRE(d[i].M >= 0 && d[i].N > 0 && d[i].K > 0 && d[i].K % 8 == 0 &&
                       d[i].lddy % 8 == 0 && d[i].ldx % 8 == 0 && d[i].lddy >= (d[i].N + 7) / 8 * 8,
                   "linear_wgrad_group[%d]: bad shape M=%d N=%d K=%d", i, d[i].M, d[i].N, d[i].K);
    const WPlan p = wgrad_plan(n, d);
    if (retr_tune_get(RETR_TUNE_WGRAD_FUSED) == 1) {
      // split-K reduction by each tile's last-arriving block, partial rows as side blocks: one
      // launch, no slab_sum_group -- bitwise equal, but 0.31 ms per step SLOWER in the graphed
      // cfg2 step (profiles/r4_ab_wgrad_lastarriver.txt: the last arriver's serial read of
      // 8-16 slabs is the launch's tail), so not the default
      RETR_REQUIRE(p.n == 0 || workspace != nullptr, "linear_wgrad_group: workspace required");
      float* ws = (float*)workspace;
      if (p.tile == 128) return p.stages == 3 ? wgrad_fused_launch<128, 3>(p, d, ws, nx, x, st)
                                              : wgrad_fused_launch<128, 2>(p, d, ws, nx, x, st);
      return p.stages == 4 ? wgrad_fused_launch<64, 4>(p, d, ws, nx, x, st)
           : p.stages == 1 ? wgrad_fused_launch<64, 1>(p, d, ws, nx, x, st)
                           : wgrad_fused_launch<64, 2>(p, d, ws, nx, x, st);
    }
    if (p.n > 0) {
      RETR_REQUIRE(workspace != nullptr, "linear_wgrad_group: workspace required");
      float* ws = (float*)workspace;
      int e;
      if (p.tile == 128) e = p.stages == 3 ? wgrad_group_gemm<128, 3>(p, d, ws, st)
                                           : wgrad_group_gemm<128, 2>(p, d, ws, st);
      else e = p.stages == 4 ? wgrad_group_gemm<64, 4>(p, d, ws, st)
               : p.stages == 1 ? wgrad_group_gemm<64, 1>(p, d, ws, st)
                               : wgrad_group_gemm<64, 2>(p, d, ws, st);
      if (e) return e;
      for (int j = 0; j < p.n; ++j) {
        const retr_linear_wgrad_desc& q = d[p.src[j]];
        SlabSum& s = sg.p[sg.n++];
        s.ws = ws + p.ws_off[j];
        s.rows = q.N;
        s.cols = p.bias[j] ? 1 : q.K;
        s.dst = p.bias[j] ? q.db : q.dw;
        s.ld = p.bias[j] ? 1 : q.lddw;
        s.slab = (long)s.rows * s.cols;
        s.sstride = s.slab;
        s.splits = p.splits[j];
        s.accumulate = q.accumulate;
        s.vec = (s.cols % 4 == 0 && s.ld % 4 == 0 && ((uintptr_t)s.dst & 15) == 0) ||
                (s.cols == 1 && s.rows % 4 == 0 && ((uintptr_t)s.dst & 15) == 0);
        if (s.cols == 1) {   // a bias vector: one row of N elements
          s.cols = s.rows;
          s.rows = 1;
          s.ld = s.cols;
        }
        push(s);
      }
    }
  }
  for (int i = 0; i < nx; ++i) {
    const retr_slab_sum_desc& q = x[i];
    if (!q.dst || q.nparts <= 0 || q.cols <= 0) continue;
    SlabSum& s = sg.p[sg.n++];
    s.ws = q.parts;
    s.dst = q.dst;
    s.rows = 1;
    s.cols = q.cols;
    s.ld = q.cols;
    s.slab = q.cols;
    s.sstride = q.stride;
    s.splits = q.nparts;
    s.accumulate = q.accumulate;
    s.vec = 0;
    s.rowpar = 1;
    push(s);
  }
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(slab_sum_group_kernel, dim3(blocks), dim3(256), 0, st, sg);
  return retr_check_launch("linear_wgrad_group sum");
}

size_t retr_linear_wgrad_batch_table_bytes(int n, int nx) {
  if (n < 0 || nx < 0) return 0;
  return wb_table_bytes(n, nx);
}

int retr_linear_wgrad_batch(int n, const retr_linear_wgrad_desc* d, int nx,
                            const retr_slab_sum_desc* x, void* table, size_t table_bytes,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && nx >= 0 && (n == 0 || d) && (nx == 0 || x),
               "linear_wgrad_batch: n=%d nx=%d", n, nx);
  RETR_REQUIRE(table != nullptr && table_bytes >= wb_table_bytes(n, nx) &&
                   ((uintptr_t)table & 15) == 0,
               "linear_wgrad_batch: table of %zu bytes at %p (need %zu, 16-byte aligned)",
               table_bytes, table, wb_table_bytes(n, nx));
  for (int i = 0; i < n; ++i)
    RETR_REQUIRE(d[i].M >= 0 && d[i].N > 0 && d[i].K > 0 && d[i].K % 8 == 0 &&
                     d[i].lddy % 8 == 0 && d[i].ldx % 8 == 0 && d[i].lddy >= d[i].N &&
                     d[i].ldx >= d[i].K && d[i].lddw >= d[i].K && d[i].lddy < (1L << 31) &&
                     d[i].ldx < (1L << 31) && d[i].lddw < (1L << 31),
                 "linear_wgrad_batch[%d]: bad shape M=%d N=%d K=%d", i, d[i].M, d[i].N, d[i].K);
  // tile: 128x128 once the batch has enough of them to fill the chip (2 blocks per CU)
  long t128 = 0;
  for (int i = 0; i < n; ++i)
    if (d[i].M > 0) t128 += (long)cdiv(d[i].N, 128) * cdiv(d[i].K, 128);
  int bm = t128 >= 384 ? 128 : 64;
  const int tt = retr_tune_get(RETR_TUNE_WGRAD_TILE);
  if (tt == 64 || tt == 128) bm = tt;
  // longest reductions first (the hardware hands out blocks in order; the short ones fill
  // the tail), stable within equal lengths
  int order[1024];
  RETR_REQUIRE(n <= 1024, "linear_wgrad_batch: n=%d (max 1024)", n);
  int np = 0;
  for (int i = 0; i < n; ++i)
    if (d[i].M > 0) order[np++] = i;
  for (int i = 1; i < np; ++i) {
    const int v = order[i];
    int j = i - 1;
    while (j >= 0 && d[order[j]].M < d[v].M) {
      order[j + 1] = order[j];
      --j;
    }
    order[j + 1] = v;
  }
  std::vector<char> buf(wb_table_bytes(np, nx) + 16, 0);
  WBHead* h = (WBHead*)buf.data();
  WBProb* P = (WBProb*)(buf.data() + sizeof(WBHead));
  int blocks = 0;
  for (int j = 0; j < np; ++j) {
    const retr_linear_wgrad_desc& q = d[order[j]];
    WBProb& p = P[j];
    p.dy = (const bf16*)q.dy;
    p.x = (const bf16*)q.x;
    p.dw = q.dw;
    p.db = q.db;
    p.lddy = (int)q.lddy;
    p.ldx = (int)q.ldx;
    p.lddw = (int)q.lddw;
    p.M = q.M;
    p.N = q.N;
    p.K = q.K;
    p.blk0 = blocks;
    const int tiles_n = cdiv(q.K, bm);
    const int vec = vec8_ok<float>(q.dw, q.lddw) ? 1 : 0;
    p.flags = (q.accumulate ? 1 : 0) | vec << 1 | tiles_n << 2;
    blocks += cdiv(q.N, bm) * tiles_n;
  }
  WBRow* R = (WBRow*)(buf.data() + sizeof(WBHead) + (size_t)np * sizeof(WBProb));
  int nr = 0, rblocks = 0;
  for (int i = 0; i < nx; ++i) {
    const retr_slab_sum_desc& q = x[i];
    if (!q.dst || q.nparts <= 0 || q.cols <= 0) continue;
    RETR_REQUIRE(q.stride < (1L << 31), "linear_wgrad_batch: extra stride %ld", q.stride);
    WBRow& r = R[nr++];
    r.parts = q.parts;
    r.dst = q.dst;
    r.stride = (int)q.stride;
    r.nparts = q.nparts;
    r.cols = q.cols;
    r.accumulate = q.accumulate;
    r.blk0 = rblocks;
    rblocks += cdiv(q.cols, 64);
  }
  h->nprob = np;
  h->nrow = nr;
  h->gemm_blocks = blocks;
  h->total = blocks + rblocks;
  if (h->total == 0) return 0;
  // the table into device memory, in stream order before the GEMM launch
  const size_t used = sizeof(WBHead) + (size_t)np * sizeof(WBProb) + (size_t)nr * sizeof(WBRow);
  const int words = (int)((used + 3) / 4);
  const unsigned* src = (const unsigned*)buf.data();
  for (int off = 0; off < words; off += 640) {
    PutChunk c;
    c.off = off;
    c.n = words - off < 640 ? words - off : 640;
    memcpy(c.w, src + off, (size_t)c.n * 4);
    hipLaunchKernelGGL(table_put_kernel, dim3(1), dim3(256), 0, st, c, (unsigned*)table);
    if (int e = retr_check_launch("linear_wgrad_batch table")) return e;
  }
  const char* tb = (const char*)table;
  return bm == 128 ? wgrad_batch_launch<128, 2>(tb, h->total, st)
                   : wgrad_batch_launch<64, 2>(tb, h->total, st);
}

}  // extern "C"
