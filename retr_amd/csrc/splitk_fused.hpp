// Split-K GEMM with the slice reduction and the GEMM's own epilogue inside the same launch
// (RETR_TUNE_SPLITK_FUSED = 1; linear.hip splitk_run).
//
// The split-K linears (FFN down-projections at d_model 256, the FFN up-projections' data
// gradients: 50-200 output tiles over a 2048-deep reduction) otherwise write every slice's fp32
// partial tile to HBM and run a second launch (slab_epilogue_kernel) that re-reads all of them,
// adds them in slice order and applies bias / residual / dropout (or addend / ReLU gate).  Here
// each (tile, slice) block stores its partial tile with write-through stores, draws the tile's
// ticket (agent-scope atomic), and the block that arrives LAST sums the tile's slices -- in
// slice order, whoever arrives last, so the result is bitwise the two-launch path's -- while
// they are still L2 / Infinity-Cache resident, and applies the epilogue.  With 3-4 slices of a
// 64x64 / 128x128 tile the last arriver's serial read is 48-192 KB (the weight-gradient
// variant of round 4 summed 8-16 slabs of 64 KB and lost on that tail,
// profiles/r4_ab_wgrad_lastarriver.txt).  Tickets are re-armed by their last arriver, so a
// captured launch replays correctly.
#pragma once
#include "gemm2.hpp"

namespace retr {

struct EpiSlabWT {
  float* ws;               // slice 0's partial tile image, row-major [M][N]
  long ld;                 // = N
  long split_stride;       // = M * N
  int split = 0;
  static constexpr bool kRowSum = false;
  RETR_DEVICE __amdgpu_buffer_rsrc_t rsrc() const {
    return __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  }
  RETR_DEVICE unsigned off(int m, int n) const {
    return (unsigned)(((long)split * split_stride + (long)m * ld + n) * 4);
  }
  // write-through (sc1) stores: the partial tile reaches memory without an L2 write-back, so
  // publishing it needs no release fence
  RETR_DEVICE void apply(int m, int n, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc(), off(m, n), 0,
                                          16);
  }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const {
    const auto r = rsrc();
    const unsigned o = off(m, n);
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__builtin_bit_cast(unsigned, v[0]), __builtin_bit_cast(unsigned, v[1]),
              __builtin_bit_cast(unsigned, v[2]), __builtin_bit_cast(unsigned, v[3])},
        r, o, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__builtin_bit_cast(unsigned, v[4]), __builtin_bit_cast(unsigned, v[5]),
              __builtin_bit_cast(unsigned, v[6]), __builtin_bit_cast(unsigned, v[7])},
        r, o + 16, 0, 16);
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return false; }
};

template <int FAM, int BM, int BN, int WM, int WN, int S, class LA, class LB, class EP>
__global__ void __launch_bounds__(WM * WN * 64)
splitk_fused_kernel(LA la, LB lb, EP ep, float* ws, int* tickets, int M, int N, int K, int kchunk,
                    int tiles_n) {
  constexpr int NT = WM * WN * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = gridDim.x, splits = gridDim.y;
  const int r = xcd_remap(blockIdx.y * tiles + blockIdx.x, tiles * splits);
  const int split = r / tiles, tile = r - split * tiles;
  EpiSlabWT sl{ws, (long)N, (long)M * N, split};
  gemm2_tile<FAM, BM, BN, WM, WN, S, 0>(la, lb, sl, M, N, K, kchunk, tiles_n, tile, split);
  // publish this slice (every storing wave drains its write-through stores), draw the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = (int*)smem;
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(tickets + tile, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == splits - 1;
    if (last) {
      __hip_atomic_exchange(tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  // the tile's 8-column chunks: slices added in slice order, then the GEMM's epilogue
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const long MN = (long)M * N;
  constexpr int CH = BN / 8;
  for (int q = threadIdx.x; q < BM * CH; q += NT) {
    const int m = m0 + q / CH, n = n0 + (q % CH) * 8;
    if (m >= M || n >= N) continue;
    const float* p = ws + (long)m * N + n;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) {
      const f32x4 a = *(const f32x4*)(p + s * MN), b = *(const f32x4*)(p + s * MN + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += a[e], v[e + 4] += b[e];
    }
    ep.apply8(m, n, v);
  }
}

int* splitk_tickets(int n);   // linear.hip: n zeroed counters (re-armed by the kernels)

template <int FAM, int BM, int BN, int WM, int WN, int S, class LA, class LB, class EP>
int launch_splitk_fused(const LA& la, const LB& lb, const EP& ep, float* ws, int M, int N, int K,
                        int splits, hipStream_t st, const char* what) {
  constexpr int BK = 64;
  const int tm = cdiv(M, BM), tn = cdiv(N, BN);
  const int ksteps = cdiv(K, BK);
  if (splits > ksteps) splits = ksteps;
  if (splits < 1) splits = 1;
  const int kchunk = cdiv(ksteps, splits) * BK;
  splits = cdiv(K, kchunk);
  int* tk = splitk_tickets(tm * tn);
  RETR_REQUIRE(tk != nullptr, "%s: ticket array unavailable", what);
  constexpr size_t lds = gemm2_lds_bytes<BM, BN, S, 0>();
  auto kern = splitk_fused_kernel<FAM, BM, BN, WM, WN, S, LA, LB, EP>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(tm * tn, splits), dim3(WM * WN * 64), lds, st, la, lb, ep, ws,
                     tk, M, N, K, kchunk, tn);
  return retr_check_launch(what);
}

}  // namespace retr
