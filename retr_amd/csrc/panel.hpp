// Short-reduction, wide-output bf16 GEMMs with the A panel resident in LDS (linear.hip):
// the FFN expansions h = relu(LN(x) W1^T + b1) (models/transformer_modules.py:6-11: M tokens x
// 2048 x K 256) and their ReLU-gated data gradients dh = [h > 0] (dY W2) (K 256 -> 2048).
//
// With K = 256 a 64x64 output tile is four K-steps: the gemm2 tile spends its life in the
// prologue (both operands' DMA latency) and the epilogue, and fetches its 64-row A panel again
// for every one of the 32 column tiles.  Here a block owns BM rows and a run of NPB column tiles:
// the whole A panel (BM x K) is staged once by LDS-DMA, then the B tiles stream through an
// S-stage ring, one K-step per ring slot, without a drain between column tiles; each finished
// column tile goes through its own LDS staging area to the epilogue while the next tile's B
// stages are already in flight.  Every output is the same v_mfma_f32_16x16x32_bf16 chain over
// K in the same order as the gemm2 64x64 tile (bitwise equal results).
#pragma once
#include "gemm2.hpp"

namespace retr {

template <int FAM, int BM, int BN, int WM, int WN, int S, int MAXK, class LA, class LB, class EP>
__global__ void __launch_bounds__(WM * WN * 64)
panel_kernel(LA la, LB lb, EP ep, int M, int N, int K, int npb, int ngroups) {
  constexpr int NT = WM * WN * 64;
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int NKMAX = MAXK / BK;
  constexpr int ASZ = NKMAX * BM * kBKBytes;         // resident A panel: one image per K-step
  constexpr int BST = BN * kBKBytes;                 // one B ring slot
  constexpr int CS = BN + 4;
  using SA = GStager<BM, NT, LA>;
  using SB = GStager<BN, NT, LB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;
  char* Bs = smem + ASZ;
  float* ct = (float*)(smem + ASZ + S * BST);        // epilogue staging [BM][BN + 4]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int pm = bid / ngroups, ng = bid % ngroups;
  const int m0 = pm * BM;
  const int ntiles = (N + BN - 1) / BN;
  const int t0 = ng * npb;
  const int t1 = min(ntiles, t0 + npb);
  if (t0 >= t1) return;
  const int nk = (K + BK - 1) / BK;                  // <= NKMAX
  const int nsteps = (t1 - t0) * nk;

  // A panel: all nk K-steps, issued first (oldest in the load counter)
  SA sa;
  sa.init(la, m0, tid, 0);
  for (int k = 0; k < nk; ++k) sa.issue(la, As + k * BM * kBKBytes, wave);
  // B ring: step q = (column tile t0 + q / nk, K-step q % nk); the stager walks K and is re-aimed
  // at the next column tile's rows after every nk steps
  SB sb;
  int bt = t0, bk = 0;                               // next step to issue
  sb.init(lb, bt * BN, tid, 0);
  auto issue_b = [&](int q) {
    sb.issue(lb, Bs + (q % S) * BST, wave);
    if (++bk == nk) {
      bk = 0;
      ++bt;
      if (bt < t1) sb.init(lb, bt * BN, tid, 0);
    }
  };
#pragma unroll
  for (int q = 0; q < S - 1; ++q)
    if (q < nsteps) issue_b(q);

  f32x4 acc[TM][TN];
  int q = 0;
  for (int t = t0; t < t1; ++t) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nk; ++k, ++q) {
      // B step q (and, on the first step, the whole A panel) landed: S - 2 younger B steps may
      // stay in flight (each SB::NCH DMA instructions per thread)
      if (q + S - 2 < nsteps) wait_vmcnt_lgkm0<SB::NCH * (S - 2)>();
      else wait_vmcnt_lgkm0<0>();
      raw_barrier();
      if (q + S - 1 < nsteps) issue_b(q + S - 1);
      const char* A = As + k * BM * kBKBytes;
      const char* B = Bs + (q % S) * BST;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = Stager<bf16, BM, LA>::frag(A, wm * WTM + 16 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = Stager<bf16, BN, LB>::frag(B, wn * WTN + 16 * j, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mfma_step<bf16>(acc[i][j], af[i], bfr[j]);
      }
    }
    // column tile t done: through the staging area to the epilogue (the staging area is only
    // shared with the previous tile's epilogue, which every thread finished before the barrier
    // at the top of this tile's last K-step)
    const int n0 = t * BN;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ct[(wm * WTM + 16 * i + 4 * (lane >> 4) + e) * CS + wn * WTN + 16 * j + (lane & 15)] =
              acc[i][j][e];
    // LDS-only barriers: __syncthreads() would also drain the B stages in flight (vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    constexpr int CH = BN / 8;
    for (int r = tid; r < BM * CH; r += NT) {
      const int rr = r / CH, c = (r % CH) * 8;
      const int m = m0 + rr, n = n0 + c;
      if (m >= M || n >= N) continue;
      const f32x4 lo = *(const f32x4*)(ct + rr * CS + c);
      const f32x4 hi = *(const f32x4*)(ct + rr * CS + c + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (n + 8 <= N) {
        ep.apply8(m, n, v);
      } else {
        for (int e = 0; e < 8 && n + e < N; ++e) ep.apply(m, n + e, v[e]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                                   // staging area free for the next tile
  }
}

template <int BM, int BN, int S, int MAXK>
constexpr size_t panel_lds() {
  return (size_t)(MAXK / 64) * BM * kBKBytes + (size_t)S * BN * kBKBytes +
         (size_t)BM * (BN + 4) * 4;
}

// BM 64 x BN 64 column tiles, 4 waves (2 x 2, 32 x 32 each), 3-slot B ring, K <= 256: 32 KB A
// panel + 24 KB ring + 17 KB staging = 73 KB (two blocks per CU).  Column tiles per block so
// the grid is ~512 blocks.
template <int FAM, class LA, class LB, class EP>
int launch_panel(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, hipStream_t st,
                 const char* what) {
  constexpr int BM = 64, BN = 64, S = 3, MAXK = 256;
  const int panels = cdiv(M, BM), ntiles = cdiv(N, BN);
  int groups = cdiv(512, panels);
  const int tg = retr_tune_get(RETR_TUNE_PANEL_GROUPS);
  if (tg > 0) groups = tg;
  if (groups > ntiles) groups = ntiles;
  if (groups < 1) groups = 1;
  const int npb = cdiv(ntiles, groups);
  groups = cdiv(ntiles, npb);
  constexpr size_t lds = panel_lds<BM, BN, S, MAXK>();
  auto kern = panel_kernel<FAM, BM, BN, 2, 2, S, MAXK, LA, LB, EP>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(panels * groups), dim3(256), lds, st, la, lb, ep, M, N, K, npb,
                     groups);
  return retr_check_launch(what);
}

}  // namespace retr
