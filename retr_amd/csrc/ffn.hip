// Fused position-wise feed-forward block at d_model 256 (bf16 operands, fp32 accumulation):
// the two GEMMs of FFResidual's feed_forward (models/transformer_modules.py:6-11,77-97:
// Linear(C, F) -> ReLU -> Linear(F, C)) in ONE launch, the hidden activation chunk going from the
// first GEMM's accumulators straight into the second GEMM's LDS operand image.
//
//   forward   h  = relu(n W1^T + b1)            -> written to H (saved for the backward)
//             y  = h W2^T                        -> fp32 slab of the block's F-split
//   backward  dh = [h > 0] (dbr W2)              (P = W2^T [F][C], gate = h) -> written to H
//             dn = dh W1                         (Q = W1^T [C][F]) -> fp32 slab
// then slab_epilogue (linear.hip) adds the F-splits' slabs in split order and runs the second
// linear's epilogue (+ b2, dropout, + residual | plain bf16 store).
//
// Each block owns 64 token rows (its A panel [64][256] stays in LDS for the whole launch) and
// one F-split; per 64-wide hidden chunk it streams P rows [64][256] and Q columns [256][64] by
// LDS-DMA into a 2-stage ring (one barrier per chunk, the next chunk's DMA in flight across the
// chunk's compute), computes the [64 f][64 m] chunk of h^T (swapped product: a lane holds 4
// consecutive f of one m, written to the [m][f] image with one 8-byte LDS store per tile), and
// accumulates y[64][256] in registers (4 waves x 64 columns).  LDS: A 32 KB + 2 x (32 + 32) KB =
// 160 KB, one block per CU.
//
// Status: correct (bitwise) but slower than the two-launch path at cfg2 (profiles/r4_ffn_fused.txt:
// 47.8 us vs 44.5 us forward at M 6400, 10 % MFMA busy: one 4-wave block per CU exposes every
// barrier / DMA wait), so ops.FUSE_FFN is off by default.
//
// With the F-split of retr_linear_splits (4 at cfg2) the slabs, and so every output bit, equal
// the unfused path's (linear_fwd + linear_fwd_splitk; linear_dgrad + linear_dgrad_splitk): the
// same products accumulated in the same order (tests/test_gpu_kernels.py).
#include "gemm2.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

using namespace retr;

namespace {

constexpr int kBM = 64, kFC = 64, kC = 256, kNT = 256;
constexpr int kKS1 = kC / 64;                 // K-steps of the first GEMM
constexpr int kImg = 64 * kBKBytes;           // one [64 rows][64 k] bf16 image: 8 KB
constexpr int kABytes = kKS1 * kImg;          // A panel: 32 KB
constexpr int kPBytes = kKS1 * kImg;          // P chunk: [64 f][256]: 32 KB
constexpr int kQBytes = kC * kBKBytes;        // Q chunk: [256 c][64 f]: 32 KB
constexpr int kStage = kPBytes + kQBytes;
constexpr int kLds = kABytes + 2 * kStage;    // 163840 B
constexpr int kCS = kC + 4;                   // fp32 staging row stride of the slab store

struct FfnArgs {
  const bf16* A;      // [M][C]   n (forward) / dropout(dy) (backward)
  long lda;
  const bf16* P;      // [F][C]   W1 / W2^T
  long ldp;
  const float* bias;  // [F]      b1 (forward)
  const bf16* gate;   // [M][F]   h (backward)
  long ldg;
  const bf16* Q;      // [C][F]   W2 / W1^T
  long ldq;
  bf16* H;            // [M][F]   h / dh
  long ldh;
  float* ws;          // [S][M][C] fp32 slabs
  int M, F, chunks;   // chunks (of 64 hidden units) per split
  int rblocks;        // row blocks
};

// fragment of an operand image: row-contiguous ([rows][k], DenseK) or k-major ([k][rows],
// DenseT: the backward reads W2 / W1 themselves as W2^T / W1^T, transposed by
// ds_read_b64_tr_b16, no transposed weight copies)
template <int ROWS, class L>
RETR_DEVICE u32x4 frag(const char* img, int r0, int ks, int lane) {
  return Stager<bf16, ROWS, L>::frag(img, r0, ks, lane);
}
RETR_DEVICE u32x4 hfrag(const char* img, int r0, int ks, int lane) {
  return *(const u32x4*)(img + lds_off(r0 + (lane & 15), (lane >> 4) + 4 * ks));
}

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

// MODE 0: forward (P = W1 [F][C], Q = W2 [C][F], both row-major: DenseK);
// MODE 1: backward data (P(f, c) = W2[c][f], Q(c, f) = W1[f][c]: DenseT views of the weights)
template <int MODE, class LP, class LQ>
__global__ void __launch_bounds__(kNT) ffn_chain_kernel(FfnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // split-major logical order, dealt to XCDs in contiguous runs: the row blocks of one split
  // (which stream the same weight columns) share an L2
  const int nblk = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nblk);
  const int split = bid / a.rblocks, rb = bid - split * a.rblocks;
  const int row0 = rb * kBM;
  const int fbase = split * a.chunks * kFC;

  using L = DenseK<bf16>;
  const L la{a.A, a.lda, a.M, kC};
  const LP lp{a.P, a.ldp, a.F, kC};
  const LQ lq{a.Q, a.ldq, kC, a.F};
  // Q chunk staged as four 64-row sub-images (rows [64 q, +64): wave q's columns), so a chunk's
  // DMA splits into four equal pieces (P K-step s + Q sub-image s) issued between the first
  // GEMM's K-steps instead of in one burst ahead of them
  GStager<kBM, kNT, L> sa;
  GStager<kFC, kNT, LP> sp;
  GStager<kFC, kNT, LQ> sq[4];

  char* apanel = smem;
  char* stage0 = smem + kABytes;
  sa.init(la, row0, tid, 0);
#pragma unroll
  for (int s = 0; s < kKS1; ++s) sa.issue(la, apanel + s * kImg, wave);
  auto init_chunk = [&](int j) {
    const int f0 = fbase + j * kFC;
    sp.init(lp, f0, tid, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) sq[q].init(lq, 64 * q, tid, f0);
  };
  auto issue_piece = [&](int s, char* st) {
    sp.issue(lp, st + s * kImg, wave);
    sq[s].issue(lq, st + kPBytes + s * kImg, wave);
  };
  init_chunk(0);
#pragma unroll
  for (int s = 0; s < kKS1; ++s) issue_piece(s, stage0);

  // first GEMM: wave (wf, wm) owns f rows [32 wf, +32) x m columns [32 wm, +32) of h^T
  const int wf = wave >> 1, wm = wave & 1;
  f32x4 acc2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int j = 0; j < a.chunks; ++j) {
    const int f0 = fbase + j * kFC;
    char* st = stage0 + (j & 1) * kStage;
    // the chunk's bias / gate operands: plain loads issued BEFORE the wait that retires the
    // chunk's DMA, consumed through an opaque register barrier right after it, so the
    // compiler's own wait for them lands where no LDS-DMA is in flight (a wait at their use
    // would drain the next chunk's prefetch: cdna_hip_programming.md §5 trap (b))
    f32x4 bia[2];
    u32x2 gat[2][2];
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        bia[i] = *(const f32x4*)(a.bias + f0 + 32 * wf + 16 * i + 4 * (lane >> 4));
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          int m = row0 + 32 * wm + 16 * jj + (lane & 15);
          m = m < a.M ? m : a.M - 1;
          gat[i][jj] = *(const u32x2*)(a.gate + (long)m * a.ldg + f0 + 32 * wf + 16 * i +
                                       4 * (lane >> 4));
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (MODE == 0) {
      asm volatile("" : "+v"(bia[0]), "+v"(bia[1]));
    } else {
      asm volatile("" : "+v"(gat[0][0]), "+v"(gat[0][1]), "+v"(gat[1][0]), "+v"(gat[1][1]));
    }
    raw_barrier();
    const bool more = j + 1 < a.chunks;
    char* nst = stage0 + ((j + 1) & 1) * kStage;
    if (more) init_chunk(j + 1);

    // h^T chunk [64 f][64 m] = P_chunk . A^T
    f32x4 acc1[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc1[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kKS1; ++s) {
      if (more) issue_piece(s, nst);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = frag<kFC, LP>(st + s * kImg, 32 * wf + 16 * i, ks, lane);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          bfr[jj] = hfrag(apanel + s * kImg, 32 * wm + 16 * jj, ks, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) mfma_step<bf16>(acc1[i][jj], af[i], bfr[jj]);
      }
    }
    // every wave is done with the P chunk (its first 8 KB take the h image).  Raw barriers: a
    // __syncthreads() would wait vmcnt(0) and drain the next chunk's LDS-DMA
    raw_barrier();
    char* himg = st;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int m = 32 * wm + 16 * jj + (lane & 15);
        const int f = 32 * wf + 16 * i + 4 * (lane >> 4);
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc1[i][jj][e];
          if constexpr (MODE == 0) {
            v = fmaxf(v + bia[i][e], 0.f);
          } else {
            const unsigned w = gat[i][jj][e >> 1];
            const float g = __builtin_bit_cast(float, (e & 1) ? (w & 0xFFFF0000u) : (w << 16));
            v = g > 0.f ? v : 0.f;
          }
          hv[e] = (bf16)v;
        }
        *(bf16x4*)(himg + lds_off(m, f >> 3) + (f & 7) * 2) = hv;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    // h chunk -> H (16-byte rows pieces, coalesced)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = tid + kNT * u;
      const int r = q >> 3, c = q & 7;
      if (row0 + r < a.M)
        *(u32x4*)(a.H + (long)(row0 + r) * a.ldh + f0 + 8 * c) =
            *(const u32x4*)(himg + lds_off(r, c));
    }
    // y[64 m][256 c] += h_chunk . Q_chunk^T: wave w owns c columns [64 w, +64)
    const char* qimg = st + kPBytes;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = hfrag(himg, 16 * i, ks, lane);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        bfr[jj] = frag<kFC, LQ>(qimg + wave * kImg, 16 * jj, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) mfma_step<bf16>(acc2[i][jj], af[i], bfr[jj]);
    }
  }
  // the split's y slab, staged through LDS for 16-byte row stores
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  float* ct = (float*)(smem + kABytes);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ct[(16 * i + 4 * (lane >> 4) + e) * kCS + 64 * wave + 16 * jj + (lane & 15)] =
            acc2[i][jj][e];
  __syncthreads();
  float* slab = a.ws + (long)split * a.M * kC;
#pragma unroll 4
  for (int q = tid; q < kBM * (kC / 4); q += kNT) {
    const int r = q / (kC / 4), c = (q % (kC / 4)) * 4;
    if (row0 + r < a.M)
      *(f32x4*)(slab + (long)(row0 + r) * kC + c) = *(const f32x4*)(ct + r * kCS + c);
  }
}

template <class EP>
__global__ void ffn_slab_epilogue_kernel(const float* ws, int splits, int M, EP ep) {
  constexpr int N = kC, CH = N / 8;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)M * CH) return;
  const int m = (int)(i / CH), n = (int)(i % CH) * 8;
  const long MN = (long)M * N;
  const float* p = ws + (long)m * N + n;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 3 < splits; s += 4) {
    f32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] = *(const f32x4*)(p + (s + u) * MN);
      y[u] = *(const f32x4*)(p + (s + u) * MN + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += x[u][e], v[e + 4] += y[u][e];
  }
  for (; s < splits; ++s) {
    const f32x4 x = *(const f32x4*)(p + s * MN), y = *(const f32x4*)(p + s * MN + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += x[e], v[e + 4] += y[e];
  }
  ep.apply8(m, n, v);
}

int ffn_launch(int mode, const FfnArgs& args, int splits, hipStream_t st) {
  const int blocks = args.rblocks * splits;
  auto kern = mode == 0 ? ffn_chain_kernel<0, DenseK<bf16>, DenseK<bf16>>
                        : ffn_chain_kernel<1, DenseT<bf16>, DenseT<bf16>>;
  static bool attr[2] = {false, false};
  if (!attr[mode]) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    attr[mode] = true;
  }
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kNT), kLds, st, args);
  return retr_check_launch(mode == 0 ? "ffn_fwd" : "ffn_bwd_data");
}

template <class EP>
int ffn_epilogue(const float* ws, int splits, int M, const EP& ep, hipStream_t st,
                 const char* what) {
  const long chunks = (long)M * (kC / 8);
  hipLaunchKernelGGL((ffn_slab_epilogue_kernel<EP>), dim3((unsigned)cdiv(chunks, 256)),
                     dim3(256), 0, st, ws, splits, M, ep);
  return retr_check_launch(what);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int retr_ffn_splits(int M, int C, int F) {
  // the unfused path's split of the second GEMM (retr_linear_splits of [M][F] x [C][F]^T), so
  // both paths produce the same bits; at least 2 chunks per split
  if (M <= 0 || C != kC || F % kFC != 0) return 0;
  int s = retr_linear_splits(RETR_BF16, M, C, F);
  const int chunks = F / kFC;
  while (s > 1 && (chunks % s != 0 || chunks / s < 2)) --s;
  return s < 1 ? 1 : s;
}

int retr_ffn_fwd(const void* n, long ldn, const void* w1, const float* b1, const void* w2,
                 const float* b2, void* h, long ldh, const float* residual, long ldr, float* y,
                 long ldy, int M, int C, int F, float drop_p, unsigned long long seed, float* ws,
                 int splits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(C == kC && F % kFC == 0 && F > 0, "ffn_fwd: C=%d F=%d (C 256, F %% 64)", C, F);
  RETR_REQUIRE(splits >= 1 && (F / kFC) % splits == 0 && ws != nullptr, "ffn_fwd: splits=%d",
               splits);
  RETR_REQUIRE(ldn % 8 == 0 && ldh % 8 == 0 && aligned16(n) && aligned16(w1) && aligned16(w2) &&
                   aligned16(h) && aligned16(b1) && aligned16(ws) && b1 != nullptr,
               "ffn_fwd: operands must be 16-byte aligned with 8-element row strides");
  FfnArgs a{};
  a.A = (const bf16*)n;
  a.lda = ldn;
  a.P = (const bf16*)w1;
  a.ldp = C;
  a.bias = b1;
  a.Q = (const bf16*)w2;
  a.ldq = F;
  a.H = (bf16*)h;
  a.ldh = ldh;
  a.ws = ws;
  a.M = M;
  a.F = F;
  a.chunks = F / kFC / splits;
  a.rblocks = cdiv(M, kBM);
  if (int e = ffn_launch(0, a, splits, st)) return e;
  EpiFwd<float, float> ep{y, ldy, b2, residual, ldr, 0, make_dp(drop_p, seed), (long)C};
  ep.set_vec();
  return ffn_epilogue(ws, splits, M, ep, st, "ffn_fwd_epilogue");
}

int retr_ffn_bwd_data(const void* dbr, long lddbr, const void* w2, const void* h, long ldh,
                      const void* w1, void* dh, long lddh, void* dn, long lddn, int M, int C,
                      int F, float* ws, int splits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) return 0;
  RETR_REQUIRE(C == kC && F % kFC == 0 && F > 0, "ffn_bwd_data: C=%d F=%d (C 256, F %% 64)", C,
               F);
  RETR_REQUIRE(splits >= 1 && (F / kFC) % splits == 0 && ws != nullptr,
               "ffn_bwd_data: splits=%d", splits);
  RETR_REQUIRE(lddbr % 8 == 0 && ldh % 8 == 0 && lddh % 8 == 0 && aligned16(dbr) &&
                   aligned16(w2) && aligned16(w1) && aligned16(h) && aligned16(dh) &&
                   aligned16(ws),
               "ffn_bwd_data: operands must be 16-byte aligned with 8-element row strides");
  FfnArgs a{};
  a.A = (const bf16*)dbr;
  a.lda = lddbr;
  a.P = (const bf16*)w2;   // (f, c) = W2[c][f]: DenseT, row stride F
  a.ldp = F;
  a.gate = (const bf16*)h;
  a.ldg = ldh;
  a.Q = (const bf16*)w1;   // (c, f) = W1[f][c]: DenseT, row stride C
  a.ldq = C;
  a.H = (bf16*)dh;
  a.ldh = lddh;
  a.ws = ws;
  a.M = M;
  a.F = F;
  a.chunks = F / kFC / splits;
  a.rblocks = cdiv(M, kBM);
  if (int e = ffn_launch(1, a, splits, st)) return e;
  EpiDgrad<bf16, bf16, bf16> ep{(bf16*)dn, lddn, nullptr, 0, nullptr, 0};
  ep.set_vec();
  return ffn_epilogue(ws, splits, M, ep, st, "ffn_bwd_data_epilogue");
}

}  // extern "C"
