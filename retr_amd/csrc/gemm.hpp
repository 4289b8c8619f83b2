// Generic LDS-tiled MFMA GEMM core for gfx950:  C[m][n] = sum_k A(m,k) * B(n,k)
//
//  * 256 threads = 4 waves in a 2x2 arrangement; block tile BM x BN, K-step of 128 bytes
//    (64 bf16 / 32 f32) per LDS row.
//  * bf16 operands use v_mfma_f32_16x16x32_bf16, f32 operands the exact-f32
//    v_mfma_f32_16x16x4_f32 (parity mode).  Accumulation is always fp32.
//  * Operands are produced by "loaders" (implicit GEMM): a loader maps a 16-byte chunk request
//    to global memory.  Two chunk orientations exist:
//      - kContig: the chunk holds EPC consecutive K elements of one row (activations/weights in
//        [row][k] layout, NHWC im2col);
//      - !kContig: the chunk holds EPC consecutive ROWS at one k (operands stored [k][row], e.g.
//        the token/pixel-major tensors of a weight-gradient GEMM).  They are transposed while
//        being written to LDS.
//  * LDS image: [rows][8 chunks of 16 B], chunk position XOR-swizzled with (row>>1)&7 so the
//    ds_read_b128 fragment reads of the 16x16x32 operand map are bank-conflict free.
//  * Register-staged double buffer: tile k+1 is fetched into VGPRs before the MFMAs of tile k
//    and written to the other LDS buffer after them; one barrier per K-step.
//  * Split-K over blockIdx.z; the epilogue decides (store vs atomic) from its own state.
#pragma once
#include "common.hpp"

namespace retr {

constexpr int kBKBytes = 128;

template <typename T> struct Elem {
  static constexpr int EPC = 16 / sizeof(T);       // elements per 16-byte chunk
  static constexpr int BK = kBKBytes / sizeof(T);   // K elements per tile step
};

RETR_DEVICE int lds_off(int r, int c) { return r * kBKBytes + ((c ^ ((r >> 1) & 7)) << 4); }

RETR_DEVICE u32x4 zero16() { return u32x4{0u, 0u, 0u, 0u}; }

// Loaders return the address of a 16-byte operand chunk, or nullptr for a chunk outside the
// operand (padding, ragged edges): register staging reads it as zeros, LDS-DMA staging
// (gemm2.hpp) points the lane at a zero page instead.
RETR_DEVICE u32x4 ld16(const void* p) { return p ? *(const u32x4*)p : zero16(); }

// k-major LDS image [BK][ROWS] (bf16) of an operand whose global chunks run along rows: written
// with 16-byte stores, read as MFMA fragments with ds_read_b64_tr_b16 (gfx950 transposing LDS
// read).  The 8-byte column unit is XOR-swizzled by k so the 8 k-rows touched by one 32-lane
// half of a transposed read land on distinct banks.
template <int ROWS>
RETR_DEVICE int kmaj_off(int k, int r) {  // r multiple of 4
  static_assert(ROWS >= 64, "k-major image needs >= 64 rows (swizzle stays inside the row)");
  constexpr int RB = ROWS * 2;
  int f;
  if constexpr (ROWS >= 128) f = 4 * ((k & 3) | (((k >> 3) & 1) << 2));
  else f = 4 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  return k * RB + (((r >> 2) ^ f) << 3);
}

typedef __attribute__((ext_vector_type(4))) short s16x4;
RETR_DEVICE s16x4 ds_read_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

template <typename T>
RETR_DEVICE void mfma_step(f32x4& acc, const u32x4& a, const u32x4& b);

template <>
RETR_DEVICE void mfma_step<bf16>(f32x4& acc, const u32x4& a, const u32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
RETR_DEVICE void mfma_step<float>(f32x4& acc, const u32x4& a, const u32x4& b) {
  f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
}

// Staging of one operand tile (ROWS x BK) through registers into the swizzled LDS image.
template <typename T, int ROWS, class L>
struct Stager {
  static constexpr int EPC = Elem<T>::EPC;
  static constexpr int BK = Elem<T>::BK;
  static constexpr int NCH = ROWS / 32;  // chunks per thread (ROWS*128B / 16B / 256 threads)
  static constexpr int RCH = ROWS / EPC; // row-chunks per k (row-contig orientation)
  // row-contig bf16 operands use the k-major image + transposing reads
  static constexpr bool kTr = !L::kContig && sizeof(T) == 2;
  // Each thread owns fixed (row, k-offset) slots of the tile; the loader keeps a k cursor per
  // slot that advances by BK per tile (no per-load index divisions in the implicit GEMMs).
  typename L::Ctx ctx[L::kContig ? NCH : 1];
  typename L::KCur kc[L::kContig ? 1 : NCH];
  u32x4 reg[NCH];

  RETR_DEVICE void init(const L& l, int row0, int tid, int kb) {
    if constexpr (L::kContig) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) ctx[i] = l.row_ctx(row0 + (tid >> 3) + 32 * i);
      kc[0] = l.kcur(kb + (tid & 7) * EPC);
    } else {
      ctx[0] = l.row_ctx(row0 + (tid % RCH) * EPC);
#pragma unroll
      for (int i = 0; i < NCH; ++i) kc[i] = l.kcur(kb + tid / RCH + (256 / RCH) * i);
    }
  }
  // loads the tile at the cursors, then advances them to the next tile
  RETR_DEVICE void fetch(const L& l) {
    if constexpr (L::kContig) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) reg[i] = ld16(l.addr(ctx[i], kc[0]));
      l.advance(kc[0], BK);
    } else {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        reg[i] = ld16(l.addr(ctx[0], kc[i]));
        l.advance(kc[i], BK);
      }
    }
  }
  RETR_DEVICE void store(char* lds, int tid) {
    if constexpr (L::kContig) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int r = (tid >> 3) + 32 * i, c = tid & 7;
        *(u32x4*)(lds + lds_off(r, c)) = reg[i];
      }
    } else if constexpr (kTr) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int k = tid / RCH + (256 / RCH) * i;
        *(u32x4*)(lds + kmaj_off<ROWS>(k, (tid % RCH) * EPC)) = reg[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int k = tid / RCH + (256 / RCH) * i;
        int r0 = (tid % RCH) * EPC;
        const T* v = (const T*)&reg[i];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          int r = r0 + e;
          *(T*)(lds + lds_off(r, k / EPC) + (k % EPC) * (int)sizeof(T)) = v[e];
        }
      }
    }
  }
  // row sums of the staged chunks (row-contig orientation: the thread's EPC rows are fixed)
  RETR_DEVICE void add_rowsum(float (&s)[EPC]) const {
    if constexpr (!L::kContig) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const T* v = (const T*)&reg[i];
#pragma unroll
        for (int e = 0; e < EPC; ++e) s[e] += to_f(v[e]);
      }
    }
  }
  // MFMA operand fragment of rows [r0, r0+16) for k sub-step ks (32 bf16 / 16 f32 of K):
  // lane l holds row r0 + (l&15), k chunk (l>>4) + 4 ks.
  RETR_DEVICE static u32x4 frag(const char* lds, int r0, int ks, int lane) {
    if constexpr (kTr) {
      const int k = 32 * ks + 8 * (lane >> 4) + ((lane & 15) >> 2);
      const int r = r0 + 4 * (lane & 3);
      s16x4 lo = ds_read_tr16(lds + kmaj_off<ROWS>(k, r));
      s16x4 hi = ds_read_tr16(lds + kmaj_off<ROWS>(k + 4, r));
      return u32x4{(unsigned)(unsigned short)lo[0] | ((unsigned)(unsigned short)lo[1] << 16),
                   (unsigned)(unsigned short)lo[2] | ((unsigned)(unsigned short)lo[3] << 16),
                   (unsigned)(unsigned short)hi[0] | ((unsigned)(unsigned short)hi[1] << 16),
                   (unsigned)(unsigned short)hi[2] | ((unsigned)(unsigned short)hi[3] << 16)};
    } else {
      return *(const u32x4*)(lds + lds_off(r0 + (lane & 15), (lane >> 4) + 4 * ks));
    }
  }
};

// FAM: call-site family tag (kFam* below); it only makes every family's instantiations
// distinct kernel symbols, so rocprof summaries group by family (gemm_kernel<FAM, ...>).
enum { kFamLinearFwd = 0, kFamLinearDgrad = 1, kFamLinearWgrad = 2, kFamConvFwd = 3,
       kFamConvDgrad = 4, kFamConvWgrad = 5 };

template <int FAM, typename T, int BM, int BN, class LA, class LB, class EP>
__global__ void __launch_bounds__(256)
gemm_kernel(LA la, LB lb, EP ep, int M, int N, int K, int kchunk, int tiles_n) {
  constexpr int BK = Elem<T>::BK;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 subtiles per wave (2x2 waves)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kBuf = (BM + BN) * kBKBytes;  // one stage: A tile then B tile

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: consecutive tile ids that share an A panel land on one XCD.
  const int nblk = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r = nblk % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
  const int kb = blockIdx.y * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke && K > 0) {   // (K == 0: no reduction, the epilogue still runs on zeros)
    ep.empty_split(m0, n0);
    return;
  }

  Stager<T, BM, LA> sa;
  Stager<T, BN, LB> sb;
  sa.init(la, m0, tid, kb);
  sb.init(lb, n0, tid, kb);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused row sums of A (bias gradient) in the blocks of the first column tile
  constexpr int EPCA = Stager<T, BM, LA>::EPC;
  const bool do_rs = EP::kRowSum && !LA::kContig && ep.rowsum != nullptr && (bid % tiles_n) == 0;
  float rs[EPCA];
#pragma unroll
  for (int e = 0; e < EPCA; ++e) rs[e] = 0.f;

  sa.fetch(la);
  sb.fetch(lb);
  if (do_rs) sa.add_rowsum(rs);
  sa.store(smem, tid);
  sb.store(smem + BM * kBKBytes, tid);
  __syncthreads();

  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      sa.fetch(la);
      sb.fetch(lb);
      if (do_rs) sa.add_rowsum(rs);
    }
    const char* A = smem + cur * kBuf;
    const char* B = A + BM * kBKBytes;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = Stager<T, BM, LA>::frag(A, wm * (BM / 2) + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = Stager<T, BN, LB>::frag(B, wn * (BN / 2) + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_step<T>(acc[i][j], af[i], bfr[j]);
    }
    if (more) {
      sa.store(smem + (cur ^ 1) * kBuf, tid);
      sb.store(smem + (cur ^ 1) * kBuf + BM * kBKBytes, tid);
    }
    __syncthreads();
    cur ^= 1;
  }

  if constexpr (EP::kRowSum && !LA::kContig) {
    if (do_rs) {  // block-uniform
      // thread t holds rows [(t % RG) * EPCA, +EPCA); the 256 / RG threads of one row group
      // are added in thread order (no LDS atomics: the bias gradient is reproducible bitwise
      // whenever one block owns a row, i.e. without split-K)
      constexpr int RG = BM / EPCA, NG = 256 / RG;
      float* part = (float*)smem;
#pragma unroll
      for (int e = 0; e < EPCA; ++e) part[tid * EPCA + e] = rs[e];
      __syncthreads();
      for (int i = tid; i < BM; i += 256) {
        float s = 0.f;
        for (int g = 0; g < NG; ++g) s += part[((i / EPCA) + g * RG) * EPCA + i % EPCA];
        if (m0 + i < M) atomicAdd(ep.rowsum + m0 + i, s);
      }
      __syncthreads();
    }
  }

  // ---- epilogue through LDS: the accumulator tile (MFMA C layout: 4 rows x 1 column per lane)
  // is re-laid as fp32 [BM][BN+4] so each thread owns 8 consecutive columns of a row and the
  // epilogue issues 16-byte loads/stores (rows of 16 threads = 256 contiguous bf16 bytes).
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
  if (ep.lane_contiguous()) {
    // float atomics: one wave instruction = 64 consecutive columns of a row (256 contiguous
    // bytes, the full-rate atomic shape; an 8-column-per-lane layout would be ~8x slower)
    for (int q = tid; q < BM * BN; q += 256) {
      const int r = q / BN, c = q % BN;
      const int m = m0 + r, n = n0 + c;
      if (m < M && n < N) ep.apply(m, n, ct[r * CS + c]);
    }
    return;
  }
  constexpr int CH = BN / 8;
#pragma unroll 2
  for (int q = tid; q < BM * CH; q += 256) {
    const int r = q / CH, c = (q % CH) * 8;
    const int m = m0 + r, n = n0 + c;
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

template <typename T, int BM, int BN>
constexpr size_t gemm_lds_bytes() {
  constexpr size_t stage = 2 * (BM + BN) * kBKBytes;
  constexpr size_t epi = (size_t)BM * (BN + 4) * 4;
  return stage > epi ? stage : epi;
}

// Host-side launcher: picks split-K so that the grid has enough blocks to fill 256 CUs.
template <int FAM, typename T, int BM, int BN, class LA, class LB, class EP>
int launch_gemm(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits,
                hipStream_t st, const char* what) {
  constexpr int BK = Elem<T>::BK;
  const int tm = cdiv(M, BM), tn = cdiv(N, BN);
  if (splits < 1) splits = 1;
  const int ksteps = cdiv(K, BK);
  int kchunk = BK;                 // K == 0: one split, the epilogue runs on zeros
  if (K > 0) {
    if (splits > ksteps) splits = ksteps;
    kchunk = cdiv(ksteps, splits) * BK;
    splits = cdiv(K, kchunk);
  } else {
    splits = 1;
  }
  dim3 grid(tm * tn, splits);
  constexpr size_t lds = gemm_lds_bytes<T, BM, BN>();
  if constexpr (lds > 65536) {
    static bool attr_set = false;   // once per instantiation (host attribute, capture-safe)
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)gemm_kernel<FAM, T, BM, BN, LA, LB, EP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL((gemm_kernel<FAM, T, BM, BN, LA, LB, EP>), grid, dim3(256), lds, st, la, lb, ep,
                     M, N, K, kchunk, tn);
  return retr_check_launch(what);
}

// Tile choice for a single-pass (no split-K) GEMM: the biggest tile that still puts about one
// block on every CU.  The transformer's skinny GEMMs (M 2048-6400, N 256) otherwise run on
// 32-100 blocks of 128x128 and leave most of the 256 CUs idle.
template <int FAM, typename T, class LA, class LB, class EP>
int launch_sized(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, hipStream_t st,
                 const char* what) {
  const long b128 = (long)cdiv(M, 128) * cdiv(N, 128);
  const long b64 = (long)cdiv(M, 64) * cdiv(N, 64);
  if (b128 >= 240) return launch_gemm<FAM, T, 128, 128>(la, lb, ep, M, N, K, 1, st, what);
  if (b64 >= 192 || N < 64) return launch_gemm<FAM, T, 64, 64>(la, lb, ep, M, N, K, 1, st, what);
  return launch_gemm<FAM, T, 32, 64>(la, lb, ep, M, N, K, 1, st, what);
}

// Split-K heuristic: aim for >= ~2 waves of blocks over 256 CUs when the reduction is long.
static inline int pick_splits(int M, int N, int K, int BM, int BN, int BK, int max_splits = 64) {
  long tiles = (long)cdiv(M, BM) * cdiv(N, BN);
  int ksteps = cdiv(K, BK);
  if (tiles >= 384 || ksteps < 8) return 1;
  long want = (512 + tiles - 1) / tiles;
  long by_k = ksteps / 4;  // keep >= 4 K-steps per split
  long s = want < by_k ? want : by_k;
  if (s > max_splits) s = max_splits;
  return s < 1 ? 1 : (int)s;
}

// ----------------------------------------------------------------------------------------------
// Common loaders
// ----------------------------------------------------------------------------------------------

// Row-major [rows][ld] operand, K contiguous (activations X[M][K], weights W[N][K]).
// kUniformK (gemm2.hpp GStager): the K cursor is the block's (wave-uniform, SGPRs); the
// thread's chunk offset lives in the row context (row pointer and remaining-K limit).
template <typename T>
struct DenseK {
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  static constexpr int EPC = Elem<T>::EPC;
  const T* p;
  long ld;
  int rows, K;
  struct Ctx { const T* row; int klim; };     // klim = K - chunk offset (0: row out of range)
  struct KCur { int k; };
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    return Ctx{p + (long)r * ld + coff, r < rows ? K - coff : 0};
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE KCur kcur(int k) const { return KCur{k}; }
  RETR_DEVICE void advance(KCur& c, int d) const { c.k += d; }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    return k.k < c.klim ? (const void*)(c.row + k.k) : nullptr;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& k, const void* fb) const {
    return k.k < c.klim ? (const void*)(c.row + k.k) : fb;
  }
};

// Two row-major operands side by side along K: element (r, k) = p1[r*ld1 + k] for k < K1, and
// for k >= K1 the 1x1 stride-s2 conv input of output pixel r = (n, oh, ow) of an OH x OW map:
// p2[((n*H2 + oh*s2)*W2 + ow*s2)*ld2 + k - K1] (s2 = 1: row r of p2).  A bottleneck's conv3 over
// [h2 | x] with its downsample folded in, without writing the concatenation.  K1 % EPC == 0, so
// no 16-byte chunk straddles the seam.
template <typename T>
struct DenseK2 {
  static constexpr bool kContig = true;
  static constexpr int EPC = Elem<T>::EPC;
  const T* p1;
  long ld1;
  const T* p2;
  long ld2;
  int K1, rows, K;
  int OH, OW, H2, W2, s2;
  struct Ctx { const T* r1; const T* r2; bool ok; };
  struct KCur { int k; };
  RETR_DEVICE Ctx row_ctx(int r) const {
    const int rr = r < rows ? r : 0;
    long px = rr;
    if (s2 != 1) {
      const int hw = OH * OW;
      const int n = rr / hw, rem = rr - n * hw;
      const int oh = rem / OW, ow = rem - oh * OW;
      px = ((long)n * H2 + (long)oh * s2) * W2 + (long)ow * s2;
    }
    return Ctx{p1 + (long)rr * ld1, p2 + px * ld2 - K1, r < rows};
  }
  RETR_DEVICE KCur kcur(int k) const { return KCur{k}; }
  RETR_DEVICE void advance(KCur& c, int d) const { c.k += d; }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    if (!c.ok || k.k >= K) return nullptr;
    return (k.k < K1 ? c.r1 : c.r2) + k.k;
  }
};

// Operand stored [k][ld] (rows contiguous): element (r, k) = p[k*ld + r]; chunks along rows.
// Requires rows % EPC == 0 or zero-padding beyond `rows` inside the chunk's row range.
// kUniformK (gemm2.hpp GStager): the thread's k-row offset is baked into each row context
// (pointer and remaining-K limit), the block cursor (k, k*ld) stays wave-uniform.
template <typename T>
struct DenseT {
  static constexpr bool kContig = false;
  static constexpr bool kUniformK = true;
  static constexpr int EPC = Elem<T>::EPC;
  const T* p;
  long ld;
  int rows, K;
  struct Ctx { const T* col; int klim; };
  struct KCur { int k; long off; };
  RETR_DEVICE Ctx row_ctx_c(int r, int koff) const {
    return Ctx{p + r + (long)koff * ld, r < rows ? K - koff : 0};
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE KCur kcur(int k) const { return KCur{k, (long)k * ld}; }
  RETR_DEVICE void advance(KCur& c, int d) const { c.k += d; c.off += (long)d * ld; }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    return k.k < c.klim ? (const void*)(c.col + k.off) : nullptr;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& k, const void* fb) const {
    return k.k < c.klim ? (const void*)(c.col + k.off) : fb;
  }
};

}  // namespace retr
