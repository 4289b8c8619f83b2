// Fused multi-head attention forward for bf16 operands, head dim 32 or 64 (the RE⫶TR shapes:
// d_model 256 / 512 with 8 heads), on v_mfma_f32_32x32x16_bf16.
//
// Replaces the need_weights=False core of F.multi_head_attention_forward
// (torch/nn/functional.py:6576-6606, used at models/ConcatTransformer.py:160,204,210 via
// transformer_modules.py:38,66): S = (q hd^-1/2) k^T + mask, P = softmax(S), O = dropout(P) v.
//
// Structure (one wave = 32 queries; NW waves per block share K/V tiles of 64 keys in LDS):
//  * swapped product S^T = K Q^T: the accumulator has the QUERY on the lane and 16 of the 32
//    keys in registers (the other 16 in lane ^ 32), so the online softmax needs no LDS round
//    trip: the row max is 16 register maxes + one xor-32 shuffle, the row sum stays
//    lane-partial until the end;
//  * P never leaves registers: the S^T accumulator, converted pairwise to bf16, is directly the
//    B operand of O^T = V^T P^T (the C layout of one 32x32x16 MFMA is the k-permuted B layout
//    of the next); V^T fragments come from the row-major V tile with ds_read_b64_tr_b16;
//  * Q (prescaled by hd^-1/2 * log2 e, so the softmax runs on exp2) stays in registers;
//  * K/V tiles: register-staged double buffer, one barrier per 64-key tile;
//  * key-padding mask: one byte per lane per tile -> a wave-uniform 64-bit ballot; fully valid
//    tiles skip masking; causal masking only on tiles that cross the diagonal;
//  * dropout: 16-bit keep decisions from one 32-bit integer hash per key pair
//    (common.hpp attn_keep), regenerated identically by the backward kernels.
// The log-sum-exp (natural log) of every row is saved for the backward pass.
#include <type_traits>

#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

typedef __attribute__((ext_vector_type(2))) float f2v;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;

// four scores -> elements 4 half .. 4 half + 3 of a bf16x8 MFMA fragment held as u32x4: two
// v_cvt_pk_bf16_f32 (a per-element (bf16) conversion compiles to one cvt per score + a v_perm
// per pair)
// x where the keep mask km (all ones / zero, from __builtin_amdgcn_sbfe of a saved keep word) is
// set, +0 elsewhere: one v_and instead of a compare + v_cndmask per score, the same bits as
// `keep ? x : 0.f`
RETR_DEVICE float keep_and(float x, int km) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, x) & km);
}

// bits j of [lo, hi) within a 32-bit word (empty when hi <= lo)
RETR_DEVICE uint32_t range_bits(int lo, int hi) {
  lo = lo < 0 ? 0 : lo;
  hi = hi > 32 ? 32 : hi;
  if (hi <= lo) return 0u;
  const uint32_t up = hi >= 32 ? ~0u : ((1u << hi) - 1u);
  return up & ~((1u << lo) - 1u);
}

RETR_DEVICE void put4(u32x4& w, int half, const float (&v)[4]) {
  const f2v lo = {v[0], v[1]}, hi = {v[2], v[3]};
  w[2 * half] = __builtin_bit_cast(uint32_t, __builtin_convertvector(lo, bf16x2v));
  w[2 * half + 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(hi, bf16x2v));
}

RETR_DEVICE f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

RETR_DEVICE s16x4 tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

RETR_DEVICE bf16x8 join(const s16x4& lo, const s16x4& hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// XCD-aware block order: the hardware deals workgroups round-robin to the 8 XCDs (each with its
// own L2) in linear-id order, so the blocks of one (b, h) -- which all read the same K/V (or
// Q/dO) slice -- landed on different XCDs and each fetched the slice from HBM (the resident
// kernels' prologue, 512 blocks loading at once, took 7-10 us of a 35 us dq pass;
// tools/attn_phase.py).  Physical id p runs logical id (p % 8) * (n / 8) + p / 8 (n % 8 == 0):
// consecutive logical ids -- the blocks of one (b, h) -- share an XCD and its L2.
struct BlockXYZ {
  int x, y, z;
};
RETR_DEVICE BlockXYZ xcd_block() {
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * gridDim.z;
  int p = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if ((n & 7) == 0) p = (p & 7) * (n >> 3) + (p >> 3);
  BlockXYZ r;
  r.x = p % gx;
  const int t = p / gx;
  r.y = t % gy;
  r.z = t / gy;
  return r;
}

// Key-padding / causal masking of one 64-key score tile without per-element branches (the
// short-circuit form compiled to an exec-mask branch per score: ~70 s_and_saveexec per tile).
// Score element e of sub-tile sub holds key key0 + kc + 4 hh, kc = sub*32 + (e&3) + 8*(e>>2)
// (a compile-time constant); the ballot is shifted once to this lane's key phase and tested at
// constant bit positions; the causal test is one compare against lim = qi - key0 - 4 hh.
template <int E>
RETR_DEVICE constexpr int tile_kc(int sub) { return sub * 32 + (E & 3) + 8 * (E >> 2); }

RETR_DEVICE bool key_masked(uint32_t lo, uint32_t hi, int kc, bool diag, int lim) {
  const uint32_t bit = (kc < 32 ? (lo >> kc) : (hi >> (kc - 32))) & 1u;
  return (bit != 0u) | (diag & (kc > lim));
}

// The padding bits and the causal test are first merged into one 32-bit word per sub-tile (bit
// j: key 32 sub + j of the lane's phase is masked), then each score is a constant-position bit
// test + select (3 VALU; was ~6 with the per-score shifts and the causal compare).  The
// bfe / bfi pair (2 VALU) is not reachable from C: the compiler canonicalises it back to this
// form, and inline asm that reads the MFMA result would bypass its hazard tracking.
RETR_DEVICE void mask_tile(f32x16 (&S)[2], unsigned long long pmask, bool diag, int lim, int hh) {
  const unsigned long long pm = pmask >> (4 * hh);
  uint32_t w[2] = {(uint32_t)pm, (uint32_t)(pm >> 32)};
  const uint32_t dm = diag ? ~0u : 0u;
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const int L = lim - 32 * sub;                       // key j masked when j > L
    const uint32_t cm = L < 0 ? ~0u : (L >= 31 ? 0u : (~0u << (L + 1)));
    w[sub] |= cm & dm;
  }
#pragma unroll
  for (int sub = 0; sub < 2; ++sub)
#pragma unroll
    for (int e = 0; e < 16; ++e)
      S[sub][e] = (w[sub] >> ((e & 3) + 8 * (e >> 2))) & 1u ? -INFINITY : S[sub][e];
}

// Dropout keep bits saved by the forward for the backward kernels (retr_attention_fwd_dm /
// retr_attention_bwd_dm): word (bh, w, q) = bits of keys 32 w .. 32 w + 31 of query row q of
// (batch, head) bh, laid out [B*H][ceil(Lk/32)][Lq] so that both the forward's stores (lane =
// query) and the key-on-lane backward's loads (one word per query, 4 queries per 16 bytes) are
// contiguous.  The bits are the hash decisions themselves: the backward reads them instead of
// re-hashing every score (~10 VALU per score in the key-on-lane kernel).
RETR_DEVICE void store_dmask(uint32_t* dmask, uint32_t wbits, int hh, int bh, int Lq, int Lk,
                             int qi, int w) {
  const uint32_t full = wbits | (uint32_t)xor_lane((int)wbits, 32);
  const int nw = (Lk + 31) / 32;
  if (hh == 0 && qi < Lq && w < nw) dmask[((long)bh * nw + w) * Lq + qi] = full;
}

// Keep bits of the two 32-key words of 64-key tile t for this lane's query (zero past the
// last word or query): the DMIN forwards' per-tile loads, one tile ahead.
RETR_DEVICE void load_dw(uint32_t (&dw)[2], const uint32_t* dmask, int bh, int Lq, int Lk, int qi,
                         int t) {
  const int nw = (Lk + 31) / 32, w = 2 * t;
  const bool ok = qi < Lq;
  const uint32_t* p = dmask + ((long)bh * nw + w) * Lq + qi;
  dw[0] = ok && w < nw ? p[0] : 0u;
  dw[1] = ok && w + 1 < nw ? p[Lq] : 0u;
}

// Attention-dropout keep bits of a whole (B*H, Lq, Lk) call, one thread per word of the
// [B*H][ceil(Lk/32)][Lq] layout (store_dmask's): the same (row key, key-pair) hash decisions the
// hashing forward takes, for every key of the word, so the saved mask is bit-identical either
// way.  Pure integer VALU (~4 us for the encoder's 20 M scores); run right before a DMIN forward.
__global__ void __launch_bounds__(256) attn_keep_bits_kernel(uint32_t* dmask, int BH, int Lq,
                                                             int Lk, DropoutParams dp) {
  const int nw = (Lk + 31) / 32;
  const long n = (long)BH * nw * Lq;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int qi = (int)(i % Lq);
  const long rest = i / Lq;
  const int w = (int)(rest % nw), bh = (int)(rest / nw);
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey = attn_row_key(dp_seed(dp), (uint32_t)bh * Lq + qi);
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 32; j += 2) {
    const uint32_t b = attn_pair_bits(rowkey, 32 * w + j);
    bits |= (uint32_t)((b & 0xffffu) >= th16) << j;
    bits |= (uint32_t)((b >> 16) >= th16) << (j + 1);
  }
  dmask[i] = bits;
}

template <int HD>
struct Tile {
  static constexpr int KT = 64;              // keys per LDS stage
  static constexpr int RB = HD * 2 + 16;     // row bytes (16-byte pad against bank conflicts)
  static constexpr int BYTES = KT * RB;      // one K or V tile
  static constexpr int STAGE = 2 * BYTES;    // K tile then V tile
  static constexpr int CPR = HD / 8;         // 16-byte chunks per row
};

// Stage K and V rows [key0, key0+64) of one (b, h) through registers into an LDS stage.
template <int HD, int NT>
struct KVStager {
  static constexpr int NCH = 2 * Tile<HD>::KT * Tile<HD>::CPR / NT;   // chunks per thread
  u32x4 reg[NCH];
  RETR_DEVICE void load(const bf16* kb, long ldk, const bf16* vb, long ldv, int key0, int Lk,
                        int tid) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = tid + c * NT;
      const int which = idx / (Tile<HD>::KT * Tile<HD>::CPR);
      const int rem = idx % (Tile<HD>::KT * Tile<HD>::CPR);
      const int row = rem / Tile<HD>::CPR, ch = rem % Tile<HD>::CPR;
      const int key = key0 + row;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (key < Lk)
        v = which ? *(const u32x4*)(vb + (long)key * ldv + ch * 8)
                  : *(const u32x4*)(kb + (long)key * ldk + ch * 8);
      reg[c] = v;
    }
  }
  RETR_DEVICE void store(char* stage, int tid) const {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = tid + c * NT;
      const int which = idx / (Tile<HD>::KT * Tile<HD>::CPR);
      const int rem = idx % (Tile<HD>::KT * Tile<HD>::CPR);
      const int row = rem / Tile<HD>::CPR, ch = rem % Tile<HD>::CPR;
      *(u32x4*)(stage + which * Tile<HD>::BYTES + row * Tile<HD>::RB + ch * 16) = reg[c];
    }
  }
};

// One 64-key tile of the streaming forward from K / V images of Tile<HD> layout: S^T = K Q^T,
// masking, the online-softmax update of (m, l, O) and O^T += V^T drop(P)^T.
// DROP / MASK compile-time (the kernels branch once per tile, wave-uniformly, on whether the
// tile holds padded or causal-boundary keys): no per-score runtime selects in the common case.
// DMIN: the keep bits of the tile's two 32-key words come in dw (pregenerated by
// attn_keep_bits_kernel, the same hash decisions) instead of being hashed here (~9 VALU per
// score: the pair hash, the 16-bit compare, the bit packing); nothing is stored.
template <int HD, bool DROP, bool MASK, bool DMIN = false>
RETR_DEVICE __attribute__((always_inline)) void fwd2_tile(
    const char* Kl, const char* Vl, const bf16x8 (&qf)[HD / 16], f32x16 (&O)[HD / 32], float& m,
    float& l, int key0, unsigned long long pmask, bool diag, int qi, int lane,
    uint32_t rowkey, uint32_t th16, uint32_t* dmask, int bh, int Lq, int Lk,
    const uint32_t (&dw)[2] = {0u, 0u}) {
  using TL = Tile<HD>;
  constexpr int KS = HD / 16, DT = HD / 32;
  const int r = lane & 31, hh = lane >> 5;
  // S^T (two 32-key sub-tiles): rows = keys, lane = query
  f32x16 S[2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
    for (int e = 0; e < 16; ++e) S[sub][e] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 a = *(const bf16x8*)(Kl + (sub * 32 + r) * TL::RB + (16 * s + 8 * hh) * 2);
      S[sub] = mfma32(a, qf[s], S[sub]);
    }
  }
  if constexpr (MASK) mask_tile(S, pmask, diag, qi - key0 - 4 * hh, hh);
  // online softmax (log2 domain)
  float mt = -INFINITY;
#pragma unroll
  for (int sub = 0; sub < 2; ++sub)
#pragma unroll
    for (int e = 0; e < 16; ++e) mt = fmaxf(mt, S[sub][e]);
  mt = fmaxf(mt, xor_lane(mt, 32));
  const float mn = fmaxf(m, mt);
  const float ms = (mn == -INFINITY) ? 0.f : mn;
  const float alpha = __builtin_amdgcn_exp2f(m - ms);
  m = mn;
  if (__any(alpha != 1.f)) {
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) O[dt][e] *= alpha;
  }
  // P as bf16 pairs (one v_cvt_pk_bf16_f32 per two scores; per-element conversions compiled
  // to one cvt per score plus a v_perm per pair)
  u32x4 pw[4];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    uint32_t wbits = 0;                          // keep bits of keys key0 + 32 sub + j
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int kk = key0 + sub * 32 + 8 * g + 4 * hh;   // 4 consecutive keys
      uint32_t b01 = 0, b23 = 0;
      if constexpr (DROP && !DMIN) {
        b01 = attn_pair_bits(rowkey, kk);
        b23 = attn_pair_bits(rowkey, kk + 2);
      }
      float pv[4];
      // S - max for two scores per v_pk_add_f32 (the same per-element differences)
      const f2v msv = {ms, ms};
      const f2v d01 = f2v{S[sub][4 * g], S[sub][4 * g + 1]} - msv;
      const f2v d23 = f2v{S[sub][4 * g + 2], S[sub][4 * g + 3]} - msv;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        float p = __builtin_amdgcn_exp2f(e4 < 2 ? d01[e4] : d23[e4 - 2]);
        l += p;
        if constexpr (DROP && DMIN) {
          // bit (8 g + 4 hh + e4) of the word as an all-ones / zero mask: v_bfe_i32 + v_and
          // (a shift / compare form compiles to and + cmp + cndmask)
          const int km = __builtin_amdgcn_sbfe((int)dw[sub], 8 * g + 4 * hh + e4, 1);
          p = __builtin_bit_cast(float, __builtin_bit_cast(int, p) & km);
        } else if constexpr (DROP) {
          const bool kp = attn_keep(e4 < 2 ? b01 : b23, kk + e4, th16);
          wbits |= (uint32_t)kp << (8 * g + 4 * hh + e4);
          p = kp ? p : 0.f;
        }
        pv[e4] = p;
      }
      // scores e = 4 g .. 4 g + 3 are elements 4 (g & 1) .. + 3 of pf[2 sub + (g >> 1)]
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const f2v v = {pv[2 * h2], pv[2 * h2 + 1]};
        pw[2 * sub + (g >> 1)][2 * (g & 1) + h2] =
            __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
      }
    }
    if (DROP && !DMIN && dmask) store_dmask(dmask, wbits, hh, bh, Lq, Lk, qi, key0 / 32 + sub);
  }
  bf16x8 pf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) pf[s] = __builtin_bit_cast(bf16x8, pw[s]);
  // O^T += V^T P^T  (A = V^T via transposed LDS reads, B = P in registers)
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
    const int qrow = (lane & 15) >> 2;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const char* lo = Vl + (16 * s + 4 * hh + qrow) * TL::RB + c0 * 2;
      const bf16x8 a = join(tr16(lo), tr16(lo + 8 * TL::RB));
      O[dt] = mfma32(a, pf[s], O[dt]);
    }
  }
}

// Q fragments (B operand of S^T = K Q^T): lane holds Q[qi][16s + 8hh + j], prescaled
template <int HD>
RETR_DEVICE void load_qf(bf16x8 (&qf)[HD / 16], const bf16* q, long ldq, int b, int h, int qi,
                         int Lq, int hh, float qscale) {
  const bf16* qr = q + ((long)b * Lq + (qi < Lq ? qi : Lq - 1)) * ldq + h * HD;
#pragma unroll
  for (int s = 0; s < HD / 16; ++s) {
    bf16x8 x = *(const bf16x8*)(qr + 16 * s + 8 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * qscale);
    qf[s] = x;
  }
}

// Normalised output row and log-sum-exp of one lane's query (the lane pair's l partials added).
template <int HD>
RETR_DEVICE void fwd_finish(const f32x16 (&O)[HD / 32], float m, float l, bf16* o, long ldo,
                            int b, int h, int H, int qi, int Lq, int hh, bool drop, float dscale,
                            float* lse) {
  l += xor_lane(l, 32);
  if (qi < Lq) {
    // fully masked row: 0 * inf = NaN (torch's all -inf softmax); kept probabilities were left
    // unscaled, the dropout scale is applied here once
    const float inv = (drop ? dscale : 1.f) / l;
    bf16* orow = o + ((long)b * Lq + qi) * ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 w;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) w[e4] = (bf16)(O[dt][4 * g + e4] * inv);
        *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hh) = w;
      }
    if (hh == 0 && lse) lse[((long)b * H + h) * Lq + qi] = (m + __log2f(l)) * kLn2;
  }
}

// Key-split streaming forward: NQ query waves (32 queries each) x KSP key parities per block.
// Per iteration the block stages KSP consecutive 64-key tiles; parity p's waves run tile
// KSP * it + p, so every (32-query, parity) wave carries its own online-softmax state over
// 1 / KSP of the keys -- KSP times the waves of the unsplit kernel on grids that are otherwise
// ~1.6 waves per SIMD (encoder 400 x 400) or less (cross 128 x 400).  At the end the parities'
// (m, l, O) go through LDS and parity 0 merges them in parity order (deterministic; the same
// products as the unsplit kernel, summed in another fixed order).
template <int HD, int NQ, int KSP, bool DROP, bool DMIN>
__global__ void __launch_bounds__(NQ * KSP * 64)
attn_fwd2s_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v, long ldv,
                  bf16* o, long ldo, int H, int Lq, int Lk, int kbr, const unsigned char* kpm,
                  int causal, float qscale, DropoutParams dp, float* lse, uint32_t* dmask) {
  using TL = Tile<HD>;
  constexpr int NW = NQ * KSP, NT = NW * 64, DT = HD / 32;
  constexpr int SST = KSP * TL::STAGE;              // one ring slot: KSP (K, V) tile pairs
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5;
  const int qw = wave % NQ, par = wave / NQ;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  const int qblk = bxyz.x * (32 * NQ);
  const int q0 = qblk + qw * 32;
  const int qi = q0 + (lane & 31);
  const bf16* kb = k + (long)b * kbr * ldk + h * HD;
  const bf16* vb = v + (long)b * kbr * ldv + h * HD;

  bf16x8 qf[HD / 16];
  load_qf<HD>(qf, q, ldq, b, h, qi, Lq, hh, qscale);

  int kend = Lk;
  if (causal) kend = min(Lk, qblk + 32 * NQ);
  const int ntiles = (kend + TL::KT - 1) / TL::KT;
  const int nit = (ntiles + KSP - 1) / KSP;
  // a wave's own causal range can end before the block's
  const int wtiles = causal ? min(ntiles, (q0 + 32 + 63) / 64) : ntiles;

  constexpr bool drop = DROP;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey =
      drop && !DMIN ? attn_row_key(dp_seed(dp), ((uint32_t)b * H + h) * Lq + qi) : 0u;

  f32x16 O[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[dt][e] = 0.f;
  float m = -INFINITY, l = 0.f;

  KVStager<HD, NT> stg[KSP];
#pragma unroll
  for (int j = 0; j < KSP; ++j) {
    stg[j].load(kb, ldk, vb, ldv, j * TL::KT, Lk, tid);
    stg[j].store(smem + j * TL::STAGE, tid);
  }
  uint32_t dw[2] = {0u, 0u};
  if constexpr (DMIN) load_dw(dw, dmask, b * H + h, Lq, Lk, qi, par);
  __syncthreads();

  for (int it = 0; it < nit; ++it) {
    const char* slot = smem + (it & 1) * SST;
    if (it + 1 < nit) {
#pragma unroll
      for (int j = 0; j < KSP; ++j) stg[j].load(kb, ldk, vb, ldv, ((it + 1) * KSP + j) * TL::KT, Lk, tid);
    }
    const int t = it * KSP + par;
    uint32_t dwc[2] = {dw[0], dw[1]};
    if constexpr (DMIN)
      if (t + KSP < wtiles) load_dw(dw, dmask, b * H + h, Lq, Lk, qi, t + KSP);
    if (t < wtiles) {
      const int key0 = t * TL::KT;
      bool pad = key0 + lane >= Lk;
      if (kpm && !pad) pad = kpm[(long)b * Lk + key0 + lane] != 0;
      const unsigned long long pmask = __ballot(pad);
      const bool diag = causal && (key0 + TL::KT - 1 > q0);
      const char* Kl = slot + par * TL::STAGE;
      if (pmask || diag)
        fwd2_tile<HD, DROP, true, DMIN>(Kl, Kl + TL::BYTES, qf, O, m, l, key0, pmask, diag, qi,
                                        lane, rowkey, th16, dmask, b * H + h, Lq, Lk, dwc);
      else
        fwd2_tile<HD, DROP, false, DMIN>(Kl, Kl + TL::BYTES, qf, O, m, l, key0, pmask, diag, qi,
                                         lane, rowkey, th16, dmask, b * H + h, Lq, Lk, dwc);
    }
    if (it + 1 < nit) {
#pragma unroll
      for (int j = 0; j < KSP; ++j) stg[j].store(smem + ((it + 1) & 1) * SST + j * TL::STAGE, tid);
    }
    __syncthreads();
  }

  // merge: parities 1.. publish (m, l, O) per lane, parity 0 folds them in parity order
  float* xs = (float*)smem;
  constexpr int REC = 16 * DT + 2;                  // floats per lane record
  if (par > 0) {
    float* rec = xs + (((par - 1) * NQ + qw) * 64 + lane) * REC;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) rec[16 * dt + e] = O[dt][e];
    rec[16 * DT] = m;
    rec[16 * DT + 1] = l;
  }
  __syncthreads();
  if (par > 0) return;
#pragma unroll
  for (int p = 1; p < KSP; ++p) {
    const float* rec = xs + (((p - 1) * NQ + qw) * 64 + lane) * REC;
    const float m1 = rec[16 * DT], l1 = rec[16 * DT + 1];
    const float mn = fmaxf(m, m1);
    const float ms = (mn == -INFINITY) ? 0.f : mn;
    const float a0 = __builtin_amdgcn_exp2f(m - ms), a1 = __builtin_amdgcn_exp2f(m1 - ms);
    l = l * a0 + l1 * a1;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) O[dt][e] = O[dt][e] * a0 + rec[16 * dt + e] * a1;
    m = mn;
  }
  fwd_finish<HD>(O, m, l, o, ldo, b, h, H, qi, Lq, hh, drop, dp.scale, lse);
}

template <int HD, int NW, bool DROP, bool DMIN>
__global__ void __launch_bounds__(NW * 64)
attn_fwd2_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v, long ldv,
                 bf16* o, long ldo, int H, int Lq, int Lk, int kbr, const unsigned char* kpm,
                 int causal, float qscale, DropoutParams dp, float* lse, uint32_t* dmask) {
  using TL = Tile<HD>;
  constexpr int NT = NW * 64, KS = HD / 16, DT = HD / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  const int qblk = bxyz.x * (32 * NW);
  const int q0 = qblk + wave * 32;
  const int qi = q0 + r;                          // this lane's query
  const bf16* kb = k + (long)b * kbr * ldk + h * HD;
  const bf16* vb = v + (long)b * kbr * ldv + h * HD;

  bf16x8 qf[KS];
  load_qf<HD>(qf, q, ldq, b, h, qi, Lq, hh, qscale);

  int kend = Lk;
  if (causal) kend = min(Lk, qblk + 32 * NW);
  const int ntiles = (kend + TL::KT - 1) / TL::KT;

  constexpr bool drop = DROP;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey =
      drop && !DMIN ? attn_row_key(dp_seed(dp), ((uint32_t)b * H + h) * Lq + qi) : 0u;

  f32x16 O[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[dt][e] = 0.f;
  float m = -INFINITY, l = 0.f;

  KVStager<HD, NT> stg;
  stg.load(kb, ldk, vb, ldv, 0, Lk, tid);
  stg.store(smem, tid);
  uint32_t dw[2] = {0u, 0u};
  if constexpr (DMIN) load_dw(dw, dmask, b * H + h, Lq, Lk, qi, 0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * TL::KT;
    const char* Kl = smem + (t & 1) * TL::STAGE;
    const char* Vl = Kl + TL::BYTES;
    if (t + 1 < ntiles) stg.load(kb, ldk, vb, ldv, key0 + TL::KT, Lk, tid);
    uint32_t dwc[2] = {dw[0], dw[1]};
    if constexpr (DMIN)
      if (t + 1 < ntiles) load_dw(dw, dmask, b * H + h, Lq, Lk, qi, t + 1);
    // padding mask of the tile's 64 keys, wave-uniform
    bool pad = key0 + lane >= Lk;
    if (kpm && !pad) pad = kpm[(long)b * Lk + key0 + lane] != 0;
    const unsigned long long pmask = __ballot(pad);
    const bool diag = causal && (key0 + TL::KT - 1 > q0);

    if (pmask || diag)
      fwd2_tile<HD, DROP, true, DMIN>(Kl, Vl, qf, O, m, l, key0, pmask, diag, qi, lane, rowkey,
                                      th16, dmask, b * H + h, Lq, Lk, dwc);
    else
      fwd2_tile<HD, DROP, false, DMIN>(Kl, Vl, qf, O, m, l, key0, pmask, diag, qi, lane, rowkey,
                                       th16, dmask, b * H + h, Lq, Lk, dwc);
    if (t + 1 < ntiles) stg.store(smem + ((t + 1) & 1) * TL::STAGE, tid);
    __syncthreads();
  }

  fwd_finish<HD>(O, m, l, o, ldo, b, h, H, qi, Lq, hh, drop, dp.scale, lse);
}

// RETR_TUNE_ATTN_KEEPPRE = 1: pregenerate the call's keep bits (attn_keep_bits_kernel) when
// dropout is on and the caller saves them (training), and let the forward read them instead of
// hashing.  Opt-in: the hashing moves out of the forward but is not cheaper, and the extra
// launch made the graphed step 0.036 ms slower (profiles/r4_ab_keep_bits.txt).
bool keep_bits_pre(const DropoutParams& dp, uint32_t* dmask, int BH, int Lq, int Lk,
                   hipStream_t st) {
  if (dp.thresh == 0 || !dmask || retr_tune_get(RETR_TUNE_ATTN_KEEPPRE) != 1) return false;
  const long n = (long)BH * ((Lk + 31) / 32) * Lq;
  if (n == 0) return false;
  hipLaunchKernelGGL(attn_keep_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     dmask, BH, Lq, Lk, dp);
  return retr_check_launch("attention_keep_bits") == 0;
}

template <int HD, int NW>
int launch_fwd2(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                void* o, long ldo, int B, int H, int Lq, int Lk, int kbr,
                const unsigned char* kpm, int causal, float p, unsigned long long seed,
                float* lse, uint32_t* dmask, hipStream_t st) {
  const float qscale = kLog2e / sqrtf((float)HD);
  const size_t lds = 2 * Tile<HD>::STAGE;
  dim3 grid((Lq + 32 * NW - 1) / (32 * NW), H, B);
  const DropoutParams dp = make_dp(p, seed);
  const bool dmin = keep_bits_pre(dp, dmask, B * H, Lq, Lk, st);
  auto kern = dp.thresh == 0 ? attn_fwd2_kernel<HD, NW, false, false>
              : dmin         ? attn_fwd2_kernel<HD, NW, true, true>
                             : attn_fwd2_kernel<HD, NW, true, false>;
  hipLaunchKernelGGL(kern, grid, dim3(NW * 64), lds, st, (const bf16*)q, ldq, (const bf16*)k, ldk,
                     (const bf16*)v, ldv, (bf16*)o, ldo, H, Lq, Lk, kbr, kpm, causal, qscale, dp,
                     lse, dmask);
  return retr_check_launch("attention_fwd2");
}

template <int HD, int NQ, int KSP>
int launch_fwd2s(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                 void* o, long ldo, int B, int H, int Lq, int Lk, int kbr,
                 const unsigned char* kpm, int causal, float p, unsigned long long seed,
                 float* lse, uint32_t* dmask, hipStream_t st) {
  const float qscale = kLog2e / sqrtf((float)HD);
  const size_t lds = 2 * KSP * Tile<HD>::STAGE;
  const DropoutParams dp = make_dp(p, seed);
  const bool dmin = keep_bits_pre(dp, dmask, B * H, Lq, Lk, st);
  auto kern = dp.thresh == 0 ? attn_fwd2s_kernel<HD, NQ, KSP, false, false>
              : dmin         ? attn_fwd2s_kernel<HD, NQ, KSP, true, true>
                             : attn_fwd2s_kernel<HD, NQ, KSP, true, false>;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  dim3 grid((Lq + 32 * NQ - 1) / (32 * NQ), H, B);
  hipLaunchKernelGGL(kern, grid, dim3(NQ * KSP * 64), lds, st, (const bf16*)q, ldq,
                     (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, H, Lq, Lk, kbr, kpm,
                     causal, qscale, dp, lse, dmask);
  return retr_check_launch("attention_fwd2s");
}

// =============================================================================================
// Sequence-resident variants (fwd3 / dq3 / dkdv3).  At the RE⫶TR sizes (S = 400 image tokens,
// T = 128 caption tokens, hd 32) a block's whole K/V (or Q/dO) slice is 28-64 KB: it is pulled
// into LDS once with LDS-DMA (global_load_lds_dwordx4, every tile in flight together, one
// vmcnt(0) + barrier), and the tile loop then runs from LDS with no per-tile load latency,
// register staging or barriers.  Rows are unpadded and XOR-swizzled by 16-byte chunk
// (chunk' = chunk ^ (row / rows-per-256-byte-sweep)), applied on the source side of the DMA,
// so both the row-fragment reads and the ds_read_b64_tr_b16 transposed reads are
// bank-conflict-free.  The math per tile is the streaming kernels' (same fragments, same
// order), so results are bit-identical to them.
// =============================================================================================

static __device__ __attribute__((aligned(64))) unsigned int g_attn_zero[64];

template <int HD>
struct RL {
  static constexpr int RB = HD * 2;           // row bytes
  static constexpr int CPR = HD / 8;          // 16-byte chunks per row
  static constexpr int RPW = 256 / RB;        // rows per 256-byte bank sweep
  static constexpr int TILE = 64 * RB;        // one 64-row tile
  RETR_DEVICE static int swz(int r) { return (r / RPW) & (CPR - 1); }
  // byte offset of logical 16-byte chunk lc of row r
  RETR_DEVICE static int off(int r, int lc) { return r * RB + ((lc ^ swz(r)) << 4); }
  // byte offset of element column `col` (8-byte aligned group) of row r
  RETR_DEVICE static int offc(int r, int col) {
    return r * RB + ((((col >> 3) ^ swz(r))) << 4) + (col & 7) * 2;
  }
};

// DMA rows [0, ntiles*64) of a [rows][ld] bf16 slice (rows >= valid read zeros) into the
// swizzled image at `lds`; wave w issues instructions w, w + NW, ...
template <int HD, int NW>
RETR_DEVICE void dma_rows(char* lds, const bf16* base, long ld, int ntiles, int valid, int wave,
                          int lane) {
  using L = RL<HD>;
  const int ninstr = ntiles * 64 * L::CPR / 64;
  for (int i = wave; i < ninstr; i += NW) {
    const int j = i * 64 + lane;
    const int row = j / L::CPR, pc = j % L::CPR;
    const int lc = pc ^ L::swz(row);
    const void* src = row < valid ? (const void*)(base + (long)row * ld + lc * 8)
                                  : (const void*)g_attn_zero;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + i * 1024),
                                     16, 0, 0);
  }
}

RETR_DEVICE void dma_drain_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int HD>
size_t res_lds_fwd(int ntiles) { return (size_t)2 * ntiles * RL<HD>::TILE + 8 * ntiles; }
template <int HD>
size_t res_lds_dkdv(int ntiles) {   // Q, dO tiles; lse, D, row keys; 4 waves' keep-bit columns
  return (size_t)2 * ntiles * RL<HD>::TILE + (12 + 4 * 4) * 64 * ntiles;
}

template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64)
attn_fwd3_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v, long ldv,
                 bf16* o, long ldo, int H, int Lq, int Lk, int kbr, const unsigned char* kpm,
                 int causal, float qscale, DropoutParams dp, float* lse, int ntiles_max,
                 uint32_t* dmask) {
  using L = RL<HD>;
  constexpr int KS = HD / 16, DT = HD / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  const int qblk = bxyz.x * (32 * NW);
  const int q0 = qblk + wave * 32;
  const int qi = q0 + r;
  const bf16* kb = k + (long)b * kbr * ldk + h * HD;
  const bf16* vb = v + (long)b * kbr * ldv + h * HD;

  int kend = Lk;
  if (causal) kend = min(Lk, qblk + 32 * NW);
  const int ntiles = (kend + 63) / 64;
  char* Ks = smem;
  char* Vs = smem + (size_t)ntiles_max * L::TILE;
  unsigned long long* pm = (unsigned long long*)(smem + (size_t)2 * ntiles_max * L::TILE);
  dma_rows<HD, NW>(Ks, kb, ldk, ntiles, kend, wave, lane);
  dma_rows<HD, NW>(Vs, vb, ldv, ntiles, kend, wave, lane);
  for (int t = wave; t < ntiles; t += NW) {
    const int key = t * 64 + lane;
    bool pad = key >= Lk;
    if (kpm && !pad) pad = kpm[(long)b * Lk + key] != 0;
    const unsigned long long bm = __ballot(pad);
    if (lane == 0) pm[t] = bm;
  }

  bf16x8 qf[KS];
  {
    const bf16* qr = q + ((long)b * Lq + (qi < Lq ? qi : Lq - 1)) * ldq + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 x = *(const bf16x8*)(qr + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * qscale);
      qf[s] = x;
    }
  }
  const bool drop = dp.thresh != 0;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey = drop ? attn_row_key(dp_seed(dp), ((uint32_t)b * H + h) * Lq + qi) : 0u;

  f32x16 O[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[dt][e] = 0.f;
  float m = -INFINITY, l = 0.f;
  dma_drain_barrier();

  // a wave's own causal range can end before the block's
  const int wtiles = causal ? min(ntiles, (q0 + 32 + 63) / 64) : ntiles;
  for (int t = 0; t < wtiles; ++t) {
    const int key0 = t * 64;
    const char* Kl = Ks + t * L::TILE;
    const char* Vl = Vs + t * L::TILE;
    const unsigned long long pmask = pm[t];
    const bool diag = causal && (key0 + 63 > q0);
    f32x16 S[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int e = 0; e < 16; ++e) S[sub][e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 a = *(const bf16x8*)(Kl + L::off(sub * 32 + r, 2 * s + hh));
        S[sub] = mfma32(a, qf[s], S[sub]);
      }
    }
    if (pmask || diag) mask_tile(S, pmask, diag, qi - key0 - 4 * hh, hh);
    float mt = -INFINITY;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int e = 0; e < 16; ++e) mt = fmaxf(mt, S[sub][e]);
    mt = fmaxf(mt, xor_lane(mt, 32));
    const float mn = fmaxf(m, mt);
    // a row with no valid key so far keeps m = -inf: exponentiate against 0 instead (every
    // score is -inf then, so every p is 0) -- no per-element select
    const float ms = (mn == -INFINITY) ? 0.f : mn;
    const float alpha = __builtin_amdgcn_exp2f(m - ms);
    m = mn;
    if (__any(alpha != 1.f)) {        // the running max moved for some row of the wave
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) O[dt][e] *= alpha;
    }
    u32x4 pw[4];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      uint32_t wbits = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int kk = key0 + sub * 32 + 8 * g + 4 * hh;
        uint32_t b01 = 0, b23 = 0;
        if (drop) {
          b01 = attn_pair_bits(rowkey, kk);
          b23 = attn_pair_bits(rowkey, kk + 2);
        }
        float pv[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const int e = 4 * g + e4;
          float p = __builtin_amdgcn_exp2f(S[sub][e] - ms);
          l += p;
          if (drop) {
            const bool kp = attn_keep(e4 < 2 ? b01 : b23, kk + e4, th16);
            wbits |= (uint32_t)kp << (8 * g + 4 * hh + e4);
            p = kp ? p : 0.f;
          }
          pv[e4] = p;
        }
        put4(pw[2 * sub + (g >> 1)], g & 1, pv);
      }
      if (drop && dmask) store_dmask(dmask, wbits, hh, (b * H + h), Lq, Lk, qi, key0 / 32 + sub);
    }
    bf16x8 pf[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) pf[q4] = __builtin_bit_cast(bf16x8, pw[q4]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int qrow = (lane & 15) >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = 16 * s + 4 * hh + qrow;
        const bf16x8 a = join(tr16(Vl + L::offc(row, c0)), tr16(Vl + L::offc(row + 8, c0)));
        O[dt] = mfma32(a, pf[s], O[dt]);
      }
    }
  }

  l += xor_lane(l, 32);
  if (qi < Lq) {
    const float inv = (drop ? dp.scale : 1.f) / l;
    bf16* orow = o + ((long)b * Lq + qi) * ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 w;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) w[e4] = (bf16)(O[dt][4 * g + e4] * inv);
        *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hh) = w;
      }
    if (hh == 0 && lse) lse[((long)b * H + h) * Lq + qi] = (m + __log2f(l)) * kLn2;
  }
}

// Per-block timestamps (start, LDS-DMA drained, tile loop done) of the resident backward
// kernels for tools/attn_phase.py: a separate -DRETR_ATTN_TIMING build in tools/_timing_attn/.
#ifdef RETR_ATTN_TIMING
__device__ long long g_attn_t[2][8192][3];
#define ATTN_T(K, i)                                                                          \
  if (threadIdx.x == 0) {                                                                     \
    const int blk_ = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;          \
    if (blk_ < 8192) g_attn_t[K][blk_][i] = wall_clock64();                                   \
  }
#else
#define ATTN_T(K, i)
#endif

// KSP = 2: the key tiles are split between two waves per 32 queries (even / odd tiles), which
// doubles the waves of a grid that is otherwise ~6 waves per CU at the RE⫶TR sizes; the two
// partial dQ accumulators are added through LDS at the end (fixed order: even + odd).
// DM (dropout source, compile-time so the score loop carries no runtime selects): 0 no dropout,
// 1 the forward's saved keep bits, 2 re-hashed decisions.
template <int HD, int NW, int KSP = 1, int DM = 1>
__global__ void __launch_bounds__(NW * 64)
attn_bwd_dq3_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v, long ldv,
                    const bf16* o, long ldo, const bf16* dout, long lddo, const float* lse,
                    float* Dout, bf16* dq, long lddq, int H, int Lq, int Lk,
                    const unsigned char* kpm, int causal, float qscale, float scale,
                    DropoutParams dp, int ntiles_max, const uint32_t* dmask) {
  using L = RL<HD>;
  constexpr int KS = HD / 16, DT = HD / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  constexpr int QW = NW / KSP;                    // query waves
  const int qw = wave % QW, kh = wave / QW;       // this wave's queries / key-tile parity
  const int qblk = bxyz.x * (32 * QW);
  const int q0 = qblk + qw * 32;
  const int qi = q0 + r;
  const int qc = qi < Lq ? qi : Lq - 1;
  const bf16* kb = k + (long)b * Lk * ldk + h * HD;
  const bf16* vb = v + (long)b * Lk * ldv + h * HD;
  const long srow = ((long)b * H + h) * Lq + qc;
  ATTN_T(0, 0)

  int kend = Lk;
  if (causal) kend = min(Lk, qblk + 32 * QW);
  const int ntiles = (kend + 63) / 64;
  char* Ks = smem;
  char* Vs = smem + (size_t)ntiles_max * L::TILE;
  unsigned long long* pm = (unsigned long long*)(smem + (size_t)2 * ntiles_max * L::TILE);
  dma_rows<HD, NW>(Ks, kb, ldk, ntiles, kend, wave, lane);
  dma_rows<HD, NW>(Vs, vb, ldv, ntiles, kend, wave, lane);
  for (int t = wave; t < ntiles; t += NW) {
    const int key = t * 64 + lane;
    bool pad = key >= Lk;
    if (kpm && !pad) pad = kpm[(long)b * Lk + key] != 0;
    const unsigned long long bm = __ballot(pad);
    if (lane == 0) pm[t] = bm;
  }

  bf16x8 qf[KS], dof[KS];
  float dpart = 0.f;
  {
    const bf16* qr = q + ((long)b * Lq + qc) * ldq + h * HD;
    const bf16* dr = dout + ((long)b * Lq + qc) * lddo + h * HD;
    const bf16* orr = o + ((long)b * Lq + qc) * ldo + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 x = *(const bf16x8*)(qr + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * qscale);
      qf[s] = x;
      const bf16x8 d8 = *(const bf16x8*)(dr + 16 * s + 8 * hh);
      const bf16x8 o8 = *(const bf16x8*)(orr + 16 * s + 8 * hh);
      dof[s] = d8;
#pragma unroll
      for (int j = 0; j < 8; ++j) dpart += (float)d8[j] * (float)o8[j];
    }
  }
  const float Dq = dpart + xor_lane(dpart, 32);
  if (hh == 0 && qi < Lq && kh == 0) Dout[srow] = Dq;
  const float lq2 = lse[srow] * kLog2e;
  const bool drop = dp.thresh != 0;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey = drop ? attn_row_key(dp_seed(dp), ((uint32_t)b * H + h) * Lq + qi) : 0u;
  const int nwm = (Lk + 31) / 32;

  f32x16 G[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) G[dt][e] = 0.f;
  dma_drain_barrier();
  ATTN_T(0, 1)

  const int wtiles = causal ? min(ntiles, (q0 + 32 + 63) / 64) : ntiles;
  for (int t = kh; t < wtiles; t += KSP) {
    const int key0 = t * 64;
    const char* Kl = Ks + t * L::TILE;
    const char* Vl = Vs + t * L::TILE;
    const unsigned long long pmask = pm[t];
    const bool diag = causal && (key0 + 63 > q0);
    const bool anym = pmask != 0ull || diag;      // wave-uniform: masking needed on this tile
    // keep words of the tile's two sub-tiles (bit j: key 32 sub + 8 g + 4 hh + e4 with
    // j = 8 g + e4 is neither padding nor past the causal diagonal): a bfe + and per score
    const unsigned long long pml = pmask >> (4 * hh);
    const int mlim = qi - key0 - 4 * hh;
    uint32_t kw[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int L = mlim - 32 * sub;                  // key j masked when j > L (causal)
      const uint32_t cm = diag ? (L < 0 ? ~0u : (L >= 31 ? 0u : (~0u << (L + 1)))) : 0u;
      kw[sub] = ~((uint32_t)(pml >> (32 * sub)) | cm);
    }
    uint32_t wm[2] = {0u, 0u};                     // saved keep bits of the tile's two sub-tiles
    if constexpr (DM == 1) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int w = min(key0 / 32 + sub, nwm - 1);
        wm[sub] = dmask[((long)(b * H + h) * nwm + w) * Lq + qc];
      }
    }
    f32x16 S[2], P[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int e = 0; e < 16; ++e) S[sub][e] = 0.f, P[sub][e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int off = L::off(sub * 32 + r, 2 * s + hh);
        S[sub] = mfma32(*(const bf16x8*)(Kl + off), qf[s], S[sub]);
        P[sub] = mfma32(*(const bf16x8*)(Vl + off), dof[s], P[sub]);
      }
    }
    // dS = P (drop(dP) - D); masking only on tiles that hold padded / causal-boundary keys
    u32x4 sw[4];
    auto scores = [&](auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int kk = key0 + sub * 32 + 8 * g + 4 * hh;
          uint32_t b01 = 0, b23 = 0;
          if constexpr (DM == 2) {
            b01 = attn_pair_bits(rowkey, kk);
            b23 = attn_pair_bits(rowkey, kk + 2);
          }
          float sv[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) {
            const int e = 4 * g + e4, kl = sub * 32 + 8 * g + 4 * hh + e4;
            float p = __builtin_amdgcn_exp2f(S[sub][e] - lq2);
            if constexpr (MASK)
              p = keep_and(p, __builtin_amdgcn_sbfe((int)kw[sub], kl - 4 * hh - 32 * sub, 1));
            float dpv = P[sub][e];
            if constexpr (DM == 1) {
              dpv = keep_and(dpv * dp.scale,
                             __builtin_amdgcn_sbfe((int)wm[sub], 8 * g + 4 * hh + e4, 1));
            } else if constexpr (DM == 2) {
              const bool kp = attn_keep(e4 < 2 ? b01 : b23, kk + e4, th16);
              dpv = kp ? dpv * dp.scale : 0.f;
            }
            sv[e4] = p * (dpv - Dq);
          }
          put4(sw[2 * sub + (g >> 1)], g & 1, sv);
        }
    };
    if (anym) scores(std::true_type{});
    else scores(std::false_type{});
    bf16x8 sf[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) sf[q4] = __builtin_bit_cast(bf16x8, sw[q4]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int qrow = (lane & 15) >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = 16 * s + 4 * hh + qrow;
        G[dt] = mfma32(join(tr16(Kl + L::offc(row, c0)), tr16(Kl + L::offc(row + 8, c0))),
                       sf[s], G[dt]);
      }
    }
  }
  ATTN_T(0, 2)
  if constexpr (KSP == 2) {
    // odd-tile partials -> LDS (over the K tiles: every wave is past its loop), even + odd
    __syncthreads();
    float* red = (float*)smem + (long)qw * DT * 16 * 64;
    if (kh == 1) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[(dt * 16 + e) * 64 + lane] = G[dt][e];
    }
    __syncthreads();
    if (kh == 1) return;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) G[dt][e] += red[(dt * 16 + e) * 64 + lane];
  }
  if (qi < Lq) {
    bf16* row = dq + ((long)b * Lq + qi) * lddq + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 w;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) w[e4] = (bf16)(G[dt][4 * g + e4] * scale);
        *(bf16x4*)(row + dt * 32 + 8 * g + 4 * hh) = w;
      }
  }
}

// KSP = 2: the query tiles are split between two waves per 32 keys (even / odd tiles); the
// dK / dV partials are added through LDS at the end (even + odd).
template <int HD, int NW, int KSP = 1, int DM = 1>
__global__ void __launch_bounds__(NW * 64)
attn_bwd_dkdv3_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v,
                      long ldv, const bf16* dout, long lddo, const float* lse, const float* D,
                      bf16* dk, long lddk, bf16* dv, long lddv, int H, int Lq, int Lk,
                      const unsigned char* kpm, int causal, float kscale, float scale,
                      DropoutParams dp, int ntiles_max, const uint32_t* dmask) {
  using L = RL<HD>;
  constexpr int KS = HD / 16, DT = HD / 32, NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  constexpr int KW = NW / KSP;                    // key waves
  const int kw = wave % KW, qh = wave / KW;       // this wave's keys / query-tile parity
  const int kblk = bxyz.x * (32 * KW);
  const int kj = kblk + kw * 32 + r;
  const int kc = kj < Lk ? kj : Lk - 1;
  const bf16* qb = q + (long)b * Lq * ldq + h * HD;
  const bf16* db = dout + (long)b * Lq * lddo + h * HD;
  const long sbase = ((long)b * H + h) * Lq;
  const bool drop = dp.thresh != 0;
  const uint64_t seed = drop ? dp_seed(dp) : 0ull;
  ATTN_T(1, 0)

  // queries [qstart, Lq) resident: tiles are numbered from qstart (causal skips the rows no key
  // of this block sees)
  const int qstart = causal ? (kblk / 64) * 64 : 0;
  const int ntiles = (Lq - qstart + 63) / 64;
  char* Qs = smem;
  char* Ds = smem + (size_t)ntiles_max * L::TILE;
  float* exl = (float*)(smem + (size_t)2 * ntiles_max * L::TILE);   // lse * log2e
  float* exd = exl + 64 * ntiles_max;                                 // D
  uint32_t* exk = (uint32_t*)(exd + 64 * ntiles_max);                 // dropout row keys
  // with saved keep bits: this wave's word column (its 32 keys) for every resident query
  uint32_t* exw = exk + 64 * ntiles_max + kw * 64 * ntiles_max;
  dma_rows<HD, NW>(Qs, qb + (long)qstart * ldq, ldq, ntiles, Lq - qstart, wave, lane);
  dma_rows<HD, NW>(Ds, db + (long)qstart * lddo, lddo, ntiles, Lq - qstart, wave, lane);
  for (int i = tid; i < ntiles * 64; i += NT) {
    const int qq = qstart + i;
    const int qcl = qq < Lq ? qq : Lq - 1;
    exl[i] = lse[sbase + qcl] * kLog2e;
    exd[i] = D[sbase + qcl];
    exk[i] = (drop && !dmask) ? attn_row_key(seed, (uint32_t)((b * H + h) * Lq) + (uint32_t)qq)
                              : 0u;
  }
  if (drop && dmask && qh == 0) {
    const int nwm = (Lk + 31) / 32;
    const int wc = min((kblk + kw * 32) / 32, nwm - 1);
    const uint32_t* col = dmask + ((long)(b * H + h) * nwm + wc) * Lq;
    for (int i = lane; i < ntiles * 64; i += 64) {
      const int qq = qstart + i;
      exw[i] = qq < Lq ? col[qq] : 0u;
    }
  }

  bf16x8 kf[KS], vf[KS];
  {
    const bf16* kr = k + ((long)b * Lk + kc) * ldk + h * HD;
    const bf16* vr = v + ((long)b * Lk + kc) * ldv + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 x = *(const bf16x8*)(kr + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * kscale);
      kf[s] = x;
      vf[s] = *(const bf16x8*)(vr + 16 * s + 8 * hh);
    }
  }
  const bool kmask = kj >= Lk || (kpm && kpm[(long)b * Lk + kc]);
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;

  f32x16 GK[DT], GV[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) GK[dt][e] = 0.f, GV[dt][e] = 0.f;
  dma_drain_barrier();
  ATTN_T(1, 1)

  // a wave's keys see no query below its first key (causal): skip those tiles
  const int kfirst = kblk + kw * 32;
  const int wt0 = causal ? max(0, (kfirst - qstart) / 64) : 0;
  for (int it = wt0 + ((wt0 & (KSP - 1)) != qh ? 1 : 0); it < ntiles; it += KSP) {
    const int qt = qstart + it * 64;
    const char* Ql = Qs + it * L::TILE;
    const char* Dl = Ds + it * L::TILE;
    const float* el = exl + it * 64;
    const float* ed = exd + it * 64;
    const uint32_t* ek = exk + it * 64;
    f32x16 S[2], P[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int e = 0; e < 16; ++e) S[sub][e] = 0.f, P[sub][e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int off = L::off(sub * 32 + r, 2 * s + hh);
        S[sub] = mfma32(*(const bf16x8*)(Ql + off), kf[s], S[sub]);
        P[sub] = mfma32(*(const bf16x8*)(Dl + off), vf[s], P[sub]);
      }
    }
    // P and dS.  Padded keys (kmask) are left unmasked here -- a lane's accumulators are only
    // ever its own key's dK / dV columns, written as zeros below -- and the row / causal masks
    // run only on tiles that hold rows past Lq or cross this wave's diagonal
    u32x4 pw[4], sw[4];
    auto scores = [&](auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      // keep words (bit j = 8 g + e4: query qt + 32 sub + 4 hh + j is a real row and, causal,
      // not above this lane's key): a bfe + and per score instead of two compares and a select
      uint32_t rw[2] = {~0u, ~0u};
      if constexpr (MASK) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          const int base = qt + 32 * sub + 4 * hh;
          rw[sub] = range_bits(causal ? kj - base : 0, Lq - base);
        }
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ql = sub * 32 + 8 * g + 4 * hh;
          const f32x4 l4 = *(const f32x4*)(el + ql);
          const f32x4 d4 = *(const f32x4*)(ed + ql);
          uint4 w4 = {0u, 0u, 0u, 0u};
          if constexpr (DM == 1) w4 = *(const uint4*)(exw + it * 64 + ql);
          float pv[4], sv[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) {
            const int e = 4 * g + e4;
            float p = __builtin_amdgcn_exp2f(S[sub][e] - l4[e4]);
            if constexpr (MASK) p = keep_and(p, __builtin_amdgcn_sbfe((int)rw[sub], 8 * g + e4, 1));
            float dpv = P[sub][e], pmv = p;
            if constexpr (DM == 1) {
              const uint32_t wv = e4 == 0 ? w4.x : e4 == 1 ? w4.y : e4 == 2 ? w4.z : w4.w;
              const int km = __builtin_amdgcn_sbfe((int)wv, r, 1);
              dpv = keep_and(dpv * dp.scale, km);
              pmv = keep_and(p * dp.scale, km);
            } else if constexpr (DM == 2) {
              const bool kp = attn_keep(attn_pair_bits(ek[ql + e4], (uint32_t)kj), (uint32_t)kj,
                                        th16);
              dpv = kp ? dpv * dp.scale : 0.f;
              pmv = kp ? p * dp.scale : 0.f;
            }
            pv[e4] = pmv;
            sv[e4] = p * (dpv - d4[e4]);
          }
          put4(pw[2 * sub + (g >> 1)], g & 1, pv);
          put4(sw[2 * sub + (g >> 1)], g & 1, sv);
        }
    };
    if (qt + 64 > Lq || (causal && qt < kfirst + 32)) scores(std::true_type{});
    else scores(std::false_type{});
    bf16x8 pf[4], sf[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      pf[q4] = __builtin_bit_cast(bf16x8, pw[q4]);
      sf[q4] = __builtin_bit_cast(bf16x8, sw[q4]);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int qrow = (lane & 15) >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = 16 * s + 4 * hh + qrow;
        GV[dt] = mfma32(join(tr16(Dl + L::offc(row, c0)), tr16(Dl + L::offc(row + 8, c0))),
                        pf[s], GV[dt]);
        GK[dt] = mfma32(join(tr16(Ql + L::offc(row, c0)), tr16(Ql + L::offc(row + 8, c0))),
                        sf[s], GK[dt]);
      }
    }
  }
  ATTN_T(1, 2)
  if constexpr (KSP == 2) {
    // odd-tile partials -> LDS (over the Q / dO tiles: every wave is past its loop)
    __syncthreads();
    float* red = (float*)smem + (long)kw * 2 * DT * 16 * 64;
    if (qh == 1) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          red[((2 * dt) * 16 + e) * 64 + lane] = GK[dt][e];
          red[((2 * dt + 1) * 16 + e) * 64 + lane] = GV[dt][e];
        }
    }
    __syncthreads();
    if (qh == 1) return;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        GK[dt][e] += red[((2 * dt) * 16 + e) * 64 + lane];
        GV[dt][e] += red[((2 * dt + 1) * 16 + e) * 64 + lane];
      }
  }
  if (kj < Lk) {
    bf16* krow = dk + ((long)b * Lk + kj) * lddk + h * HD;
    bf16* vrow = dv + ((long)b * Lk + kj) * lddv + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 wk, wv;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {   // a padded key's gradients are zero
          wk[e4] = kmask ? (bf16)0.f : (bf16)(GK[dt][4 * g + e4] * scale);
          wv[e4] = kmask ? (bf16)0.f : (bf16)GV[dt][4 * g + e4];
        }
        *(bf16x4*)(krow + dt * 32 + 8 * g + 4 * hh) = wk;
        *(bf16x4*)(vrow + dt * 32 + 8 * g + 4 * hh) = wv;
      }
  }
}

constexpr size_t kResLdsMax = 80 * 1024;   // two blocks per CU

template <class K>
void allow_lds(K kern, size_t lds) {
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
}

// resident mode: 0 auto, 1 streaming kernels only, 2 resident whenever it fits
int attn_res_mode() { return retr_tune_get(RETR_TUNE_ATTN_MODE); }

template <int HD, int NW>
int launch_fwd3(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                void* o, long ldo, int B, int H, int Lq, int Lk, const unsigned char* kpm,
                int causal, float p, unsigned long long seed, float* lse, uint32_t* dmask,
                hipStream_t st) {
  const float qscale = kLog2e / sqrtf((float)HD);
  const int nt = (Lk + 63) / 64;
  const size_t lds = res_lds_fwd<HD>(nt);
  auto kern = attn_fwd3_kernel<HD, NW>;
  allow_lds(kern, lds);
  dim3 grid((Lq + 32 * NW - 1) / (32 * NW), H, B);
  hipLaunchKernelGGL(kern, grid, dim3(NW * 64), lds, st, (const bf16*)q, ldq, (const bf16*)k,
                     ldk, (const bf16*)v, ldv, (bf16*)o, ldo, H, Lq, Lk, Lk, kpm, causal, qscale,
                     make_dp(p, seed), lse, nt, dmask);
  return retr_check_launch("attention_fwd3");
}

template <int HD, int NW, int DM>
int launch_bwd3_t(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                const void* o, long ldo, const void* dout, long lddo, const float* lse,
                void* dq, long lddq, void* dk, long lddk, void* dv, long lddv, int B, int H,
                int Lq, int Lk, const unsigned char* kpm, int causal, float p,
                unsigned long long seed, float* D, int nwq, int nwk, const uint32_t* dmask,
                hipStream_t st) {
  const float scale = 1.f / sqrtf((float)HD);
  const float cs = kLog2e * scale;
  const DropoutParams dp = make_dp(p, seed);
  const int ntk = (Lk + 63) / 64, ntq = (Lq + 63) / 64;
  // split knob: 1 off; 2 dq on every grid, dkdv on the 2-wave grids; 0 (auto) / 3 both only on
  // the 2-wave grids; 4 both everywhere.  With the branch-free score loops the 4-wave encoder
  // grid no longer gains from the dq split (tools/attn_micro.py bsplit,
  // profiles/r3_attn_bsplit.txt: encoder 400 x 400 52.9 -> 47.5 us at 3; the pre-rewrite A/B
  // that chose 2 is profiles/r3_attn_split.txt)
  const int sk = retr_tune_get(RETR_TUNE_ATTN_SPLIT);
  const bool split = sk == 2 || sk == 4 || ((sk == 0 || sk == 3) && nwq == 2);
  const bool split2 = sk != 1;          // dkdv: 2-wave grids only (below)
  {
    // the split kernel's partial-sum exchange (DT x 4 KB per query wave) aliases the K tiles
    const size_t lds = std::max(res_lds_fwd<HD>(ntk), (size_t)(split ? nwq * (HD / 32) * 4096 : 0));
    if (split) {   // 2 x nwq waves per block: nwq query waves x 2 key-tile parities
      if (nwq == 4) {
        auto kern = attn_bwd_dq3_kernel<HD, 8, 2, DM>;
        allow_lds(kern, lds);
        hipLaunchKernelGGL(kern, dim3((Lq + 127) / 128, H, B), dim3(512), lds, st, (const bf16*)q,
                           ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)o, ldo,
                           (const bf16*)dout, lddo, lse, D, (bf16*)dq, lddq, H, Lq, Lk, kpm,
                           causal, cs, scale, dp, ntk, dmask);
      } else {
        auto kern = attn_bwd_dq3_kernel<HD, 4, 2, DM>;
        allow_lds(kern, lds);
        hipLaunchKernelGGL(kern, dim3((Lq + 63) / 64, H, B), dim3(256), lds, st, (const bf16*)q,
                           ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)o, ldo,
                           (const bf16*)dout, lddo, lse, D, (bf16*)dq, lddq, H, Lq, Lk, kpm,
                           causal, cs, scale, dp, ntk, dmask);
      }
    } else if (nwq == 4) {
      auto kern = attn_bwd_dq3_kernel<HD, 4, 1, DM>;
      allow_lds(kern, lds);
      hipLaunchKernelGGL(kern, dim3((Lq + 127) / 128, H, B), dim3(256), lds, st, (const bf16*)q,
                         ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)o, ldo,
                         (const bf16*)dout, lddo, lse, D, (bf16*)dq, lddq, H, Lq, Lk, kpm, causal,
                         cs, scale, dp, ntk, dmask);
    } else {
      auto kern = attn_bwd_dq3_kernel<HD, 2, 1, DM>;
      allow_lds(kern, lds);
      hipLaunchKernelGGL(kern, dim3((Lq + 63) / 64, H, B), dim3(128), lds, st, (const bf16*)q,
                         ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)o, ldo,
                         (const bf16*)dout, lddo, lse, D, (bf16*)dq, lddq, H, Lq, Lk, kpm, causal,
                         cs, scale, dp, ntk, dmask);
    }
    if (int e = retr_check_launch("attention_bwd_dq3")) return e;
  }
  // the query-tile split of dkdv pays only on the 2-wave grids (decoder causal 128 x 128:
  // 21.5 -> 15.8 us); on the 4-wave ones it adds its exchange to short loops (cross 128 x 400:
  // 31.1 -> 35.1 us, tools/attn_bwd_ab.py, profiles/r3_attn_split.txt)
  const bool split_kv = split2 && (nwk == 2 || sk == 4);   // knob 4: on every grid
  const size_t lds = std::max(res_lds_dkdv<HD>(ntq),
                              (size_t)(split_kv ? nwk * 2 * (HD / 32) * 4096 : 0));
  if (split_kv) {
    if (nwk == 4) {
      auto kern = attn_bwd_dkdv3_kernel<HD, 8, 2, DM>;
      allow_lds(kern, lds);
      hipLaunchKernelGGL(kern, dim3((Lk + 127) / 128, H, B), dim3(512), lds, st, (const bf16*)q,
                         ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)dout, lddo,
                         lse, D, (bf16*)dk, lddk, (bf16*)dv, lddv, H, Lq, Lk, kpm, causal, cs,
                         scale, dp, ntq, dmask);
    } else {
      auto kern = attn_bwd_dkdv3_kernel<HD, 4, 2, DM>;
      allow_lds(kern, lds);
      hipLaunchKernelGGL(kern, dim3((Lk + 63) / 64, H, B), dim3(256), lds, st, (const bf16*)q,
                         ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)dout, lddo,
                         lse, D, (bf16*)dk, lddk, (bf16*)dv, lddv, H, Lq, Lk, kpm, causal, cs,
                         scale, dp, ntq, dmask);
    }
  } else if (nwk == 4) {
    auto kern = attn_bwd_dkdv3_kernel<HD, 4, 1, DM>;
    allow_lds(kern, lds);
    hipLaunchKernelGGL(kern, dim3((Lk + 127) / 128, H, B), dim3(256), lds, st, (const bf16*)q,
                       ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)dout, lddo, lse,
                       D, (bf16*)dk, lddk, (bf16*)dv, lddv, H, Lq, Lk, kpm, causal, cs, scale, dp,
                       ntq, dmask);
  } else {
    auto kern = attn_bwd_dkdv3_kernel<HD, 2, 1, DM>;
    allow_lds(kern, lds);
    hipLaunchKernelGGL(kern, dim3((Lk + 63) / 64, H, B), dim3(128), lds, st, (const bf16*)q,
                       ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)dout, lddo, lse,
                       D, (bf16*)dk, lddk, (bf16*)dv, lddv, H, Lq, Lk, kpm, causal, cs, scale, dp,
                       ntq, dmask);
  }
  return retr_check_launch("attention_bwd_dkdv3");
}

// dropout source of the backward kernels: 0 none, 1 the forward's saved keep bits, 2 re-hash
template <int HD, int NW>
int launch_bwd3(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                const void* o, long ldo, const void* dout, long lddo, const float* lse,
                void* dq, long lddq, void* dk, long lddk, void* dv, long lddv, int B, int H,
                int Lq, int Lk, const unsigned char* kpm, int causal, float p,
                unsigned long long seed, float* D, int nwq, int nwk, const uint32_t* dmask,
                hipStream_t st) {
  if (make_dp(p, seed).thresh == 0) return launch_bwd3_t<HD, NW, 0>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, nwq, nwk, dmask, st);
  if (dmask) return launch_bwd3_t<HD, NW, 1>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, nwq, nwk, dmask, st);
  return launch_bwd3_t<HD, NW, 2>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, nwq, nwk, dmask, st);
}

// 4 waves per block when that still gives >= 384 blocks, else 2
inline int pick_nw(int B, int H, int L) { return (long)B * H * ((L + 127) / 128) >= 384 ? 4 : 2; }

}  // namespace

// Internal entry (called by retr_attention_fwd for bf16 with hd in {32, 64}).
int retr_attention_fwd2(const void* q, long ldq, const void* k, long ldk, const void* v,
                        long ldv, void* o, long ldo, int B, int H, int Lq, int Lk, int hd,
                        const unsigned char* kpm, int causal, float p, unsigned long long seed,
                        float* lse, uint32_t* dmask, hipStream_t st) {
  // forward: the streaming kernel (20 KB of LDS, up to 8 blocks per CU) beats the resident
  // one (2 blocks per CU) at every cfg2 shape (tools/attn_micro.py: 400x400 24.8 vs 28.1 us);
  // the resident forward stays selectable (RETR_TUNE_ATTN_MODE = 2) for sweeps
  const int mode = attn_res_mode();
  const int ntk = (Lk + 63) / 64;
  const bool fits = hd == 32 ? res_lds_fwd<32>(ntk) <= kResLdsMax : res_lds_fwd<64>(ntk) <= kResLdsMax;
  if (mode == 2 && fits) {
    const int nw = pick_nw(B, H, Lq);
    if (hd == 32)
      return nw == 4 ? launch_fwd3<32, 4>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, kpm, causal, p, seed, lse, dmask, st)
                     : launch_fwd3<32, 2>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, kpm, causal, p, seed, lse, dmask, st);
    return nw == 4 ? launch_fwd3<64, 4>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, kpm, causal, p, seed, lse, dmask, st)
                   : launch_fwd3<64, 2>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, kpm, causal, p, seed, lse, dmask, st);
  }
  // key split (attn_fwd2s_kernel): knob 1 off; RETR_TUNE_ATTN_SPLIT = 1 (the unsplit kernels
  // everywhere) also turns it off, so the resident / streaming bitwise comparisons keep holding
  int fs = retr_tune_get(RETR_TUNE_ATTN_FSPLIT);
  if (retr_tune_get(RETR_TUNE_ATTN_SPLIT) == 1) fs = 1;
  // auto: split only grids of <= 1024 query waves (tools/attn_micro.py fsplit,
  // profiles/r3_attn_fsplit.txt: cross 128 x 400 18.8 -> 10.7 us at four parities, decoder
  // causal 128 x 128 7.9 -> 6.4 us at two; the encoder's 1664 query waves run 24.8 us unsplit
  // vs 30.1 split)
  if (fs == 0) {
    const long qwaves = (long)B * H * ((Lq + 31) / 32);
    fs = qwaves > 1024 || ntk < 2 ? 1 : (ntk >= 4 ? 3 : 2);
  }
  if (fs >= 2) {
#define RETR_FWD2S(HDV, NQ, KSP)                                                                  \
  launch_fwd2s<HDV, NQ, KSP>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, Lk, kpm, causal, p,  \
                             seed, lse, dmask, st)
    if (hd == 32) {
      if (fs == 3) return RETR_FWD2S(32, 1, 4);
      if (fs == 4) return RETR_FWD2S(32, 1, 2);
      return RETR_FWD2S(32, 2, 2);
    }
    if (fs == 3) return RETR_FWD2S(64, 1, 4);
    if (fs == 4) return RETR_FWD2S(64, 1, 2);
    return RETR_FWD2S(64, 2, 2);
#undef RETR_FWD2S
  }
  const bool big = (long)B * H * ((Lq + 63) / 64) >= 1024;
  if (hd == 32) {
    return big ? launch_fwd2<32, 4>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, Lk, kpm, causal, p, seed, lse, dmask, st)
               : launch_fwd2<32, 2>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, Lk, kpm, causal, p, seed, lse, dmask, st);
  }
  return big ? launch_fwd2<64, 4>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, Lk, kpm, causal, p, seed, lse, dmask, st)
             : launch_fwd2<64, 2>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, Lk, kpm, causal, p, seed, lse, dmask, st);
}

// =============================================================================================
// Backward (bf16, head dim 32 / 64).  Two kernels, no atomics (deterministic):
//  * dq2:   one wave = 32 queries (query on the lane, as the forward).  Per 64-key LDS tile:
//           S^T = K Q^T and dP^T = V dO^T, P = exp2(S^T - lse), dS = P (drop(dP) - D),
//           dQ^T += K^T dS^T (K^T by transposed LDS reads).  D = rowsum(dO * O) is formed in
//           the prologue from the lane's own dO / O fragments and written out for dkdv2.
//  * dkdv2: one wave = 32 keys (key on the lane).  Per 64-query LDS tile (Q, dO, lse, D):
//           S = Q K^T, dP = dO V^T, the same P / dS, then dV^T += dO^T drop(P) and
//           dK^T += Q^T dS (dO^T / Q^T by transposed LDS reads).
// Dropout masks are regenerated from the forward's (seed, row, key) hash.
// =============================================================================================

// one 64-row tile of two [rows][HD] tensors plus per-row scalars, register-staged into LDS
template <int HD, int NT>
struct RowStager {
  KVStager<HD, NT> kv;
  float lse2, dd;
  uint32_t rk;
  RETR_DEVICE void load(const bf16* a, long lda, const bf16* b, long ldb, int row0, int rows,
                        const float* lse, const float* D, long sbase, uint64_t seed, bool drop,
                        uint32_t rowbase, int tid) {
    kv.load(a, lda, b, ldb, row0, rows, tid);
    if (tid < 64) {
      const int rr = row0 + tid;
      const int rc = rr < rows ? rr : rows - 1;
      lse2 = lse[sbase + rc] * kLog2e;
      dd = D[sbase + rc];
      rk = drop ? attn_row_key(seed, rowbase + (uint32_t)rr) : 0u;
    }
  }
  RETR_DEVICE void store(char* stage, int tid) const {
    kv.store(stage, tid);
    if (tid < 64) {
      float* ex = (float*)(stage + Tile<HD>::STAGE);
      ex[tid] = lse2;
      ex[64 + tid] = dd;
      ((uint32_t*)ex)[128 + tid] = rk;
    }
  }
};

template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64)
attn_bwd_dq2_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v, long ldv,
                    const bf16* o, long ldo, const bf16* dout, long lddo, const float* lse,
                    float* Dout, bf16* dq, long lddq, int H, int Lq, int Lk,
                    const unsigned char* kpm, int causal, float qscale, float scale,
                    DropoutParams dp) {
  using TL = Tile<HD>;
  constexpr int NT = NW * 64, KS = HD / 16, DT = HD / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  const int qblk = bxyz.x * (32 * NW);
  const int q0 = qblk + wave * 32;
  const int qi = q0 + r;
  const int qc = qi < Lq ? qi : Lq - 1;
  const bf16* kb = k + (long)b * Lk * ldk + h * HD;
  const bf16* vb = v + (long)b * Lk * ldv + h * HD;
  const long srow = ((long)b * H + h) * Lq + qc;

  bf16x8 qf[KS], dof[KS];
  float dpart = 0.f;
  {
    const bf16* qr = q + ((long)b * Lq + qc) * ldq + h * HD;
    const bf16* dr = dout + ((long)b * Lq + qc) * lddo + h * HD;
    const bf16* orr = o + ((long)b * Lq + qc) * ldo + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 x = *(const bf16x8*)(qr + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * qscale);
      qf[s] = x;
      const bf16x8 d8 = *(const bf16x8*)(dr + 16 * s + 8 * hh);
      const bf16x8 o8 = *(const bf16x8*)(orr + 16 * s + 8 * hh);
      dof[s] = d8;
#pragma unroll
      for (int j = 0; j < 8; ++j) dpart += (float)d8[j] * (float)o8[j];
    }
  }
  const float Dq = dpart + xor_lane(dpart, 32);
  if (hh == 0 && qi < Lq) Dout[srow] = Dq;
  const float lq2 = lse[srow] * kLog2e;

  int kend = Lk;
  if (causal) kend = min(Lk, qblk + 32 * NW);
  const int ntiles = (kend + TL::KT - 1) / TL::KT;
  const bool drop = dp.thresh != 0;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint32_t rowkey = drop ? attn_row_key(dp_seed(dp), ((uint32_t)b * H + h) * Lq + qi) : 0u;

  f32x16 G[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) G[dt][e] = 0.f;

  KVStager<HD, NT> stg;
  stg.load(kb, ldk, vb, ldv, 0, Lk, tid);
  stg.store(smem, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * TL::KT;
    const char* Kl = smem + (t & 1) * TL::STAGE;
    const char* Vl = Kl + TL::BYTES;
    if (t + 1 < ntiles) stg.load(kb, ldk, vb, ldv, key0 + TL::KT, Lk, tid);
    bool pad = key0 + lane >= Lk;
    if (kpm && !pad) pad = kpm[(long)b * Lk + key0 + lane] != 0;
    const unsigned long long pmask = __ballot(pad);
    const bool diag = causal && (key0 + TL::KT - 1 > q0);
    const bool anym = pmask != 0ull || diag;      // wave-uniform: masking needed on this tile
    const unsigned long long pml = pmask >> (4 * hh);
    const uint32_t pmlo = (uint32_t)pml, pmhi = (uint32_t)(pml >> 32);
    const int mlim = qi - key0 - 4 * hh;
    u32x4 sw[4];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16 S, P;
#pragma unroll
      for (int e = 0; e < 16; ++e) S[e] = 0.f, P[e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int off = (sub * 32 + r) * TL::RB + (16 * s + 8 * hh) * 2;
        S = mfma32(*(const bf16x8*)(Kl + off), qf[s], S);
        P = mfma32(*(const bf16x8*)(Vl + off), dof[s], P);     // dP^T
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int kk = key0 + sub * 32 + 8 * g + 4 * hh;
        uint32_t b01 = 0, b23 = 0;
        if (drop) {
          b01 = attn_pair_bits(rowkey, kk);
          b23 = attn_pair_bits(rowkey, kk + 2);
        }
        float sv[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const int e = 4 * g + e4, kl = sub * 32 + 8 * g + 4 * hh + e4;
          const bool msk = anym & key_masked(pmlo, pmhi, kl - 4 * hh, diag, mlim);
          const float p = msk ? 0.f : __builtin_amdgcn_exp2f(S[e] - lq2);
          float dpv = P[e];
          if (drop) dpv = attn_keep(e4 < 2 ? b01 : b23, kk + e4, th16) ? dpv * dp.scale : 0.f;
          sv[e4] = p * (dpv - Dq);
        }
        put4(sw[2 * sub + (g >> 1)], g & 1, sv);
      }
    }
    bf16x8 sf[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) sf[q4] = __builtin_bit_cast(bf16x8, sw[q4]);
    // dQ^T += K^T dS^T
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int qrow = (lane & 15) >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const char* lo = Kl + (16 * s + 4 * hh + qrow) * TL::RB + c0 * 2;
        G[dt] = mfma32(join(tr16(lo), tr16(lo + 8 * TL::RB)), sf[s], G[dt]);
      }
    }
    if (t + 1 < ntiles) stg.store(smem + ((t + 1) & 1) * TL::STAGE, tid);
    __syncthreads();
  }
  if (qi < Lq) {
    bf16* row = dq + ((long)b * Lq + qi) * lddq + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 w;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) w[e4] = (bf16)(G[dt][4 * g + e4] * scale);
        *(bf16x4*)(row + dt * 32 + 8 * g + 4 * hh) = w;
      }
  }
}

template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64)
attn_bwd_dkdv2_kernel(const bf16* q, long ldq, const bf16* k, long ldk, const bf16* v,
                      long ldv, const bf16* dout, long lddo, const float* lse, const float* D,
                      bf16* dk, long lddk, bf16* dv, long lddv, int H, int Lq, int Lk,
                      const unsigned char* kpm, int causal, float kscale, float scale,
                      DropoutParams dp) {
  using TL = Tile<HD>;
  constexpr int NT = NW * 64, KS = HD / 16, DT = HD / 32;
  constexpr int STAGE = TL::STAGE + 3 * 64 * 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bxyz = xcd_block();
  const int b = bxyz.z, h = bxyz.y;
  const int kblk = bxyz.x * (32 * NW);
  const int kj = kblk + wave * 32 + r;          // this lane's key
  const int kc = kj < Lk ? kj : Lk - 1;
  const bf16* qb = q + (long)b * Lq * ldq + h * HD;
  const bf16* db = dout + (long)b * Lq * lddo + h * HD;
  const long sbase = ((long)b * H + h) * Lq;

  bf16x8 kf[KS], vf[KS];
  {
    const bf16* kr = k + ((long)b * Lk + kc) * ldk + h * HD;
    const bf16* vr = v + ((long)b * Lk + kc) * ldv + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 x = *(const bf16x8*)(kr + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * kscale);
      kf[s] = x;
      vf[s] = *(const bf16x8*)(vr + 16 * s + 8 * hh);
    }
  }
  const bool kmask = kj >= Lk || (kpm && kpm[(long)b * Lk + kc]);
  const bool drop = dp.thresh != 0;
  const uint32_t th16 = (dp.thresh + 0x8000u) >> 16;
  const uint64_t seed = drop ? dp_seed(dp) : 0ull;

  f32x16 GK[DT], GV[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) GK[dt][e] = 0.f, GV[dt][e] = 0.f;

  const int qstart = causal ? (kblk / TL::KT) * TL::KT : 0;
  RowStager<HD, NT> stg;
  stg.load(qb, ldq, db, lddo, qstart, Lq, lse, D, sbase, seed, drop,
           (uint32_t)((b * H + h) * Lq), tid);
  stg.store(smem, tid);
  __syncthreads();
  int it = 0;
  for (int qt = qstart; qt < Lq; qt += TL::KT, ++it) {
    const char* Ql = smem + (it & 1) * STAGE;
    const char* Dl = Ql + TL::BYTES;
    const float* ex = (const float*)(Ql + TL::STAGE);
    if (qt + TL::KT < Lq)
      stg.load(qb, ldq, db, lddo, qt + TL::KT, Lq, lse, D, sbase, seed, drop,
               (uint32_t)((b * H + h) * Lq), tid);
    u32x4 pw[4], sw[4];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16 S, P;
#pragma unroll
      for (int e = 0; e < 16; ++e) S[e] = 0.f, P[e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int off = (sub * 32 + r) * TL::RB + (16 * s + 8 * hh) * 2;
        S = mfma32(*(const bf16x8*)(Ql + off), kf[s], S);       // S = Q K^T (key on lane)
        P = mfma32(*(const bf16x8*)(Dl + off), vf[s], P);       // dP = dO V^T
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ql = sub * 32 + 8 * g + 4 * hh;               // 4 consecutive queries
        const f32x4 l4 = *(const f32x4*)(ex + ql);
        const f32x4 d4 = *(const f32x4*)(ex + 64 + ql);
        float pv[4], sv[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const int e = 4 * g + e4, qq = qt + ql + e4;
          const bool msk = kmask || qq >= Lq || (causal && kj > qq);
          float p = msk ? 0.f : __builtin_amdgcn_exp2f(S[e] - l4[e4]);
          float dpv = P[e], pm = p;
          if (drop) {
            const uint32_t rk = ((const uint32_t*)ex)[128 + ql + e4];
            const bool kp = attn_keep(attn_pair_bits(rk, (uint32_t)kj), (uint32_t)kj, th16);
            dpv = kp ? dpv * dp.scale : 0.f;
            pm = kp ? p * dp.scale : 0.f;
          }
          pv[e4] = pm;
          sv[e4] = p * (dpv - d4[e4]);
        }
        put4(pw[2 * sub + (g >> 1)], g & 1, pv);
        put4(sw[2 * sub + (g >> 1)], g & 1, sv);
      }
    }
    bf16x8 pf[4], sf[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      pf[q4] = __builtin_bit_cast(bf16x8, pw[q4]);
      sf[q4] = __builtin_bit_cast(bf16x8, sw[q4]);
    }
    // dV^T += dO^T drop(P);  dK^T += Q^T dS  (A operands by transposed reads of the tiles)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const int qrow = (lane & 15) >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int roff = (16 * s + 4 * hh + qrow) * TL::RB + c0 * 2;
        GV[dt] = mfma32(join(tr16(Dl + roff), tr16(Dl + roff + 8 * TL::RB)), pf[s], GV[dt]);
        GK[dt] = mfma32(join(tr16(Ql + roff), tr16(Ql + roff + 8 * TL::RB)), sf[s], GK[dt]);
      }
    }
    if (qt + TL::KT < Lq) stg.store(smem + ((it + 1) & 1) * STAGE, tid);
    __syncthreads();
  }
  if (kj < Lk) {
    bf16* krow = dk + ((long)b * Lk + kj) * lddk + h * HD;
    bf16* vrow = dv + ((long)b * Lk + kj) * lddv + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 wk, wv;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          wk[e4] = (bf16)(GK[dt][4 * g + e4] * scale);
          wv[e4] = (bf16)GV[dt][4 * g + e4];
        }
        *(bf16x4*)(krow + dt * 32 + 8 * g + 4 * hh) = wk;
        *(bf16x4*)(vrow + dt * 32 + 8 * g + 4 * hh) = wv;
      }
  }
}

template <int HD, int NW>
int launch_bwd2(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                const void* o, long ldo, const void* dout, long lddo, const float* lse,
                void* dq, long lddq, void* dk, long lddk, void* dv, long lddv, int B, int H,
                int Lq, int Lk, const unsigned char* kpm, int causal, float p,
                unsigned long long seed, float* D, hipStream_t st) {
  const float scale = 1.f / sqrtf((float)HD);
  const float cs = kLog2e * scale;
  const DropoutParams dp = make_dp(p, seed);
  hipLaunchKernelGGL((attn_bwd_dq2_kernel<HD, NW>), dim3((Lq + 32 * NW - 1) / (32 * NW), H, B),
                     dim3(NW * 64), 2 * Tile<HD>::STAGE, st, (const bf16*)q, ldq,
                     (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)o, ldo,
                     (const bf16*)dout, lddo, lse, D, (bf16*)dq, lddq, H, Lq, Lk, kpm, causal,
                     cs, scale, dp);
  if (int e = retr_check_launch("attention_bwd_dq2")) return e;
  hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<HD, NW>),
                     dim3((Lk + 32 * NW - 1) / (32 * NW), H, B), dim3(NW * 64),
                     2 * (Tile<HD>::STAGE + 3 * 64 * 4), st, (const bf16*)q, ldq,
                     (const bf16*)k, ldk, (const bf16*)v, ldv, (const bf16*)dout, lddo, lse, D,
                     (bf16*)dk, lddk, (bf16*)dv, lddv, H, Lq, Lk, kpm, causal, cs, scale, dp);
  return retr_check_launch("attention_bwd_dkdv2");
}

#ifdef RETR_ATTN_TIMING
extern "C" int retr_attn_timing_read(long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_t), sizeof(long long) * 2 * 8192 * 3);
}
#endif

int retr_attention_bwd2(const void* q, long ldq, const void* k, long ldk, const void* v,
                        long ldv, const void* o, long ldo, const void* dout, long lddo,
                        const float* lse, void* dq, long lddq, void* dk, long lddk, void* dv,
                        long lddv, int B, int H, int Lq, int Lk, int hd,
                        const unsigned char* kpm, int causal, float p, unsigned long long seed,
                        float* D, const uint32_t* dmask, hipStream_t st) {
  const int mode = attn_res_mode();
  const int ntk = (Lk + 63) / 64, ntq = (Lq + 63) / 64;
  const bool fits = hd == 32 ? (res_lds_fwd<32>(ntk) <= kResLdsMax && res_lds_dkdv<32>(ntq) <= kResLdsMax)
                             : (res_lds_fwd<64>(ntk) <= kResLdsMax && res_lds_dkdv<64>(ntq) <= kResLdsMax);
  if (mode != 1 && fits) {
    const int nwq = pick_nw(B, H, Lq), nwk = pick_nw(B, H, Lk);
    if (hd == 32)
      return launch_bwd3<32, 2>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk,
                                lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, nwq, nwk,
                                dmask, st);
    return launch_bwd3<64, 2>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk,
                              lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, nwq, nwk,
                              dmask, st);
  }
  if (hd == 32)
    return launch_bwd2<32, 2>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk,
                              lddk, dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, st);
  return launch_bwd2<64, 2>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk,
                            dv, lddv, B, H, Lq, Lk, kpm, causal, p, seed, D, st);
}
