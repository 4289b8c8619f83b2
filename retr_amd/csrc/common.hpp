// Shared definitions for the RE⫶TR gfx950 kernels (HIP, CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <algorithm>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

#define RETR_DEVICE __device__ __forceinline__

// ---- dtype tags (mirror include/retr_hip.h) --------------------------------------------------
enum { RETR_F32 = 0, RETR_BF16 = 1 };

// ---- error plumbing ---------------------------------------------------------------------------
void retr_set_error(const char* fmt, ...);
int retr_check_launch(const char* what);

#define RETR_REQUIRE(cond, ...)                  \
  do {                                           \
    if (!(cond)) {                               \
      retr_set_error(__VA_ARGS__);               \
      return 1;                                  \
    }                                            \
  } while (0)

// ---- conversions -------------------------------------------------------------------------------
template <typename T> RETR_DEVICE float to_f(T v) { return (float)v; }
template <typename T> RETR_DEVICE T from_f(float v) { return (T)v; }

// ---- counter-based dropout RNG -----------------------------------------------------------------
// keep(seed, idx) is a pure function of (seed, idx) so backward regenerates forward's mask.
RETR_DEVICE uint32_t retr_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
// threshold = p * 2^32 (host computes); element kept iff hash >= threshold
RETR_DEVICE bool retr_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  return retr_hash(seed, idx) >= thresh;
}

struct DropoutParams {
  uint64_t seed;
  uint32_t thresh;  // 0 => dropout disabled
  float scale;      // 1/(1-p)
  const unsigned long long* base = nullptr;  // device-side step seed (graph replays advance it)
};
// effective seed: per-op constant + the device-resident step seed (so a captured hipGraph draws
// fresh masks on every replay while backward still regenerates forward's mask)
RETR_DEVICE uint64_t dp_seed(const DropoutParams& dp) {
  return dp.base ? dp.seed + *dp.base : dp.seed;
}
const unsigned long long* retr_seed_base();
int retr_tune_get(int knob);  // retr_tune (capi.hip): launch-configuration overrides, 0 = auto
int retr_deterministic();   // retr_set_deterministic (capi.hip): fixed-order reductions only
inline DropoutParams make_dp(float p, unsigned long long seed) {
  DropoutParams dp{seed, 0u, 1.f, nullptr};
  if (p > 0.f) {
    dp.thresh = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
    dp.scale = 1.f / (1.f - p);
    dp.base = retr_seed_base();
  }
  return dp;
}

// ---- cheap attention-dropout RNG (fused attention kernels) -------------------------------------
// keep(row, key) from 16 bits of a 32-bit integer hash; one hash serves the key pair
// (2j, 2j+1).  row_key = attn_row_key(seed, row) is computed once per query row.  The keep
// probability is quantised to 1/65536 (p = 0.1 -> 0.100006); scale stays 1/(1-p).
RETR_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
RETR_DEVICE uint32_t attn_row_key(uint64_t seed, uint32_t row) {
  return mix32((uint32_t)seed ^ mix32(row * 0x9E3779B9u + (uint32_t)(seed >> 32)));
}
// per-element hash: the same xorshift-multiply finaliser on 24-bit multiplies
// (v_mul_u32_u24, full rate; a 32-bit v_mul_lo_u32 is quarter rate) -- the xorshift before
// each multiply folds bits 24..31 into the low 24, so no input bit is dropped
RETR_DEVICE uint32_t mix24(uint32_t x) {
  x ^= x >> 16;
  x = __umul24(x, 0xEB352Du);
  x ^= x >> 15;
  x = __umul24(x, 0x6CA68Bu);
  x ^= x >> 16;
  return x;
}
RETR_DEVICE uint32_t attn_pair_bits(uint32_t row_key, uint32_t key) {
  return mix24(row_key + __umul24(key >> 1, 0xEBCA77u));
}
RETR_DEVICE bool attn_keep(uint32_t bits, uint32_t key, uint32_t thresh16) {
  return ((key & 1) ? (bits >> 16) : (bits & 0xffffu)) >= thresh16;
}

// Element dropout of row-major activations (residual branches, embeddings): the same
// construction per (row, column pair) -- one 32-bit hash decides two columns -- instead of a
// 64-bit mix per element (3 64-bit multiplies).  Used identically by the forward epilogues and
// the backward's mask regeneration (retr_dropout_apply).
RETR_DEVICE uint32_t drop_th16(uint32_t thresh) { return (thresh + 0x8000u) >> 16; }
RETR_DEVICE uint32_t drop_row_key(uint64_t seed, uint32_t row) {
  return attn_row_key(seed ^ 0xA5A5F00Dull, row);
}
RETR_DEVICE bool drop_keep(uint32_t row_key, uint32_t col, uint32_t th16) {
  return attn_keep(attn_pair_bits(row_key, col), col, th16);
}
// keep bits of columns n .. n+7 (n even): bit e = column n + e
RETR_DEVICE uint32_t drop_keep8(uint32_t row_key, uint32_t n, uint32_t th16) {
  uint32_t m = 0;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const uint32_t b = attn_pair_bits(row_key, n + e);
    m |= (uint32_t)((b & 0xffffu) >= th16) << e;
    m |= (uint32_t)((b >> 16) >= th16) << (e + 1);
  }
  return m;
}

// keep bits of columns n .. n+3 (n even): bit e = column n + e
RETR_DEVICE uint32_t drop_keep4(uint32_t row_key, uint32_t n, uint32_t th16) {
  uint32_t m = 0;
#pragma unroll
  for (int e = 0; e < 4; e += 2) {
    const uint32_t b = attn_pair_bits(row_key, n + e);
    m |= (uint32_t)((b & 0xffffu) >= th16) << e;
    m |= (uint32_t)((b >> 16) >= th16) << (e + 1);
  }
  return m;
}

// ---- wave reductions (wave64) ------------------------------------------------------------------
// The xor butterfly v = op(v, v[lane ^ o]) for o = 32, 16, 8, 4, 2, 1 -- the bits of the
// __shfl_xor loop -- without its six ds_bpermute round trips through the LDS crossbar:
//   o = 32 / 16: v_permlane32_swap / v_permlane16_swap of v with itself hand every lane the
//                value of the other half / the neighbouring 16-lane row;
//   o = 8, 4, 2, 1: DPP row rotations: after the wider steps each value equals (bitwise) its
//                partners' under those xors, so lane (l + o) mod 16 holds the bits of lane l ^ o.
// The swaps give the two operands in lane-half order; they are put back in (own, partner)
// order per lane, so even an operand-order-sensitive op returns the butterfly's bits.
// v of lane (lane ^ o), o in {1, 2, 4, 8, 16, 32} -- what __shfl_xor(v, o, 64) returns -- from
// DPP moves / permlane swaps instead of a ds_bpermute through the LDS crossbar (o must fold to
// a constant; tools/wave_reduce_check.py checks every o against __shfl_xor)
RETR_DEVICE unsigned xor_lane_u(unsigned v, int o) {
  const unsigned lane = __lane_id();
  if (o == 32 || o == 16) {
    const auto s = o == 32 ? __builtin_amdgcn_permlane32_swap(v, v, false, false)
                           : __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & o) ? s[0] : s[1];
  }
  if (o == 8) return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xf, 0xf, false);   // row_ror:8
  if (o == 4) {   // row_shl:4 / row_shr:4 (lane i <- i + 4 / i - 4 within the 16-lane row)
    const unsigned up = __builtin_amdgcn_update_dpp(0u, v, 0x104, 0xf, 0xf, false);
    const unsigned dn = __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);
    return (lane & 4) ? dn : up;
  }
  if (o == 2) return __builtin_amdgcn_update_dpp(0u, v, 0x4e, 0xf, 0xf, false);    // quad [2,3,0,1]
  return __builtin_amdgcn_update_dpp(0u, v, 0xb1, 0xf, 0xf, false);                 // quad [1,0,3,2]
}
RETR_DEVICE float xor_lane(float v, int o) { return __uint_as_float(xor_lane_u(__float_as_uint(v), o)); }
RETR_DEVICE int xor_lane(int v, int o) { return (int)xor_lane_u((unsigned)v, o); }

template <class F>
RETR_DEVICE float wave_butterfly(float v, F op) {
  const unsigned lane = __lane_id();
  const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                    false, false);
  float lo = __uint_as_float(s32[0]), hi = __uint_as_float(s32[1]);
  v = (lane & 32) ? op(hi, lo) : op(lo, hi);
  const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v),
                                                    false, false);
  lo = __uint_as_float(s16[0]);
  hi = __uint_as_float(s16[1]);
  v = (lane & 16) ? op(hi, lo) : op(lo, hi);
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false)));
  return v;
}
RETR_DEVICE float wave_sum(float v) {
  return wave_butterfly(v, [](float a, float b) { return a + b; });
}
RETR_DEVICE float wave_max(float v) {
  return wave_butterfly(v, [](float a, float b) { return fmaxf(a, b); });
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
