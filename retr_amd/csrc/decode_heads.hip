// Decode-step attention sub-layers as one WAVE per (query row, head) (round 5).
//
// csrc/decode.hip's dec_attn_row runs one block per query row: at B = 64 captions that is 64
// blocks on 256 CUs, and each of them streams the whole out-projection and next-query weights
// (2 x 128 KB at C = 256) and every head's keys / values through one CU's load pipeline (13.7 /
// 11.9 us per launch at cfg5, profiles/r4_rocprof_decode.txt).  Here a launch has R x H waves
// (512 at B = 64, 2 per CU), and each wave reads only its head's slices:
//
//   dec_self_heads   q|k|v of head h from LN1(x) (+pos) -- the [q | k | v] projection rows
//                    of the head (3 x HD x C weights), k / v appended to the cache row -- then
//                    attention over the cache (beam ancestry), then the head's PARTIAL
//                    out-projection o_h Wo[:, h]^T into slab[h][r][:] (fp32)
//   dec_cross_heads  x' = x + (sum_h slab_in[h][r] + b_o) (heads in order; wave h = 0 writes x'),
//                    LN2(x') + pos, the head's cross query q_h = (.) Wq[h]^T + b_q, attention over
//                    the image memory (key-padding mask), the head's partial out-projection
//                    into slab_out[h][r][:]
//   (retr_dec_rows then sums slab_out in head order + b_o + residual and runs LN3.)
//
// The old dec_gemm launch is folded into dec_self_heads.  Roundings follow the unfused path:
// bf16 q / k / v / attention output (q also rounded after the 1/sqrt(hd) scale), fp32
// accumulation and residual; the out-projection sums per head and then over heads (a different
// fp32 order than one 256-term dot).
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

template <int CTRL>
RETR_DEVICE float dh_dpp(float s) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s),
                                                               CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of G lanes (G = 4 or 8); every lane of a group ends with the sum
template <int G>
RETR_DEVICE float gsum(float s) {
  static_assert(G == 4 || G == 8, "group of 4 or 8 lanes");
  s += dh_dpp<0xB1>(s);
  s += dh_dpp<0x4E>(s);
  if constexpr (G == 8) s += dh_dpp<0x141>(s);
  return s;
}

RETR_DEVICE float bfr(float v) { return (float)(bf16)v; }   // round to bf16 and back

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// sum_e a[e] b[e] over 8 bf16 pairs by v_dot2c_f32_bf16, two independent chains (a single wave
// per SIMD: every dependent VALU op exposes its latency)
RETR_DEVICE float dot8(const bf16x8& a, const bf16x8& b) {
  float s0 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a[0], a[1]}, bf16x2{b[0], b[1]}, 0.f, false);
  float s1 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a[2], a[3]}, bf16x2{b[2], b[3]}, 0.f, false);
  s0 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a[4], a[5]}, bf16x2{b[4], b[5]}, s0, false);
  s1 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a[6], a[7]}, bf16x2{b[6], b[7]}, s1, false);
  return s0 + s1;
}
RETR_DEVICE bf16x8 to_bf8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (bf16)v[e];
  return r;
}

// (row unit, head) of block b.  Hardware dispatches block b to XCD b % 8; with every head block
// of a row on one XCD that XCD's L2 serves the row's partial slabs to all its heads (they were
// fetched into all eight L2s) and the 128-byte K / V cache lines the row's heads share (a head's
// 32 dimensions are half a line), at the price of every XCD reading every head's weight slices
// (a few hundred KB per launch).  Needs units % 8 == 0, else row-major.
RETR_DEVICE void dec_block_rh(int b, int units, int H, bool xcd, int& r, int& h) {
  if ((units & 7) == 0 && xcd) {
    const int x = b & 7, q = b >> 3;
    r = x * (units >> 3) + q / H;
    h = q % H;
  } else {
    r = b / H;
    h = b % H;
  }
}

// this lane's activation chunks (c + 8 m) of a bf16 row
template <int C>
RETR_DEVICE void load_act(const bf16* row, int lane, bf16x8 (&act)[C / 64]) {
  const int c = lane & 7;
#pragma unroll
  for (int m = 0; m < C / 64; ++m) act[m] = *(const bf16x8*)(row + 8 * (c + 8 * m));
}

// Attention of one wave over its key range [j0, j1), at most NCH x CH keys: every key / value load
// is issued by load() (at kernel start: they depend on nothing computed in the step), then
// compute() runs an online softmax over the NCH chunks.  Lane = (dim group g = lane % NG of 8
// dims, key part = lane / NG): key j = j0 + CH c + part + NPART u.  key_row(j) gives the K/V row
// of key j, -1 for the step's own key (its K/V in LDS: kn / vn) or -2 for a masked key.
template <int HD, int NCH, int KU>
struct WaveAttn {
  static constexpr int NG = HD / 8, NPART = 64 / NG, CH = NPART * KU;
  long row[NCH][KU];
  bf16x8 kk[NCH][KU], vv[NCH][KU];
  bool mk[NCH][KU] = {};                            // key-padding flags (load_mask)
  float mx = -INFINITY, sum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  // key-padding flags of the wave's keys, loaded BEFORE (and independently of) the keys /
  // values: a mask test inside key_row would make every K / V address wait for its mask byte
  RETR_DEVICE void load_mask(const unsigned char* km, int j0, int j1, int lane) {
    if (!km) return;
    const int part = lane / NG;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int j = j0 + CH * c + part + NPART * u;
        mk[c][u] = j < j1 && km[j] != 0;
      }
  }

  // the K / V rows of the wave's keys (key_row may read memory: the beam ancestry table) --
  // called first in a kernel, so that waiting for those reads does not wait for later loads
  template <class RowFn>
  RETR_DEVICE void set_rows(int j0, int j1, RowFn key_row, int lane) {
    const int part = lane / NG;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int j = j0 + CH * c + part + NPART * u;
        row[c][u] = j < j1 ? key_row(j) : -2;
      }
  }
  template <int C, class RowFn>
  RETR_DEVICE void load(const bf16* __restrict__ K, const bf16* __restrict__ V, int h, int j0,
                        int j1, RowFn key_row, int lane) {
    set_rows(j0, j1, key_row, lane);
    load_rows<C>(K, V, h, lane);
  }
  template <int C>
  RETR_DEVICE void load_rows(const bf16* __restrict__ K, const bf16* __restrict__ V, int h,
                             int lane) {
    const int g = lane % NG;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int u = 0; u < KU; ++u)
        kk[c][u] = row[c][u] >= 0 ? *(const bf16x8*)(K + row[c][u] * C + h * HD + 8 * g)
                                  : bf16x8{};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int u = 0; u < KU; ++u)
        vv[c][u] = row[c][u] >= 0 ? *(const bf16x8*)(V + row[c][u] * C + h * HD + 8 * g)
                                  : bf16x8{};
  }

  RETR_DEVICE void compute(const float* qs, const float* kn, const float* vn, int lane) {
    const int g = lane % NG;
    const bf16x8 q = to_bf8(qs + 8 * g);            // bf16-rounded values: exact
    const bf16x8 knb = kn ? to_bf8(kn + 8 * g) : bf16x8{};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float sc[KU];
      float cm = -INFINITY;
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        float s = dot8(q, row[c][u] == -1 ? knb : kk[c][u]);
        s = gsum<NG>(s);
        sc[u] = (row[c][u] == -2 || mk[c][u]) ? -INFINITY : s;
        cm = fmaxf(cm, sc[u]);
      }
      cm = wave_max(cm);
      const float nm = fmaxf(mx, cm);
      if (nm != -INFINITY) {
        const float f = mx == -INFINITY ? 0.f : __expf(mx - nm);
        sum *= f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] *= f;
        float cs = 0.f;
#pragma unroll
        for (int u = 0; u < KU; ++u) {
          const float p = sc[u] == -INFINITY ? 0.f : __expf(sc[u] - nm);
          cs += p;                                 // NG copies of every key: divided out below
          if (row[c][u] == -1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += p * vn[8 * g + e];
          } else {
            const bf16x8 vs = mk[c][u] ? bf16x8{} : vv[c][u];   // as an unloaded masked key
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += p * (float)vs[e];
          }
        }
        sum += wave_sum(cs) * (1.0f / NG);
        mx = nm;
      }
    }
  }
  // compute() over keys / values resident in LDS ([keys][HD] images, key j of the wave at row
  // j): the same arithmetic, each key's K / V read inside the loops instead of held in registers
  // from load() (NCH = 1)
  RETR_DEVICE void compute_lds(const float* qs, const bf16* Ks, const bf16* Vs, int j0, int j1,
                               int lane) {
    static_assert(NCH == 1, "one chunk");
    const int g = lane % NG, part = lane / NG;
    const bf16x8 q = to_bf8(qs + 8 * g);
    float sc[KU];
    float cm = -INFINITY;
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int j = j0 + part + NPART * u;
      const bool ok = j < j1 && !mk[0][u];
      const bf16x8 kk8 = ok ? *(const bf16x8*)(Ks + j * HD + 8 * g) : bf16x8{};
      float sv = dot8(q, kk8);
      sv = gsum<NG>(sv);
      sc[u] = ok ? sv : -INFINITY;
      cm = fmaxf(cm, sc[u]);
    }
    cm = wave_max(cm);
    const float nm = fmaxf(mx, cm);
    if (nm != -INFINITY) {
      const float f = mx == -INFINITY ? 0.f : __expf(mx - nm);
      sum *= f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= f;
      float cs = 0.f;
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int j = j0 + part + NPART * u;
        const float p = sc[u] == -INFINITY ? 0.f : __expf(sc[u] - nm);
        cs += p;
        const bf16x8 vv8 = sc[u] == -INFINITY ? bf16x8{} : *(const bf16x8*)(Vs + j * HD + 8 * g);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += p * (float)vv8[e];
      }
      sum += wave_sum(cs) * (1.0f / NG);
      mx = nm;
    }
  }
  // this wave's (max, sum, unnormalised P V) into LDS slot w
  RETR_DEVICE void publish(float* mxs, float* sms, float* accs, int w, int lane) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = NG; o < 64; o <<= 1) acc[e] += xor_lane(acc[e], o);
    if (lane == 0) {
      mxs[w] = mx;
      sms[w] = sum;
    }
    if (lane < NG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) accs[w * HD + 8 * lane + e] = acc[e];
    }
  }
};

// o[d] (bf16-rounded, normalised) from NW waves' partial softmax states, for d = lane < HD
template <int HD, int NW>
RETR_DEVICE void merge_heads(const float* mxs, const float* sms, const float* accs, float* os,
                             int lane) {
  if (lane >= HD) return;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) M = fmaxf(M, mxs[w]);
  float num = 0.f, den = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float f = mxs[w] == -INFINITY ? 0.f : __expf(mxs[w] - M);
    num += accs[w * HD + lane] * f;
    den += sms[w] * f;
  }
  os[lane] = bfr(num * (1.f / den));               // a fully masked row gives NaN, as torch
}

// ND of a head's projection rows, [row0, row0 + ND) of W (C columns each), loaded up front in
// the dot's lane layout: lane = (row group rg = lane / 8, chunk column c = lane % 8), lane c owns
// the 16-byte chunks c, c + 8, ... of every row
template <int C, int ND>
struct ProjW {
  static constexpr int CPL = C / 64;
  bf16x8 w[ND / 8][CPL];
  RETR_DEVICE void load(const bf16* __restrict__ W, int row0, int lane, int ld = C) {
    const int rg = lane >> 3, c = lane & 7;
#pragma unroll
    for (int it = 0; it < ND / 8; ++it)
#pragma unroll
      for (int m = 0; m < CPL; ++m)
        w[it][m] = *(const bf16x8*)(W + (long)(row0 + 8 * it + rg) * ld + 8 * (c + 8 * m));
  }
  // out[d] (LDS) = sum_k W[row0 + d][k] act[k]  (one dot8 per chunk, chunks summed pairwise)
  RETR_DEVICE void dot(const bf16x8 (&act)[CPL], int lane, float* out) const {
    const int rg = lane >> 3, c = lane & 7;
#pragma unroll
    for (int it = 0; it < ND / 8; ++it) {
      float p[CPL];
#pragma unroll
      for (int m = 0; m < CPL; ++m) p[m] = dot8(w[it][m], act[m]);
#pragma unroll
      for (int st = 1; st < CPL; st <<= 1)
#pragma unroll
        for (int m = 0; m + st < CPL; m += 2 * st) p[m] += p[m + st];
      const float s = gsum<8>(p[0]);
      if (c == 0) out[8 * it + rg] = s;
    }
  }
};

// NM groups of 64 out-projection rows (n = lane + 64 (m0 + m)), the head's HD columns of each
template <int C, int HD, int NM>
struct OutW {
  bf16x8 w[NM][HD / 8];
  RETR_DEVICE void load(const bf16* __restrict__ Wo, int h, int m0, int lane, int ld = C) {
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int t = 0; t < HD / 8; ++t)
        w[m][t] = *(const bf16x8*)(Wo + (long)(lane + 64 * (m0 + m)) * ld + h * HD + 8 * t);
  }
  // slab[n] = sum_{d < HD} o[d] Wo[n][h HD + d]
  RETR_DEVICE void apply(const float* os, float* slab, int m0, int lane) const {
    bf16x8 o[HD / 8];                               // bf16-rounded attention output: exact
#pragma unroll
    for (int t = 0; t < HD / 8; ++t) o[t] = to_bf8(os + 8 * t);
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      float p[HD / 8];
#pragma unroll
      for (int t = 0; t < HD / 8; ++t) p[t] = dot8(o[t], w[m][t]);
#pragma unroll
      for (int st = 1; st < HD / 8; st <<= 1)
#pragma unroll
        for (int t = 0; t + st < HD / 8; t += 2 * st) p[t] += p[t + st];
      slab[lane + 64 * (m0 + m)] = p[0];
    }
  }
};

struct SelfHeadsArgs {
  const bf16* n;        // LN1(x) [R][C]
  const bf16* npos;     // LN1(x) + qpos
  const bf16* win;      // [3C][C]
  const float* bin;     // [3C]
  bf16* kc;             // caches [R * Lmax][C]
  bf16* vc;
  int i, Lmax;          // this step's position (keys 0..i), cache rows per caption
  const int* anc;       // [R][Lmax] beam ancestry or null
  const bf16* wo;       // [C][C]
  float* slab;          // [H][R][C]
  int R;
  // LN1 prologue (xin != null; n / npos unused): x = xin + (sum_j slabs[j] + b2) (the previous
  // layer's FFN partials [nslab][R][C]) -> xout (block h = 0), n = bf16(LN1(x)), npos =
  // bf16(LN1(x) + qpos) -- instead of a retr_dec_rows launch between the layers
  const float* xin;
  const float* slabs;
  int nslab;
  const float* b2;
  const float* gamma;
  const float* beta;
  float eps;
  const float* qpos;
  float* xout;
  bool xcd = true;      // dec_block_rh order (RETR_TUNE_DEC_ORDER)
  // embedding prologue (tok != null, layer 0; xin / slabs unused): x = LN_e(word[tok] + qpos)
  // (DecoderEmbeddings) -> xout (block h = 0), then LN1 as above -- instead of a
  // retr_dec_embed_rows launch before the first layer
  const long long* tok = nullptr;
  const float* word = nullptr;
  const float* ge = nullptr;
  const float* be = nullptr;
  float epse = 0.f;
};

// One block of NW waves per (row, head): wave w computes rows [w HD / NW, (w + 1) HD / NW) of
// the head's q, k, v, attends over keys [w KPW, (w + 1) KPW), and computes out-projection rows
// n in its NM-group share; the waves' softmax states merge through LDS.
template <int C, int HD, int NW, int NCH, int KU>
__global__ void __launch_bounds__(64 * NW) dec_self_heads_kernel(SelfHeadsArgs a, float scale) {
  constexpr int H = C / HD, ND = HD / NW, NM = C / 64 / NW;
  constexpr int KPW = NCH * (64 / (HD / 8)) * KU;  // keys per wave
  constexpr int CPL = C / 64;
  typedef __attribute__((ext_vector_type(4))) float f4v;
  __shared__ float qs[HD], ks[HD], vs[HD], os[HD];
  __shared__ float mxs[NW], sms[NW], accs[NW * HD];
  __shared__ __attribute__((aligned(16))) float part[NW][C];   // LN1 prologue slab partials
  __shared__ __attribute__((aligned(16))) bf16 lnb[2][C];      // LN1 prologue n / npos
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int r, h;
  dec_block_rh(blockIdx.x, a.R, H, a.xcd, r, h);
  const int* ar = a.anc ? a.anc + (long)r * a.Lmax : nullptr;
  const int i = a.i, Lmax = a.Lmax;
  const bool emb = a.tok != nullptr;
  const bool pro = a.xin != nullptr || emb;
  const long long tokr = emb ? a.tok[r] : 0;
  WaveAttn<HD, NCH, KU> at;
  at.set_rows(w * KPW, min(i + 1, (w + 1) * KPW),
              [&](int j) -> long {
                if (j == i) return -1;
                return (long)(ar ? ar[j] : r) * Lmax + j;
              },
              lane);
  // every global load first (one dependent memory round trip per launch): the LN1 prologue's
  // slab share (wave w: slabs [w S / NW, (w + 1) S / NW)), activations, this wave's q|k|v and
  // out-projection weight rows, its cached keys / values of positions < i
  const int c0 = CPL * lane;
  float ps[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) ps[e] = 0.f;
  if (emb) {                                   // the token's word-embedding chunk
#pragma unroll
    for (int e = 0; e < CPL; e += 4) *(f4v*)(ps + e) = *(const f4v*)(a.word + tokr * C + c0 + e);
  } else if (pro) {
    const long RC = (long)a.R * C;
    const int s0 = w * a.nslab / NW, s1 = (w + 1) * a.nslab / NW;
    for (int j = s0; j < s1; j += 8) {
      f4v t[8][CPL / 4];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < CPL / 4; ++e)
          t[u][e] = j + u < s1 ? *(const f4v*)(a.slabs + (j + u) * RC + (long)r * C + c0 + 4 * e)
                               : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < CPL / 4; ++e)
#pragma unroll
          for (int f = 0; f < 4; ++f)
            if (j + u < s1) ps[4 * e + f] += t[u][e][f];
    }
  }
  bf16x8 actp[C / 64], actn[C / 64];
  if (!pro) {
    load_act<C>(a.npos + (long)r * C, lane, actp);
    load_act<C>(a.n + (long)r * C, lane, actn);
  }
  ProjW<C, ND> wq, wk, wv;
  wq.load(a.win, h * HD + w * ND, lane);
  wk.load(a.win, C + h * HD + w * ND, lane);
  wv.load(a.win, 2 * C + h * HD + w * ND, lane);
  at.template load_rows<C>(a.kc, a.vc, h, lane);
  OutW<C, HD, NM> wo;
  wo.load(a.wo, h, w * NM, lane);
  const int d = w * ND + lane;
  const float bq = lane < ND ? a.bin[h * HD + d] : 0.f;
  const float bk = lane < ND ? a.bin[C + h * HD + d] : 0.f;
  const float bv = lane < ND ? a.bin[2 * C + h * HD + d] : 0.f;
  if (pro) {
    // x = xin + (slab partials in wave order + b2), or the token embedding; LN1 (+ qpos) -> LDS
    float xv[CPL], b2[CPL], gm[CPL], bt[CPL], qp[CPL];
#pragma unroll
    for (int e = 0; e < CPL; e += 4) {
      if (emb) {
        *(f4v*)(xv + e) = *(const f4v*)(a.ge + c0 + e);
        *(f4v*)(b2 + e) = *(const f4v*)(a.be + c0 + e);
      } else {
        *(f4v*)(xv + e) = *(const f4v*)(a.xin + (long)r * C + c0 + e);
        *(f4v*)(b2 + e) = *(const f4v*)(a.b2 + c0 + e);
      }
      *(f4v*)(gm + e) = *(const f4v*)(a.gamma + c0 + e);
      *(f4v*)(bt + e) = *(const f4v*)(a.beta + c0 + e);
      *(f4v*)(qp + e) = *(const f4v*)(a.qpos + c0 + e);
    }
    float v[CPL], sm = 0.f;
    if (emb) {
      // DecoderEmbeddings: LN_e(word + position) (ps holds the word chunk; xv / b2 = ge / be)
      float u[CPL], su = 0.f;
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        u[e] = ps[e] + qp[e];
        su += u[e];
      }
      const float me = wave_sum(su) / C;
      float qe = 0.f;
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        const float dd = u[e] - me;
        qe += dd * dd;
      }
      const float re = 1.0f / sqrtf(wave_sum(qe) / C + a.epse);
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        v[e] = (u[e] - me) * re * xv[e] + b2[e];
        sm += v[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < CPL; ++e) part[w][c0 + e] = ps[e];
      __syncthreads();
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        float t = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) t += part[ww][c0 + e];
        v[e] = xv[e] + (t + b2[e]);
        sm += v[e];
      }
    }
    if (h == 0 && w == 0) {
#pragma unroll
      for (int e = 0; e < CPL; e += 4) *(f4v*)(a.xout + (long)r * C + c0 + e) = *(f4v*)(v + e);
    }
    const float mean = wave_sum(sm) / C;
    float q2 = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const float dd = v[e] - mean;
      q2 += dd * dd;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q2) / C + a.eps);
    if (w == 0) {
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        const float o = (v[e] - mean) * rstd * gm[e] + bt[e];
        lnb[0][c0 + e] = (bf16)o;
        lnb[1][c0 + e] = (bf16)(o + qp[e]);
      }
    }
    __syncthreads();
    const int c = lane & 7;
#pragma unroll
    for (int m = 0; m < C / 64; ++m) {
      actn[m] = *(const bf16x8*)(&lnb[0][8 * (c + 8 * m)]);
      actp[m] = *(const bf16x8*)(&lnb[1][8 * (c + 8 * m)]);
    }
  }
  wq.dot(actp, lane, qs + w * ND);
  wk.dot(actp, lane, ks + w * ND);
  wv.dot(actn, lane, vs + w * ND);
  __syncthreads();
  // bias + bf16 rounding (the unfused path's bf16 q / k / v); k, v appended to the cache
  float q = 0.f, k = 0.f, v = 0.f;
  if (lane < ND) {
    q = bfr(qs[d] + bq);
    k = bfr(ks[d] + bk);
    v = bfr(vs[d] + bv);
  }
  __syncthreads();
  if (lane < ND) {
    qs[d] = bfr(q * scale);
    ks[d] = k;
    vs[d] = v;
    const long crow = ((long)r * Lmax + i) * C + h * HD + d;
    a.kc[crow] = (bf16)k;
    a.vc[crow] = (bf16)v;
  }
  __syncthreads();
  at.compute(qs, ks, vs, lane);
  at.publish(mxs, sms, accs, w, lane);
  __syncthreads();
  merge_heads<HD, NW>(mxs, sms, accs, os, lane);
  __syncthreads();
  wo.apply(os, a.slab + ((long)h * a.R + r) * C, w * NM, lane);
}

struct CrossHeadsArgs {
  const float* slab_in;   // [H][R][C] partial out-projections of the self-attention
  const float* x;         // residual in [R][C]
  const float* bo_in;     // self out-proj bias
  float* xo;              // residual out (written by the h = 0 blocks)
  const float* gamma;     // LN2
  const float* beta;
  float eps;
  const float* pos;       // [C] query position row
  const bf16* wq;         // cross in-projection rows 0..C (queries) [C][C]
  const float* bq;
  const bf16* k;          // memory keys / values [(R / kv_group) * Lk][C]
  const bf16* v;
  int Lk, kv_group;
  const unsigned char* kpm;   // [R / kv_group][Lk] or null
  const bf16* wo;         // cross out-proj [C][C]
  float* slab_out;        // [H][R][C]
  int R;
  bool xcd = true;        // dec_block_rh order (RETR_TUNE_DEC_ORDER)
};

template <int C, int HD, int NW, int NCH, int KU>
__global__ void __launch_bounds__(64 * NW) dec_cross_heads_kernel(CrossHeadsArgs a, float scale) {
  constexpr int H = C / HD, PER = C / 64, ND = HD / NW, NM = C / 64 / NW;
  constexpr int KPW = NCH * (64 / (HD / 8)) * KU;
  __shared__ float ts[C];
  __shared__ float qs[HD], os[HD];
  __shared__ float mxs[NW], sms[NW], accs[NW * HD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int r, h;
  dec_block_rh(blockIdx.x, a.R, H, a.xcd, r, h);
  const long RC = (long)a.R * C;
  const int kvb = r / a.kv_group, Lk = a.Lk;
  const unsigned char* km = a.kpm ? a.kpm + (long)kvb * Lk : nullptr;
  // every global load first: this wave's memory keys / values, query and out-projection weight
  // rows, the self-attention head partials and the row operands
  WaveAttn<HD, NCH, KU> at;
  at.load_mask(km, w * KPW, min(Lk, (w + 1) * KPW), lane);
  at.template load<C>(a.k, a.v, h, w * KPW, min(Lk, (w + 1) * KPW),
                      [&](int j) -> long { return (long)kvb * Lk + j; }, lane);
  ProjW<C, ND> wq;
  wq.load(a.wq, h * HD + w * ND, lane);
  OutW<C, HD, NM> wo;
  wo.load(a.wo, h, w * NM, lane);
  const float bq = lane < ND ? a.bq[h * HD + w * ND + lane] : 0.f;
  float t[PER][H], xv[PER], bo[PER], gm[PER], bt[PER], ps[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int n = lane + 64 * m;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) t[m][hh] = a.slab_in[hh * RC + (long)r * C + n];
    xv[m] = a.x[(long)r * C + n];
    bo[m] = a.bo_in[n];
    gm[m] = a.gamma[n];
    bt[m] = a.beta[n];
    ps[m] = a.pos ? a.pos[n] : 0.f;
  }
  // x' = x + (sum_h slab_in[h] + b_o), heads in order (every wave: no wait on another)
  float v[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    float s = 0.f;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) s += t[m][hh];
    v[m] = xv[m] + (s + bo[m]);
  }
  if (h == 0 && w == 0) {
#pragma unroll
    for (int m = 0; m < PER; ++m) a.xo[(long)r * C + lane + 64 * m] = v[m];
  }
  // LN2 (+ pos), bf16-rounded like the unfused path's LN output
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < PER; ++m) s += v[m];
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const float dd = v[m] - mean;
    q += dd * dd;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / C + a.eps);
  if (w == 0) {
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const float o = (v[m] - mean) * rstd * gm[m] + bt[m];
      ts[lane + 64 * m] = bfr(a.pos ? o + ps[m] : o);
    }
  }
  __syncthreads();
  bf16x8 act[C / 64];                               // bf16-rounded LN output: exact
  {
    const int c = lane & 7;
#pragma unroll
    for (int m = 0; m < C / 64; ++m) act[m] = to_bf8(ts + 8 * (c + 8 * m));
  }
  wq.dot(act, lane, qs + w * ND);
  __syncthreads();
  float qv = 0.f;
  if (lane < ND) qv = bfr(bfr(qs[w * ND + lane] + bq) * scale);
  __syncthreads();
  if (lane < ND) qs[w * ND + lane] = qv;
  __syncthreads();
  at.compute(qs, nullptr, nullptr, lane);
  at.publish(mxs, sms, accs, w, lane);
  __syncthreads();
  merge_heads<HD, NW>(mxs, sms, accs, os, lane);
  __syncthreads();
  wo.apply(os, a.slab_out + ((long)h * a.R + r) * C, w * NM, lane);
}

// ---- multi-row blocks (beam search: the K beams of an image share every weight slice and, in
// the cross sub-layer, the memory keys / values) -----------------------------------------------
// A block = RB consecutive rows x one head, two waves per row (the layout of the kernels above).
// The head's weight slices (and, with KVS, the memory K / V of the rows' image) are staged in LDS
// once per block instead of once per (row, head): at beam 5 (R = 320) the per-(row, head) blocks
// moved ~80 KB (self) / ~66 KB (cross) each through their CU, ~170 MB per launch.  C = 256,
// head dim 32.
constexpr int MR_C = 256, MR_HD = 32, MR_H = MR_C / MR_HD;
constexpr int MR_WLD = MR_C + 8;                  // staged projection rows (bank offset 16 B)
constexpr int MR_OLD = MR_HD + 8;                 // staged out-projection rows (80 B)

// rows [row0, row0 + nrows) x [col0, col0 + ncols) of a bf16 matrix (ld elements) staged into LDS
// rows of dld elements, 16-byte chunks over the block's NT threads: load() issues every chunk
// (at most N per thread) before store() writes any, so the staging costs one memory round trip
template <int N, int NT, int NCOLS>
struct Stager {
  static constexpr int CPR = NCOLS / 8;           // 16-byte chunks per row (power of two)
  static_assert((CPR & (CPR - 1)) == 0, "chunks per row");
  bf16x8 t[N];
  int total;
  RETR_DEVICE void load(const bf16* __restrict__ src, long ld, int row0, int col0, int nrows,
                        int tid) {
    total = nrows * CPR;
    const bf16* base = src + (long)row0 * ld + col0;
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int q = tid + it * NT, rr = q / CPR, cc = q % CPR;
      if (q < total) t[it] = *(const bf16x8*)(base + rr * ld + 8 * cc);
    }
  }
  RETR_DEVICE void store(bf16* dst, int dld, int tid) const {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int q = tid + it * NT, rr = q / CPR, cc = q % CPR;
      if (q < total) *(bf16x8*)(dst + rr * dld + 8 * cc) = t[it];
    }
  }
};

template <int RB>
__global__ void __launch_bounds__(128 * RB) dec_self_heads_mr_kernel(SelfHeadsArgs a, float scale) {
  constexpr int C = MR_C, HD = MR_HD, H = MR_H, NW = 2, ND = HD / NW, NM = C / 64 / NW;
  constexpr int CPL = C / 64;
  constexpr int KPW = (64 / (HD / 8)) * 4;        // keys per wave (2 x 64 = 128)
  typedef __attribute__((ext_vector_type(4))) float f4v;
  __shared__ __attribute__((aligned(16))) bf16 wi_s[3 * HD * MR_WLD];
  __shared__ __attribute__((aligned(16))) bf16 wo_s[C * MR_OLD];
  __shared__ float qs[RB][HD], ks[RB][HD], vs[RB][HD], os[RB][HD];
  __shared__ float mxs[RB][NW], sms[RB][NW], accs[RB][NW * HD];
  __shared__ __attribute__((aligned(16))) float part[RB][NW][C];
  __shared__ __attribute__((aligned(16))) bf16 lnb[RB][2][C];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, rr = wv >> 1, w = wv & 1;
  int g, h;
  dec_block_rh(blockIdx.x, a.R / RB, H, a.xcd, g, h);
  const int r = g * RB + rr;
  const int* ar = a.anc ? a.anc + (long)r * a.Lmax : nullptr;
  const int i = a.i, Lmax = a.Lmax;
  const bool pro = a.xin != nullptr;
  const int c0 = CPL * lane;
  WaveAttn<HD, 1, 4> at;
  at.set_rows(w * KPW, min(i + 1, (w + 1) * KPW),
              [&](int j) -> long {
                if (j == i) return -1;
                return (long)(ar ? ar[j] : r) * Lmax + j;
              },
              lane);
  constexpr int NT = 128 * RB;
  // the head's q | k | v rows and out-projection columns, staged once per block
  Stager<(HD * C / 8 + NT - 1) / NT, NT, C> sq, sk, sv;
  Stager<(C * HD / 8 + NT - 1) / NT, NT, HD> so;
  sq.load(a.win, C, h * HD, 0, HD, tid);
  sk.load(a.win, C, C + h * HD, 0, HD, tid);
  sv.load(a.win, C, 2 * C + h * HD, 0, HD, tid);
  so.load(a.wo, C, 0, h * HD, C, tid);
  // the row's own operands: prologue slab share, activations, cached keys / values
  float ps[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) ps[e] = 0.f;
  if (pro) {
    const long RC = (long)a.R * C;
    const int s0 = w * a.nslab / NW, s1 = (w + 1) * a.nslab / NW;
    for (int j = s0; j < s1; j += 8) {
      f4v t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        t[u] = j + u < s1 ? *(const f4v*)(a.slabs + (j + u) * RC + (long)r * C + c0)
                          : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int f = 0; f < 4; ++f)
          if (j + u < s1) ps[f] += t[u][f];
    }
  }
  bf16x8 actp[C / 64], actn[C / 64];
  if (!pro) {
    load_act<C>(a.npos + (long)r * C, lane, actp);
    load_act<C>(a.n + (long)r * C, lane, actn);
  }
  at.template load_rows<C>(a.kc, a.vc, h, lane);
  const int d = w * ND + lane;
  const float bq = lane < ND ? a.bin[h * HD + d] : 0.f;
  const float bk = lane < ND ? a.bin[C + h * HD + d] : 0.f;
  const float bv = lane < ND ? a.bin[2 * C + h * HD + d] : 0.f;
  sq.store(wi_s, MR_WLD, tid);
  sk.store(wi_s + HD * MR_WLD, MR_WLD, tid);
  sv.store(wi_s + 2 * HD * MR_WLD, MR_WLD, tid);
  so.store(wo_s, MR_OLD, tid);
  if (pro) {
    float xv[CPL], b2[CPL], gm[CPL], bt[CPL], qp[CPL];
    *(f4v*)xv = *(const f4v*)(a.xin + (long)r * C + c0);
    *(f4v*)b2 = *(const f4v*)(a.b2 + c0);
    *(f4v*)gm = *(const f4v*)(a.gamma + c0);
    *(f4v*)bt = *(const f4v*)(a.beta + c0);
    *(f4v*)qp = *(const f4v*)(a.qpos + c0);
#pragma unroll
    for (int e = 0; e < CPL; ++e) part[rr][w][c0 + e] = ps[e];
    __syncthreads();
    float v[CPL], sm = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      v[e] = xv[e] + ((part[rr][0][c0 + e] + part[rr][1][c0 + e]) + b2[e]);
      sm += v[e];
    }
    if (h == 0 && w == 0) *(f4v*)(a.xout + (long)r * C + c0) = *(f4v*)v;
    const float mean = wave_sum(sm) / C;
    float q2 = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const float dd = v[e] - mean;
      q2 += dd * dd;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q2) / C + a.eps);
    if (w == 0) {
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        const float o = (v[e] - mean) * rstd * gm[e] + bt[e];
        lnb[rr][0][c0 + e] = (bf16)o;
        lnb[rr][1][c0 + e] = (bf16)(o + qp[e]);
      }
    }
  }
  __syncthreads();                                   // staged weights (and LN1) visible
  if (pro) {
    const int c = lane & 7;
#pragma unroll
    for (int m = 0; m < C / 64; ++m) {
      actn[m] = *(const bf16x8*)(&lnb[rr][0][8 * (c + 8 * m)]);
      actp[m] = *(const bf16x8*)(&lnb[rr][1][8 * (c + 8 * m)]);
    }
  }
  {
    ProjW<C, ND> pw;                                 // one slice at a time (LDS reads are cheap)
    pw.load(wi_s, w * ND, lane, MR_WLD);
    pw.dot(actp, lane, qs[rr] + w * ND);
    pw.load(wi_s + HD * MR_WLD, w * ND, lane, MR_WLD);
    pw.dot(actp, lane, ks[rr] + w * ND);
    pw.load(wi_s + 2 * HD * MR_WLD, w * ND, lane, MR_WLD);
    pw.dot(actn, lane, vs[rr] + w * ND);
  }
  __syncthreads();
  float q = 0.f, k = 0.f, v = 0.f;
  if (lane < ND) {
    q = bfr(qs[rr][d] + bq);
    k = bfr(ks[rr][d] + bk);
    v = bfr(vs[rr][d] + bv);
  }
  __syncthreads();
  if (lane < ND) {
    qs[rr][d] = bfr(q * scale);
    ks[rr][d] = k;
    vs[rr][d] = v;
    const long crow = ((long)r * Lmax + i) * C + h * HD + d;
    a.kc[crow] = (bf16)k;
    a.vc[crow] = (bf16)v;
  }
  __syncthreads();
  at.compute(qs[rr], ks[rr], vs[rr], lane);
  at.publish(mxs[rr], sms[rr], accs[rr], w, lane);
  __syncthreads();
  merge_heads<HD, NW>(mxs[rr], sms[rr], accs[rr], os[rr], lane);
  __syncthreads();
  OutW<C, HD, NM> wo;
  wo.load(wo_s, 0, w * NM, lane, MR_OLD);
  wo.apply(os[rr], a.slab + ((long)h * a.R + r) * C, w * NM, lane);
}

// KVS: the block's rows read the same memory rows (beam: kv_group a multiple of RB), whose keys /
// values for this head are staged in LDS once (Lk <= 256)
template <int RB, bool KVS>
__global__ void __launch_bounds__(128 * RB) dec_cross_heads_mr_kernel(CrossHeadsArgs a, float scale) {
  constexpr int C = MR_C, HD = MR_HD, H = MR_H, PER = C / 64, NW = 2, ND = HD / NW, NM = C / 64 / NW;
  constexpr int KPW = (64 / (HD / 8)) * 8;        // keys per wave (2 x 128 = 256)
  constexpr int KMAX = 2 * KPW;
  __shared__ __attribute__((aligned(16))) bf16 wq_s[HD * MR_WLD];
  __shared__ __attribute__((aligned(16))) bf16 wo_s[C * MR_OLD];
  __shared__ __attribute__((aligned(16))) bf16 k_s[KVS ? KMAX * HD : 8];
  __shared__ __attribute__((aligned(16))) bf16 v_s[KVS ? KMAX * HD : 8];
  __shared__ float ts[RB][C];
  __shared__ float qs[RB][HD], os[RB][HD];
  __shared__ float mxs[RB][NW], sms[RB][NW], accs[RB][NW * HD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, rr = wv >> 1, w = wv & 1;
  int g, h;
  dec_block_rh(blockIdx.x, a.R / RB, H, a.xcd, g, h);
  const int r = g * RB + rr;
  const long RC = (long)a.R * C;
  const int kvb = r / a.kv_group, Lk = a.Lk;
  const unsigned char* km = a.kpm ? a.kpm + (long)kvb * Lk : nullptr;
  constexpr int NT = 128 * RB;
  Stager<(HD * C / 8 + NT - 1) / NT, NT, C> sq;
  Stager<(C * HD / 8 + NT - 1) / NT, NT, HD> so;
  Stager<KVS ? (KMAX * HD / 8 + NT - 1) / NT : 1, NT, HD> skk, svv;
  sq.load(a.wq, C, h * HD, 0, HD, tid);
  so.load(a.wo, C, 0, h * HD, C, tid);
  if constexpr (KVS) {
    skk.load(a.k, C, kvb * Lk, h * HD, Lk, tid);
    svv.load(a.v, C, kvb * Lk, h * HD, Lk, tid);
  }
  WaveAttn<HD, 1, 8> at;
  at.load_mask(km, w * KPW, min(Lk, (w + 1) * KPW), lane);
  if constexpr (!KVS)
    at.template load<C>(a.k, a.v, h, w * KPW, min(Lk, (w + 1) * KPW),
                        [&](int j) -> long { return (long)kvb * Lk + j; }, lane);
  const float bq = lane < ND ? a.bq[h * HD + w * ND + lane] : 0.f;
  float t[PER][H], xv[PER], bo[PER], gm[PER], bt[PER], ps[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int n = lane + 64 * m;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) t[m][hh] = a.slab_in[hh * RC + (long)r * C + n];
    xv[m] = a.x[(long)r * C + n];
    bo[m] = a.bo_in[n];
    gm[m] = a.gamma[n];
    bt[m] = a.beta[n];
    ps[m] = a.pos ? a.pos[n] : 0.f;
  }
  sq.store(wq_s, MR_WLD, tid);
  so.store(wo_s, MR_OLD, tid);
  if constexpr (KVS) {
    skk.store(k_s, HD, tid);
    svv.store(v_s, HD, tid);
  }
  float v[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    float s = 0.f;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) s += t[m][hh];
    v[m] = xv[m] + (s + bo[m]);
  }
  if (h == 0 && w == 0) {
#pragma unroll
    for (int m = 0; m < PER; ++m) a.xo[(long)r * C + lane + 64 * m] = v[m];
  }
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < PER; ++m) s += v[m];
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const float dd = v[m] - mean;
    q += dd * dd;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / C + a.eps);
  if (w == 0) {
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const float o = (v[m] - mean) * rstd * gm[m] + bt[m];
      ts[rr][lane + 64 * m] = bfr(a.pos ? o + ps[m] : o);
    }
  }
  __syncthreads();                                   // staged slices + LN2 rows visible

  bf16x8 act[C / 64];
  {
    const int c = lane & 7;
#pragma unroll
    for (int m = 0; m < C / 64; ++m) act[m] = to_bf8(ts[rr] + 8 * (c + 8 * m));
  }
  {
    ProjW<C, ND> wq;
    wq.load(wq_s, w * ND, lane, MR_WLD);
    wq.dot(act, lane, qs[rr] + w * ND);
  }
  __syncthreads();
  float qv = 0.f;
  if (lane < ND) qv = bfr(bfr(qs[rr][w * ND + lane] + bq) * scale);
  __syncthreads();
  if (lane < ND) qs[rr][w * ND + lane] = qv;
  __syncthreads();
  if constexpr (KVS)
    at.compute_lds(qs[rr], k_s, v_s, w * KPW, min(Lk, (w + 1) * KPW), lane);
  else
    at.compute(qs[rr], nullptr, nullptr, lane);
  at.publish(mxs[rr], sms[rr], accs[rr], w, lane);
  __syncthreads();
  merge_heads<HD, NW>(mxs[rr], sms[rr], accs[rr], os[rr], lane);
  __syncthreads();
  OutW<C, HD, NM> wo;
  wo.load(wo_s, 0, w * NM, lane, MR_OLD);
  wo.apply(os[rr], a.slab_out + ((long)h * a.R + r) * C, w * NM, lane);
}

}  // namespace

extern "C" {

int retr_dec_self_heads(const void* n, const void* npos, int R, int C, int H, const void* win,
                        const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                        const void* wo, float* slab, void* stream) {
  return retr_dec_self_heads_ln(n, npos, R, C, H, win, bin, kc, vc, i, Lmax, anc, wo, slab,
                                nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0.f, nullptr,
                                nullptr, stream);
}

int retr_dec_self_heads_ln(const void* n, const void* npos, int R, int C, int H, const void* win,
                           const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                           const void* wo, float* slab, const float* xin, const float* slabs,
                           int nslab, const float* b2, const float* gamma, const float* beta,
                           float eps, const float* qpos, float* xout, void* stream) {
  RETR_REQUIRE(xin == nullptr || (slabs && b2 && gamma && beta && qpos && xout && nslab >= 0),
               "dec_self_heads_ln: incomplete LayerNorm prologue operands");
  const int hd = H > 0 ? C / H : 0;
  RETR_REQUIRE((C == 256 || C == 512) && (hd == 32 || hd == 64) && hd * H == C,
               "dec_self_heads: C=%d H=%d unsupported", C, H);
  RETR_REQUIRE(i >= 0 && i < Lmax, "dec_self_heads: step %d outside the %d-row cache", i, Lmax);
  if (R == 0) return 0;
  SelfHeadsArgs a{(const bf16*)n, (const bf16*)npos, (const bf16*)win, bin, (bf16*)kc,
                  (bf16*)vc, i, Lmax, anc, (const bf16*)wo, slab, R, xin, slabs, nslab, b2,
                  gamma, beta, eps, qpos, xout};
  a.xcd = retr_tune_get(RETR_TUNE_DEC_ORDER) == 0;
  const float scale = 1.0f / sqrtf((float)hd);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R * H));
  // two waves per (row, head) for up to 128 / 64 keys (hd 32 / 64), else one wave with every
  // key / value load of up to 4 chunks in flight
  const int np = 64 / (hd / 8), nk = i + 1;
#define SH(CV, HDV, NW, NC, KU) \
  hipLaunchKernelGGL((dec_self_heads_kernel<CV, HDV, NW, NC, KU>), grid, dim3(64 * NW), 0, st, a, scale)
#define SH_N(CV, HDV)                                           \
  if (nk <= 2 * np * 4) SH(CV, HDV, 2, 1, 4);                    \
  else if (nk <= np * 8) SH(CV, HDV, 1, 1, 8);                   \
  else if (nk <= 2 * np * 8) SH(CV, HDV, 1, 2, 8);               \
  else SH(CV, HDV, 1, 4, 8);
  RETR_REQUIRE(nk <= 4 * np * 8, "dec_self_heads: %d keys (at most %d)", nk, 4 * np * 8);
  if (C == 256 && hd == 32 && nk <= 128 && retr_tune_get(RETR_TUNE_DEC_WAVES) != 1)
    SH(256, 32, 4, 1, 2);
  else if (C == 256 && hd == 32) { SH_N(256, 32) }
  else if (C == 256) { SH_N(256, 64) }
  else if (hd == 32) { SH_N(512, 32) }
  else { SH_N(512, 64) }
#undef SH_N
#undef SH
  return retr_check_launch("dec_self_heads");
}

int retr_dec_self_heads_embed(const long long* tok, const float* word, const float* ge,
                              const float* be, float epse, int R, int C, int H, const void* win,
                              const float* bin, void* kc, void* vc, int i, int Lmax,
                              const int* anc, const void* wo, float* slab, const float* gamma,
                              const float* beta, float eps, const float* qpos, float* xout,
                              void* stream) {
  RETR_REQUIRE(tok && word && ge && be && gamma && beta && qpos && xout,
               "dec_self_heads_embed: missing operands");
  const int hd = H > 0 ? C / H : 0;
  RETR_REQUIRE((C == 256 || C == 512) && hd == 32 && hd * H == C,
               "dec_self_heads_embed: C=%d H=%d unsupported", C, H);
  RETR_REQUIRE(i >= 0 && i < Lmax && i + 1 <= 128,
               "dec_self_heads_embed: step %d (cache %d rows, at most 128 keys)", i, Lmax);
  if (R == 0) return 0;
  SelfHeadsArgs a{nullptr, nullptr, (const bf16*)win, bin, (bf16*)kc, (bf16*)vc, i, Lmax, anc,
                  (const bf16*)wo, slab, R, nullptr, nullptr, 0, nullptr, gamma, beta, eps, qpos,
                  xout};
  a.xcd = retr_tune_get(RETR_TUNE_DEC_ORDER) == 0;
  a.tok = tok;
  a.word = word;
  a.ge = ge;
  a.be = be;
  a.epse = epse;
  const float scale = 1.0f / sqrtf((float)hd);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R * H));
  if (C == 256)
    hipLaunchKernelGGL((dec_self_heads_kernel<256, 32, 2, 1, 4>), grid, dim3(128), 0, st, a, scale);
  else
    hipLaunchKernelGGL((dec_self_heads_kernel<512, 32, 2, 1, 4>), grid, dim3(128), 0, st, a, scale);
  return retr_check_launch("dec_self_heads_embed");
}

int retr_dec_cross_heads(const float* slab_in, const float* x, const float* bo_in, float* xo,
                         int R, int C, int H, const float* gamma, const float* beta, float eps,
                         const float* pos, const void* wq, const float* bq, const void* k,
                         const void* v, int Lk, int kv_group, const unsigned char* kpm,
                         const void* wo, float* slab_out, void* stream) {
  const int hd = H > 0 ? C / H : 0;
  RETR_REQUIRE((C == 256 || C == 512) && (hd == 32 || hd == 64) && hd * H == C,
               "dec_cross_heads: C=%d H=%d unsupported", C, H);
  RETR_REQUIRE(Lk > 0 && kv_group > 0, "dec_cross_heads: Lk=%d kv_group=%d", Lk, kv_group);
  if (R == 0) return 0;
  CrossHeadsArgs a{slab_in, x, bo_in, xo, gamma, beta, eps, pos, (const bf16*)wq, bq,
                   (const bf16*)k, (const bf16*)v, Lk, kv_group, kpm, (const bf16*)wo, slab_out, R};
  a.xcd = retr_tune_get(RETR_TUNE_DEC_ORDER) == 0;
  const float scale = 1.0f / sqrtf((float)hd);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R * H));
  // two waves per (row, head), each over up to 2 chunks of 8 keys per lane part
  const int np = 64 / (hd / 8), per = np * 8;
#define XH(CV, HDV, NC) \
  hipLaunchKernelGGL((dec_cross_heads_kernel<CV, HDV, 2, NC, 8>), grid, dim3(128), 0, st, a, scale)
#define XH_N(CV, HDV) \
  if (Lk <= 2 * per) XH(CV, HDV, 1); else XH(CV, HDV, 2);
  RETR_REQUIRE(Lk <= 4 * per, "dec_cross_heads: %d memory keys (at most %d)", Lk, 4 * per);
  if (C == 256 && hd == 32 && Lk <= 256 && retr_tune_get(RETR_TUNE_DEC_WAVES) != 1)
    hipLaunchKernelGGL((dec_cross_heads_kernel<256, 32, 4, 1, 4>), grid, dim3(256), 0, st, a, scale);
  else if (C == 256 && hd == 32) { XH_N(256, 32) }
  else if (C == 256) { XH_N(256, 64) }
  else if (hd == 32) { XH_N(512, 32) }
  else { XH_N(512, 64) }
#undef XH_N
#undef XH
  return retr_check_launch("dec_cross_heads");
}

// Multi-row blocks (rb rows x one head, 128 rb threads): the head's weight slices are staged in
// LDS once per block, and the memory keys / values too when the block's rows share an image
// (kv_group % rb == 0).  C = 256, head dim 32, rb in {2, 4, 5}, R % rb == 0, at most 128 self /
// 256 memory keys; other shapes take the per-(row, head) kernels above (rb = 1).
int retr_dec_self_heads_mr(const void* n, const void* npos, int R, int C, int H, const void* win,
                           const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                           const void* wo, float* slab, const float* xin, const float* slabs,
                           int nslab, const float* b2, const float* gamma, const float* beta,
                           float eps, const float* qpos, float* xout, int rb, void* stream) {
  if (rb == 1)
    return retr_dec_self_heads_ln(n, npos, R, C, H, win, bin, kc, vc, i, Lmax, anc, wo, slab, xin,
                                  slabs, nslab, b2, gamma, beta, eps, qpos, xout, stream);
  RETR_REQUIRE(xin == nullptr || (slabs && b2 && gamma && beta && qpos && xout && nslab >= 0),
               "dec_self_heads_mr: incomplete LayerNorm prologue operands");
  RETR_REQUIRE(C == MR_C && H == MR_H, "dec_self_heads_mr: C=%d H=%d (needs C=256, H=8)", C, H);
  RETR_REQUIRE(rb == 2 || rb == 4 || rb == 5, "dec_self_heads_mr: rb=%d", rb);
  RETR_REQUIRE(R % rb == 0, "dec_self_heads_mr: R=%d not a multiple of rb=%d", R, rb);
  RETR_REQUIRE(i >= 0 && i < Lmax, "dec_self_heads_mr: step %d outside the %d-row cache", i, Lmax);
  RETR_REQUIRE(i + 1 <= 128, "dec_self_heads_mr: %d keys (at most 128)", i + 1);
  if (R == 0) return 0;
  SelfHeadsArgs a{(const bf16*)n, (const bf16*)npos, (const bf16*)win, bin, (bf16*)kc,
                  (bf16*)vc, i, Lmax, anc, (const bf16*)wo, slab, R, xin, slabs, nslab, b2,
                  gamma, beta, eps, qpos, xout};
  a.xcd = retr_tune_get(RETR_TUNE_DEC_ORDER) == 0;
  const float scale = 1.0f / sqrtf((float)MR_HD);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R / rb * H));
#define SM(RBV) hipLaunchKernelGGL((dec_self_heads_mr_kernel<RBV>), grid, dim3(128 * RBV), 0, st, a, scale)
  if (rb == 2) SM(2);
  else if (rb == 4) SM(4);
  else SM(5);
#undef SM
  return retr_check_launch("dec_self_heads_mr");
}

int retr_dec_cross_heads_mr(const float* slab_in, const float* x, const float* bo_in, float* xo,
                            int R, int C, int H, const float* gamma, const float* beta, float eps,
                            const float* pos, const void* wq, const float* bq, const void* k,
                            const void* v, int Lk, int kv_group, const unsigned char* kpm,
                            const void* wo, float* slab_out, int rb, void* stream) {
  if (rb == 1)
    return retr_dec_cross_heads(slab_in, x, bo_in, xo, R, C, H, gamma, beta, eps, pos, wq, bq, k,
                                v, Lk, kv_group, kpm, wo, slab_out, stream);
  RETR_REQUIRE(C == MR_C && H == MR_H, "dec_cross_heads_mr: C=%d H=%d (needs C=256, H=8)", C, H);
  RETR_REQUIRE(rb == 2 || rb == 4 || rb == 5, "dec_cross_heads_mr: rb=%d", rb);
  RETR_REQUIRE(R % rb == 0, "dec_cross_heads_mr: R=%d not a multiple of rb=%d", R, rb);
  RETR_REQUIRE(Lk > 0 && Lk <= 256 && kv_group > 0,
               "dec_cross_heads_mr: Lk=%d (1..256) kv_group=%d", Lk, kv_group);
  if (R == 0) return 0;
  CrossHeadsArgs a{slab_in, x, bo_in, xo, gamma, beta, eps, pos, (const bf16*)wq, bq,
                   (const bf16*)k, (const bf16*)v, Lk, kv_group, kpm, (const bf16*)wo, slab_out, R};
  a.xcd = retr_tune_get(RETR_TUNE_DEC_ORDER) == 0;
  const float scale = 1.0f / sqrtf((float)MR_HD);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R / rb * H));
  const bool kvs = kv_group % rb == 0;
#define XM(RBV)                                                                                   \
  if (kvs) hipLaunchKernelGGL((dec_cross_heads_mr_kernel<RBV, true>), grid, dim3(128 * RBV), 0, st, \
                              a, scale);                                                          \
  else hipLaunchKernelGGL((dec_cross_heads_mr_kernel<RBV, false>), grid, dim3(128 * RBV), 0, st, a, \
                          scale);
  if (rb == 2) { XM(2) }
  else if (rb == 4) { XM(4) }
  else { XM(5) }
#undef XM
  return retr_check_launch("dec_cross_heads_mr");
}

}  // extern "C"
