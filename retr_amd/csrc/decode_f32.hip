// Fused incremental decode step of the fp32 parity mode (round 6).
//
// config.dtype = 'fp32' is the mode whose greedy ids equal the reference algorithm's
// (eval_utils/decode.py:53-81; tests/test_gpu_configs.py checks them against the CPU oracle).
// Until round 5 it ran the per-op step: LayerNorm, q | k | v, attention, out-projection, FFN1 and
// FFN2 of every sub-layer as separate launches on the skinny exact-f32 linear -- ~70 launches and
// 0.65 ms per step at B = 64 (profiles/r5_bench_final.json decode.fp32).  These kernels give it
// the bf16 step's structure (csrc/decode_heads.hip, dec_ffn_ln in csrc/decode.hip): THREE launches
// per decoder layer (models/transformer_modules.py:22-97 pre-norm, ConcatTransformer.py:187-214),
//
//   dec_self_f32   block = (query row r, head h), 8 waves: the previous layer's FFN partial slabs
//                  + residual + b2 (layer 0: the token's word embedding + query position and the
//                  embedding LayerNorm, DecoderEmbeddings) and LN1 (+ query position) in the
//                  prologue; the head's q | k | v rows, k / v appended to the fp32 cache; attention
//                  over keys 0..i (beam ancestry); the head's PARTIAL out-projection o_h Wo[:, h]^T
//                  into slab[h][r] (fp32)
//   dec_cross_f32  block = (r, h): x' = x + (sum_h slab[h][r] + b_o) (heads in order), LN2 + query
//                  position, the head's cross query, attention over the image memory (key-padding
//                  mask), partial out-projection into slab2[h][r]
//   dec_ffn_f32    block = 16 rows x 64 hidden units, 16 waves: x'' = x' + (sum_h slab2[h] + b_o)
//                  and LN3 of the block's rows, FFN1 + ReLU + FFN2 on exact-f32 16x16x4 MFMA ->
//                  fp32 partial slabs [F / 64][R][C] (the next layer's dec_self_f32 prologue, or
//                  dec_rows_f32 before the MLP head, sums them in slab order)
//
// Every value stays fp32 (no operand rounding anywhere): dot products are fp32 FMA chains and
// DPP lane-group sums, MFMAs are the exact-f32 form, so the step differs from the per-op fp32
// step only in summation order (~1e-6 relative) -- what parity needs; ids are checked equal to
// the CPU oracle's (tests/test_gpu_decode_f32.py).  Shape: d_model 256, 8 heads of 32 (the cfg2 /
// cfg5 decoder); other shapes keep the per-op step (eval_utils/decode.py _fusable_f32).
// Every global load of a wave is issued before its first arithmetic (one dependent memory round
// trip per launch, the rule of the bf16 kernels: these launches are latency-bound at B = 64).
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int FC = 256, FHD = 32, FH = FC / FHD, FNW = 8;

template <int CTRL>
RETR_DEVICE float fdpp(float s) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s),
                                                               CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of G lanes (4, 8 or 16): quad xor 1, quad xor 2, half-row mirror,
// row mirror; every lane of a group ends with the group's sum
template <int G>
RETR_DEVICE float fgsum(float s) {
  static_assert(G == 4 || G == 8 || G == 16, "group of 4, 8 or 16 lanes");
  s += fdpp<0xB1>(s);
  s += fdpp<0x4E>(s);
  if constexpr (G >= 8) s += fdpp<0x141>(s);
  if constexpr (G >= 16) s += fdpp<0x140>(s);
  return s;
}

RETR_DEVICE float fdot4(const f4& a, const f4& b, float s) {
  s = fmaf(a[0], b[0], s);
  s = fmaf(a[1], b[1], s);
  s = fmaf(a[2], b[2], s);
  return fmaf(a[3], b[3], s);
}

// (row, head) of block b: the eight head blocks of a row on one XCD (hardware puts block b on
// XCD b % 8), as csrc/decode_heads.hip's dec_block_rh
RETR_DEVICE void f32_block_rh(int b, int R, bool xcd, int& r, int& h) {
  if ((R & 7) == 0 && xcd) {
    const int x = b & 7, q = b >> 3;
    r = x * (R >> 3) + q / FH;
    h = q % FH;
  } else {
    r = b / FH;
    h = b % FH;
  }
}

// Four rows [row0, row0 + 4) of a [.][256] fp32 matrix per wave: lane (row rg = lane >> 4,
// column c = lane & 15) holds the row's 16-byte chunks c, c + 16, c + 32, c + 48.
struct ProjF {
  f4 w[4];
  RETR_DEVICE void load(const float* __restrict__ W, int row0, int lane) {
    const float* p = W + (long)(row0 + (lane >> 4)) * FC + 4 * (lane & 15);
#pragma unroll
    for (int m = 0; m < 4; ++m) w[m] = *(const f4*)(p + 64 * m);
  }
  // out[rg] = W[row0 + rg] . act (two FMA chains, then the 16-lane group sum)
  RETR_DEVICE void dot(const f4 (&act)[4], int lane, float* out) const {
    float s0 = fdot4(w[0], act[0], 0.f), s1 = fdot4(w[1], act[1], 0.f);
    s0 = fdot4(w[2], act[2], s0);
    s1 = fdot4(w[3], act[3], s1);
    const float s = fgsum<16>(s0 + s1);
    if ((lane & 15) == 0) out[lane >> 4] = s;
  }
};
// this lane's activation chunks (ProjF layout) of a 256-float row in LDS
RETR_DEVICE void load_actf(const float* row, int lane, f4 (&act)[4]) {
#pragma unroll
  for (int m = 0; m < 4; ++m) act[m] = *(const f4*)(row + 4 * ((lane & 15) + 16 * m));
}

// Out-projection rows n = 32 w + (lane & 31) of wave w, the head's 32 columns split in halves
// over lanes < 32 / >= 32: slab[n] = sum_{d < 32} o[d] Wo[n][32 h + d]
struct OutF {
  f4 w[4];
  RETR_DEVICE void load(const float* __restrict__ Wo, int h, int wv, int lane) {
    const float* p = Wo + (long)(32 * wv + (lane & 31)) * FC + FHD * h + 16 * (lane >> 5);
#pragma unroll
    for (int t = 0; t < 4; ++t) w[t] = *(const f4*)(p + 4 * t);
  }
  RETR_DEVICE void apply(const float* os, float* slab, int wv, int lane) const {
    const float* o = os + 16 * (lane >> 5);
    float s0 = fdot4(w[0], *(const f4*)o, 0.f), s1 = fdot4(w[1], *(const f4*)(o + 4), 0.f);
    s0 = fdot4(w[2], *(const f4*)(o + 8), s0);
    s1 = fdot4(w[3], *(const f4*)(o + 12), s1);
    float s = s0 + s1;
    s += xor_lane(s, 32);
    if (lane < 32) slab[32 * wv + lane] = s;
  }
};

// Attention of one wave over its keys [j0, j1) (at most 16 KU): lane = (dim group g = lane & 3
// of 8 dims, key part p = lane >> 2), key j = j0 + p + 16 u.  key_row(j) gives the K / V row of
// key j, -1 for the step's own key (k / v in LDS) or -2 for none.
template <int KU>
struct AttnF {
  long row[KU];
  f4 k[KU][2], v[KU][2];
  bool mk[KU];
  float mx = -INFINITY, sum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  template <class RowFn>
  RETR_DEVICE void set_rows(int j0, int j1, RowFn key_row, int lane) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int j = j0 + (lane >> 2) + 16 * u;
      row[u] = j < j1 ? key_row(j) : -2;
      mk[u] = false;
    }
  }
  // key-padding flags, loaded independently of (and before) the keys / values
  RETR_DEVICE void load_mask(const unsigned char* km, int j0, int j1, int lane) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int j = j0 + (lane >> 2) + 16 * u;
      mk[u] = km != nullptr && j < j1 && km[j] != 0;
    }
  }
  RETR_DEVICE void load_rows(const float* __restrict__ K, const float* __restrict__ V, int h,
                             int lane) {
    const int off = FHD * h + 8 * (lane & 3);
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const bool ok = row[u] >= 0;
      const float* kp = K + row[u] * FC + off;
      const float* vp = V + row[u] * FC + off;
      k[u][0] = ok ? *(const f4*)kp : f4{0.f, 0.f, 0.f, 0.f};
      k[u][1] = ok ? *(const f4*)(kp + 4) : f4{0.f, 0.f, 0.f, 0.f};
      v[u][0] = ok ? *(const f4*)vp : f4{0.f, 0.f, 0.f, 0.f};
      v[u][1] = ok ? *(const f4*)(vp + 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // q (scaled), and the own key / value (kn, vn: null when there is none), in LDS
  RETR_DEVICE void compute(const float* qs, const float* kn, const float* vn, int lane) {
    const int g = lane & 3;
    const f4 q0 = *(const f4*)(qs + 8 * g), q1 = *(const f4*)(qs + 8 * g + 4);
    f4 kn0{0.f, 0.f, 0.f, 0.f}, kn1{0.f, 0.f, 0.f, 0.f}, vn0{0.f, 0.f, 0.f, 0.f},
        vn1{0.f, 0.f, 0.f, 0.f};
    if (kn) {
      kn0 = *(const f4*)(kn + 8 * g);
      kn1 = *(const f4*)(kn + 8 * g + 4);
      vn0 = *(const f4*)(vn + 8 * g);
      vn1 = *(const f4*)(vn + 8 * g + 4);
    }
    float sc[KU];
    float cm = -INFINITY;
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const bool own = row[u] == -1;
      const float s = fgsum<4>(fdot4(q0, own ? kn0 : k[u][0], 0.f) +
                               fdot4(q1, own ? kn1 : k[u][1], 0.f));
      sc[u] = (row[u] == -2 || mk[u]) ? -INFINITY : s;
      cm = fmaxf(cm, sc[u]);
    }
    cm = wave_max(cm);
    if (cm == -INFINITY) return;                 // no (unmasked) key in this wave
    mx = cm;
    float cs = 0.f;
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const float p = sc[u] == -INFINITY ? 0.f : __expf(sc[u] - cm);
      cs += p;                                   // four copies of every key: divided out below
      const bool own = row[u] == -1;
      const f4 a0 = own ? vn0 : v[u][0], a1 = own ? vn1 : v[u][1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] = fmaf(p, a0[e], acc[e]);
        acc[4 + e] = fmaf(p, a1[e], acc[4 + e]);
      }
    }
    sum = wave_sum(cs) * 0.25f;
  }
  // (max, sum, unnormalised P V over the wave's keys) into LDS slot w
  RETR_DEVICE void publish(float* mxs, float* sms, float* accs, int w, int lane) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) acc[e] += xor_lane(acc[e], o);
    if (lane == 0) {
      mxs[w] = mx;
      sms[w] = sum;
    }
    if (lane < 4) {
#pragma unroll
      for (int e = 0; e < 8; ++e) accs[w * FHD + 8 * lane + e] = acc[e];
    }
  }
};

// o[d] (normalised) from the FNW waves' partial softmax states, lanes d < 32 of one wave
RETR_DEVICE void merge_f32(const float* mxs, const float* sms, const float* accs, float* os,
                           int lane) {
  if (lane >= FHD) return;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < FNW; ++w) M = fmaxf(M, mxs[w]);
  float num = 0.f, den = 0.f;
#pragma unroll
  for (int w = 0; w < FNW; ++w) {
    const float f = mxs[w] == -INFINITY ? 0.f : __expf(mxs[w] - M);
    num = fmaf(accs[w * FHD + lane], f, num);
    den = fmaf(sms[w], f, den);
  }
  os[lane] = num / den;                          // a fully masked row gives NaN, as torch
}

// LayerNorm of the 256-float row v (4 consecutive columns per lane, the whole wave)
RETR_DEVICE void ln_row(const f4& v, const f4& gm, const f4& bt, float eps, f4& out) {
  const float mean = wave_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / FC);
  f4 d;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    d[e] = v[e] - mean;
    q = fmaf(d[e], d[e], q);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / FC) + eps);
#pragma unroll
  for (int e = 0; e < 4; ++e) out[e] = d[e] * rstd * gm[e] + bt[e];
}

struct SelfF32Args {
  const float* win;      // [3C][C] in-projection
  const float* bin;      // [3C]
  float* kc;             // caches [R * Lmax][C] (fp32)
  float* vc;
  int i, Lmax;           // this step's position (keys 0..i), cache rows per row
  const int* anc;        // [R][Lmax] beam ancestry or null
  const float* wo;       // [C][C] out-projection
  float* slab;           // [H][R][C] per-head partial out-projections
  int R;
  // prologue, one of: x = xin + (sum_j slabs[j] + b2) (the previous layer's FFN partials
  // [nslab][R][C]), or (tok != null, layer 0) x = LN_e(word[tok] + qpos)
  const float* xin;
  const float* slabs;
  int nslab;
  const float* b2;
  const long long* tok;
  const float* word;     // [V][C]
  const float* ge;       // embedding LayerNorm
  const float* be;
  float epse;
  const float* gamma;    // LN1
  const float* beta;
  float eps;
  const float* qpos;     // [C] query position row of step i
  float* xout;           // x (written by the h = 0 blocks)
  bool xcd;
};

template <int KU>
__global__ void __launch_bounds__(64 * FNW, KU <= 2 ? 4 : 2) dec_self_f32_kernel(SelfF32Args a, float scale) {
  constexpr int KPW = 16 * KU;
  __shared__ __attribute__((aligned(16))) float lnf[2][FC];     // LN1(x), LN1(x) + qpos
  __shared__ __attribute__((aligned(16))) float part[FNW][FC];  // slab partial sums per wave
  __shared__ __attribute__((aligned(16))) float qs[FHD], ks[FHD], vs[FHD], os[FHD];
  __shared__ float mxs[FNW], sms[FNW];
  __shared__ __attribute__((aligned(16))) float accs[FNW * FHD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int r, h;
  f32_block_rh(blockIdx.x, a.R, a.xcd, r, h);
  const int i = a.i, Lmax = a.Lmax;
  const int* ar = a.anc ? a.anc + (long)r * Lmax : nullptr;
  AttnF<KU> at;
  at.set_rows(w * KPW, min(i + 1, (w + 1) * KPW),
              [&](int j) -> long {
                if (j == i) return -1;
                return (long)(ar ? ar[j] : r) * Lmax + j;
              },
              lane);
  // every global load first: the prologue's row operands (this wave's slab share), the wave's
  // q | k | v and out-projection weight rows, its cached keys / values of positions < i
  const int c0 = 4 * lane;
  const bool emb = a.tok != nullptr;
  f4 ps{0.f, 0.f, 0.f, 0.f};
  if (emb) {
    ps = *(const f4*)(a.word + a.tok[r] * FC + c0);
  } else {
    const long RC = (long)a.R * FC;
    const int s0 = w * a.nslab / FNW, s1 = (w + 1) * a.nslab / FNW;
    for (int j = s0; j < s1; j += 4) {
      f4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        t[u] = j + u < s1 ? *(const f4*)(a.slabs + (j + u) * RC + (long)r * FC + c0)
                          : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j + u < s1) ps += t[u];
    }
  }
  ProjF wq, wk, wv;
  wq.load(a.win, FHD * h + 4 * w, lane);
  wk.load(a.win, FC + FHD * h + 4 * w, lane);
  wv.load(a.win, 2 * FC + FHD * h + 4 * w, lane);
  at.load_rows(a.kc, a.vc, h, lane);
  OutF wo;
  wo.load(a.wo, h, w, lane);
  const float bq = lane < FHD ? a.bin[FHD * h + lane] : 0.f;
  const float bk = lane < FHD ? a.bin[FC + FHD * h + lane] : 0.f;
  const float bv = lane < FHD ? a.bin[2 * FC + FHD * h + lane] : 0.f;
  const f4 xv = emb ? *(const f4*)(a.ge + c0) : *(const f4*)(a.xin + (long)r * FC + c0);
  const f4 b2 = emb ? *(const f4*)(a.be + c0) : *(const f4*)(a.b2 + c0);
  const f4 gm = *(const f4*)(a.gamma + c0);
  const f4 bt = *(const f4*)(a.beta + c0);
  const f4 qp = *(const f4*)(a.qpos + c0);

  // x: the embedding (LN_e(word + qpos)), or xin + (slab partials in wave order + b2)
  f4 x;
  if (emb) {
    ln_row(ps + qp, xv, b2, a.epse, x);
  } else {
    *(f4*)&part[w][c0] = ps;
    __syncthreads();
    f4 t = *(const f4*)&part[0][c0];
#pragma unroll
    for (int ww = 1; ww < FNW; ++ww) t += *(const f4*)&part[ww][c0];
    x = xv + (t + b2);
  }
  if (h == 0 && w == 0) *(f4*)(a.xout + (long)r * FC + c0) = x;
  f4 o;
  ln_row(x, gm, bt, a.eps, o);
  if (w == 0) {
    *(f4*)&lnf[0][c0] = o;
    *(f4*)&lnf[1][c0] = o + qp;
  }
  __syncthreads();
  {
    f4 act[4];                                   // one activation row at a time (registers)
    load_actf(lnf[1], lane, act);
    wq.dot(act, lane, qs + 4 * w);
    wk.dot(act, lane, ks + 4 * w);
    load_actf(lnf[0], lane, act);
    wv.dot(act, lane, vs + 4 * w);
  }
  __syncthreads();
  if (w == 0 && lane < FHD) {
    // bias (q scaled); k / v appended to the cache row of step i
    const float q = (qs[lane] + bq) * scale, k = ks[lane] + bk, v = vs[lane] + bv;
    qs[lane] = q;
    ks[lane] = k;
    vs[lane] = v;
    const long crow = ((long)r * Lmax + i) * FC + FHD * h + lane;
    a.kc[crow] = k;
    a.vc[crow] = v;
  }
  __syncthreads();
  at.compute(qs, ks, vs, lane);
  at.publish(mxs, sms, accs, w, lane);
  __syncthreads();
  if (w == 0) merge_f32(mxs, sms, accs, os, lane);
  __syncthreads();
  wo.apply(os, a.slab + ((long)h * a.R + r) * FC, w, lane);
}

struct CrossF32Args {
  const float* slab_in;   // [H][R][C] self-attention partial out-projections
  const float* x;         // residual in [R][C]
  const float* bo_in;     // self out-projection bias
  float* xo;              // residual out (written by the h = 0 blocks)
  const float* gamma;     // LN2
  const float* beta;
  float eps;
  const float* pos;       // [C] query position row
  const float* wq;        // cross in-projection rows 0..C (queries) [C][C]
  const float* bq;
  const float* k;         // memory keys / values [(R / kv_group) * Lk][C] (fp32)
  const float* v;
  int Lk, kv_group;
  const unsigned char* kpm;   // [R / kv_group][Lk] or null
  const float* wo;        // cross out-projection [C][C]
  float* slab_out;        // [H][R][C]
  int R;
  bool xcd;
};

template <int KU>
__global__ void __launch_bounds__(64 * FNW, KU <= 2 ? 4 : 2) dec_cross_f32_kernel(CrossF32Args a, float scale) {
  constexpr int KPW = 16 * KU;
  __shared__ __attribute__((aligned(16))) float lnf[FC];
  __shared__ __attribute__((aligned(16))) float part[FNW][FC];  // the self-attention head partials
  __shared__ __attribute__((aligned(16))) float qs[FHD], os[FHD];
  __shared__ float mxs[FNW], sms[FNW];
  __shared__ __attribute__((aligned(16))) float accs[FNW * FHD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int r, h;
  f32_block_rh(blockIdx.x, a.R, a.xcd, r, h);
  const long RC = (long)a.R * FC;
  const int kvb = r / a.kv_group, Lk = a.Lk;
  const unsigned char* km = a.kpm ? a.kpm + (long)kvb * Lk : nullptr;
  // every global load first: this wave's memory keys / values, query and out-projection weight
  // rows, the self-attention head partials and the row operands
  AttnF<KU> at;
  const int j0 = w * KPW, j1 = min(Lk, (w + 1) * KPW);
  at.set_rows(j0, j1, [&](int j) -> long { return (long)kvb * Lk + j; }, lane);
  at.load_mask(km, j0, j1, lane);
  at.load_rows(a.k, a.v, h, lane);
  ProjF wqp;
  wqp.load(a.wq, FHD * h + 4 * w, lane);
  OutF wo;
  wo.load(a.wo, h, w, lane);
  const float bq = lane < FHD ? a.bq[FHD * h + lane] : 0.f;
  // (wave w loads head w's partial: the eight are summed in head order through LDS)
  static_assert(FH == FNW, "one self-attention head partial per wave");
  const int c0 = 4 * lane;
  const f4 tw = *(const f4*)(a.slab_in + w * RC + (long)r * FC + c0);
  const f4 xv = *(const f4*)(a.x + (long)r * FC + c0);
  const f4 bo = *(const f4*)(a.bo_in + c0);
  const f4 gm = *(const f4*)(a.gamma + c0);
  const f4 bt = *(const f4*)(a.beta + c0);
  const f4 ps = a.pos ? *(const f4*)(a.pos + c0) : f4{0.f, 0.f, 0.f, 0.f};
  // x' = x + (sum_h slab_in[h] + b_o), heads in order
  *(f4*)&part[w][c0] = tw;
  __syncthreads();
  f4 s = *(const f4*)&part[0][c0];
#pragma unroll
  for (int hh = 1; hh < FH; ++hh) s += *(const f4*)&part[hh][c0];
  const f4 x = xv + (s + bo);
  if (h == 0 && w == 0) *(f4*)(a.xo + (long)r * FC + c0) = x;
  f4 o;
  ln_row(x, gm, bt, a.eps, o);
  if (w == 0) *(f4*)&lnf[c0] = o + ps;
  __syncthreads();
  {
    f4 act[4];
    load_actf(lnf, lane, act);
    wqp.dot(act, lane, qs + 4 * w);
  }
  __syncthreads();
  if (w == 0 && lane < FHD) qs[lane] = (qs[lane] + bq) * scale;
  __syncthreads();
  at.compute(qs, nullptr, nullptr, lane);
  at.publish(mxs, sms, accs, w, lane);
  __syncthreads();
  if (w == 0) merge_f32(mxs, sms, accs, os, lane);
  __syncthreads();
  wo.apply(os, a.slab_out + ((long)h * a.R + r) * FC, w, lane);
}

// FFN of the fused fp32 step.  Block = 16 rows x HB = 64 hidden units [j0, j0 + 64), 16 waves.
// Wave w: LayerNorm row w (x'' = xin + (sum_h hslab[h] + bo), heads in order; the j0 = 0 blocks
// write x''), then FFN1 column tile w & 3 over the K quarter w >> 2 (16 exact-f32 MFMAs; the four
// quarters' partial tiles added in quarter order), then FFN2 output column tile w (16 columns,
// K = the block's 64 hidden units) -> slab blockIdx.x.
__global__ void __launch_bounds__(1024) dec_ffn_f32_kernel(
    const float* __restrict__ xin, const float* __restrict__ hslab, int nslab,
    const float* __restrict__ bo, const float* __restrict__ gamma, const float* __restrict__ beta,
    float eps, float* __restrict__ xout, int R, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, int F, float* __restrict__ slabs) {
  constexpr int HB = 64, AS = FC + 4, HS = HB + 4, MAXS = 8;
  __shared__ __attribute__((aligned(16))) float As[16 * AS];     // LN3 rows [16][C]
  __shared__ __attribute__((aligned(16))) float Hs[16 * HS];     // relu(h) [16][HB]
  __shared__ f4 red[16][64];                                     // FFN1 partial tiles
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.x * HB, r0 = blockIdx.y * 16;
  const int nl = lane & 15, g = lane >> 4;
  // weights first: FFN1 tile (hidden units j0 + 16 (w & 3) + nl) over k = 64 (w >> 2) + 16 b + 4 g;
  // FFN2 rows n = 16 w + nl over hidden units j0 + 16 b + 4 g
  const int t1 = w & 3, kq = w >> 2;
  f4 w1f[4], w2f[4];
  {
    const float* p1 = w1 + (long)(j0 + 16 * t1 + nl) * FC + 64 * kq + 4 * g;
    const float* p2 = w2 + (long)(16 * w + nl) * F + j0 + 4 * g;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      w1f[b] = *(const f4*)(p1 + 16 * b);
      w2f[b] = *(const f4*)(p2 + 16 * b);
    }
  }
  const float b1v = b1[j0 + 16 * t1 + nl];
  // LayerNorm row r0 + w: every partial / residual load in flight at once
  const int c0 = 4 * lane;
  const int r = r0 + w, rr = r < R ? r : R - 1;
  const long RC = (long)R * FC;
  f4 t[MAXS];
#pragma unroll
  for (int j = 0; j < MAXS; ++j)
    t[j] = j < nslab ? *(const f4*)(hslab + j * RC + (long)rr * FC + c0) : f4{0.f, 0.f, 0.f, 0.f};
  const f4 xv = *(const f4*)(xin + (long)rr * FC + c0);
  const f4 bb = *(const f4*)(bo + c0);
  const f4 gm = *(const f4*)(gamma + c0);
  const f4 bt = *(const f4*)(beta + c0);
  f4 s{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < MAXS; ++j)
    if (j < nslab) s += t[j];
  const f4 x = xv + (s + bb);
  if (blockIdx.x == 0 && r < R) *(f4*)(xout + (long)r * FC + c0) = x;
  f4 o;
  ln_row(x, gm, bt, eps, o);
  *(f4*)(As + w * AS + c0) = o;
  __syncthreads();
  // FFN1 partial tile (16 rows x 16 hidden units) over this wave's K quarter
  f4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const f4 xa = *(const f4*)(As + nl * AS + 64 * kq + 16 * b + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], w1f[b][e], acc, 0, 0, 0);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w < 4) {
    const f4 hsum = ((red[w][lane] + red[w + 4][lane]) + red[w + 8][lane]) + red[w + 12][lane];
#pragma unroll
    for (int e = 0; e < 4; ++e) Hs[(4 * g + e) * HS + 16 * w + nl] = fmaxf(hsum[e] + b1v, 0.f);
  }
  __syncthreads();
  // FFN2 partial: rows r0.., output columns 16 w + nl, K = the block's 64 hidden units
  f4 acc2{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const f4 ha = *(const f4*)(Hs + nl * HS + 16 * b + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[e], w2f[b][e], acc2, 0, 0, 0);
  }
  float* slab = slabs + (long)blockIdx.x * RC;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ro = r0 + 4 * g + e;
    if (ro < R) slab[(long)ro * FC + 16 * w + nl] = acc2[e];
  }
}

// x = xin + (sum_j slabs[j] + b2) (slab order), xout = x, n = LN(x) (fp32), one wave per row
__global__ void __launch_bounds__(256) dec_rows_f32_kernel(
    const float* __restrict__ xin, const float* __restrict__ slabs, int nslab,
    const float* __restrict__ b2, int R, float* __restrict__ xout,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    float* __restrict__ n) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int c0 = 4 * lane;
  const long RC = (long)R * FC;
  f4 s{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nslab; j0 += 8) {
    f4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      t[u] = j0 + u < nslab ? *(const f4*)(slabs + (j0 + u) * RC + (long)r * FC + c0)
                            : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + u < nslab) s += t[u];
  }
  const f4 x = *(const f4*)(xin + (long)r * FC + c0) + (s + *(const f4*)(b2 + c0));
  if (xout) *(f4*)(xout + (long)r * FC + c0) = x;
  f4 o;
  ln_row(x, *(const f4*)(gamma + c0), *(const f4*)(beta + c0), eps, o);
  *(f4*)(n + (long)r * FC + c0) = o;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int retr_dec_self_f32(int R, int C, int H, const float* win, const float* bin, float* kc,
                      float* vc, int i, int Lmax, const int* anc, const float* wo, float* slab,
                      const float* xin, const float* slabs, int nslab, const float* b2,
                      const long long* tok, const float* word, const float* ge, const float* be,
                      float epse, const float* gamma, const float* beta, float eps,
                      const float* qpos, float* xout, void* stream) {
  RETR_REQUIRE(C == FC && H == FH, "dec_self_f32: C=%d H=%d (needs C=256, 8 heads)", C, H);
  RETR_REQUIRE(i >= 0 && i < Lmax && i + 1 <= 512, "dec_self_f32: step %d (cache %d, <= 512 keys)",
               i, Lmax);
  RETR_REQUIRE(tok ? (word && ge && be) : (xin && slabs && b2 && nslab >= 0),
               "dec_self_f32: incomplete prologue operands");
  RETR_REQUIRE(win && bin && kc && vc && wo && slab && gamma && beta && qpos && xout,
               "dec_self_f32: missing operands");
  RETR_REQUIRE(aligned16(win) && aligned16(wo) && aligned16(kc) && aligned16(vc) &&
                   aligned16(slab) && aligned16(gamma) && aligned16(beta) && aligned16(qpos) &&
                   aligned16(xout) && (tok ? aligned16(word) && aligned16(ge) && aligned16(be)
                                           : aligned16(xin) && aligned16(slabs) && aligned16(b2)),
               "dec_self_f32: operands must be 16-byte aligned");
  if (R == 0) return 0;
  SelfF32Args a{win, bin, kc, vc, i, Lmax, anc, wo, slab, R, xin, slabs, nslab, b2, tok, word,
                ge, be, epse, gamma, beta, eps, qpos, xout,
                retr_tune_get(RETR_TUNE_DEC_ORDER) == 0};
  const float scale = 1.0f / sqrtf((float)FHD);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R * FH)), blk(64 * FNW);
  const int nk = i + 1;
  if (nk <= 128) hipLaunchKernelGGL(dec_self_f32_kernel<1>, grid, blk, 0, st, a, scale);
  else if (nk <= 256) hipLaunchKernelGGL(dec_self_f32_kernel<2>, grid, blk, 0, st, a, scale);
  else hipLaunchKernelGGL(dec_self_f32_kernel<4>, grid, blk, 0, st, a, scale);
  return retr_check_launch("dec_self_f32");
}

int retr_dec_cross_f32(int R, int C, int H, const float* slab_in, const float* x,
                       const float* bo_in, float* xo, const float* gamma, const float* beta,
                       float eps, const float* pos, const float* wq, const float* bq,
                       const float* k, const float* v, int Lk, int kv_group,
                       const unsigned char* kpm, const float* wo, float* slab_out, void* stream) {
  RETR_REQUIRE(C == FC && H == FH, "dec_cross_f32: C=%d H=%d (needs C=256, 8 heads)", C, H);
  RETR_REQUIRE(Lk > 0 && Lk <= 512 && kv_group > 0 && R % kv_group == 0,
               "dec_cross_f32: Lk=%d (1..512) kv_group=%d R=%d", Lk, kv_group, R);
  RETR_REQUIRE(slab_in && x && bo_in && xo && gamma && beta && wq && bq && k && v && wo &&
                   slab_out, "dec_cross_f32: missing operands");
  RETR_REQUIRE(aligned16(slab_in) && aligned16(x) && aligned16(bo_in) && aligned16(xo) &&
                   aligned16(gamma) && aligned16(beta) && (!pos || aligned16(pos)) &&
                   aligned16(wq) && aligned16(k) && aligned16(v) && aligned16(wo) &&
                   aligned16(slab_out), "dec_cross_f32: operands must be 16-byte aligned");
  if (R == 0) return 0;
  CrossF32Args a{slab_in, x, bo_in, xo, gamma, beta, eps, pos, wq, bq, k, v, Lk, kv_group, kpm,
                 wo, slab_out, R, retr_tune_get(RETR_TUNE_DEC_ORDER) == 0};
  const float scale = 1.0f / sqrtf((float)FHD);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(R * FH)), blk(64 * FNW);
  if (Lk <= 128) hipLaunchKernelGGL(dec_cross_f32_kernel<1>, grid, blk, 0, st, a, scale);
  else if (Lk <= 256) hipLaunchKernelGGL(dec_cross_f32_kernel<2>, grid, blk, 0, st, a, scale);
  else hipLaunchKernelGGL(dec_cross_f32_kernel<4>, grid, blk, 0, st, a, scale);
  return retr_check_launch("dec_cross_f32");
}

int retr_dec_ffn_f32(const float* xin, const float* hslab, int nslab, const float* bo,
                     const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                     const float* w1, const float* b1, const float* w2, int F, float* slabs,
                     void* stream) {
  RETR_REQUIRE(C == FC && F > 0 && F % 64 == 0 && nslab >= 0 && nslab <= 8,
               "dec_ffn_f32: C=%d F=%d nslab=%d (C 256, 64 | F, nslab <= 8)", C, F, nslab);
  RETR_REQUIRE(aligned16(xin) && aligned16(hslab) && aligned16(bo) && aligned16(gamma) &&
                   aligned16(beta) && aligned16(xout) && aligned16(w1) && aligned16(w2) &&
                   aligned16(slabs), "dec_ffn_f32: operands must be 16-byte aligned");
  if (R == 0) return 0;
  hipLaunchKernelGGL(dec_ffn_f32_kernel, dim3(F / 64, cdiv(R, 16)), dim3(1024), 0,
                     (hipStream_t)stream, xin, hslab, nslab, bo, gamma, beta, eps, xout, R, w1,
                     b1, w2, F, slabs);
  return retr_check_launch("dec_ffn_f32");
}

int retr_dec_rows_f32(const float* xin, const float* slabs, int nslab, const float* b2, int R,
                      int C, float* xout, const float* gamma, const float* beta, float eps,
                      float* n, void* stream) {
  RETR_REQUIRE(C == FC && nslab >= 0, "dec_rows_f32: C=%d (needs 256) nslab=%d", C, nslab);
  RETR_REQUIRE(aligned16(xin) && aligned16(slabs) && aligned16(b2) && aligned16(gamma) &&
                   aligned16(beta) && aligned16(n) && (!xout || aligned16(xout)),
               "dec_rows_f32: operands must be 16-byte aligned");
  if (R == 0) return 0;
  hipLaunchKernelGGL(dec_rows_f32_kernel, dim3(cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream,
                     xin, slabs, nslab, b2, R, xout, gamma, beta, eps, n);
  return retr_check_launch("dec_rows_f32");
}

}  // extern "C"
