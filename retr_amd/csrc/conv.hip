// ResNet convolutions as implicit GEMMs on the MFMA core (NHWC activations).
//
//   forward : Y[n,oh,ow,co] = act( sum_{kh,kw,ci} X[n,ih,iw,ci] Weff[co,kh,kw,ci] + beff[co] [+ R] )
//             Weff = W * bn_scale (FrozenBatchNorm2d folded, models/backbone.py:41-51)
//   dgrad   : dX[n,ih,iw,ci] = gate( sum_{kh,kw,co} G[n,oh,ow,co] Weff[co,kh,kw,ci] [+ addend] )
//             with ih = oh*s - p + kh*d  (stride handled by a divisibility test)
//   wgrad   : dWeff[co, (kh,kw,ci)] = sum_pixels G[pix,co] X[pix @ (kh,kw), ci]   (split-K)
//             then dW = dWeff * bn_scale, scattered to the OIHW parameter layout.
#include <algorithm>
#include <cstring>
#include <vector>

#include "gemm2.hpp"
#include "panel.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

using namespace retr;

namespace retr {
bool conv3x3_direct_ok(int H, int W, int CI, int CO);
int conv3x3_fwd_direct(const bf16* x, const bf16* w, const float* bias, bf16* y, int relu, int Nb,
                       int H, int W, int CI, int CO, hipStream_t st);
int conv3x3_dgrad_direct(const bf16* dy, const bf16* wt, bf16* dx, const bf16* addend,
                         const bf16* gate, int Nb, int H, int W, int CI_out, int CO_in,
                         hipStream_t st);
}  // namespace retr

namespace {

struct Geom {
  int Nb, H, W, C, Co, KH, KW, s, p, d, OH, OW;
};

// k cursor over (kh, kw, channel) for a K dimension laid out as [KH][KW][Cc]: advancing by
// the tile depth needs no division (Cc >= 8; at most a few wraps per step).
struct TapCur {
  int k, c, kw, khd, kwd;  // flat k, channel in tap, kw index, kh*dil, kw*dil
};
RETR_DEVICE TapCur tap_cur(int k, int Cc, int KW, int dil) {
  TapCur t;
  t.k = k;
  int khw = k / Cc;
  t.c = k - khw * Cc;
  int kh = khw / KW;
  t.kw = khw - kh * KW;
  t.khd = kh * dil;
  t.kwd = t.kw * dil;
  return t;
}
RETR_DEVICE void tap_advance(TapCur& t, int d, int Cc, int KW, int dil) {
  t.k += d;
  t.c += d;
  while (t.c >= Cc) {
    t.c -= Cc;
    if (++t.kw == KW) {
      t.kw = 0;
      t.kwd = 0;
      t.khd += dil;
    } else {
      t.kwd += dil;
    }
  }
}

template <typename T>
struct ConvFwdA {  // A(m = n,oh,ow ; k = kh,kw,ci)
  static constexpr bool kContig = true;
  const T* x;
  Geom g;
  int M, K;
  struct Ctx { const T* img; int ihb, iwb; bool ok; };
  using KCur = TapCur;
  RETR_DEVICE Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < M;
    int rr = c.ok ? r : 0;
    int hw = g.OH * g.OW;
    int n = rr / hw, rem = rr - n * hw;
    int oh = rem / g.OW, ow = rem - oh * g.OW;
    c.img = x + (long)n * g.H * g.W * g.C;
    c.ihb = oh * g.s - g.p;
    c.iwb = ow * g.s - g.p;
    return c;
  }
  RETR_DEVICE KCur kcur(int k) const { return tap_cur(k, g.C, g.KW, g.d); }
  RETR_DEVICE void advance(KCur& t, int d) const { tap_advance(t, d, g.C, g.KW, g.d); }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!c.ok || t.k >= K) return nullptr;
    int ih = c.ihb + t.khd, iw = c.iwb + t.kwd;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return nullptr;
    return c.img + ((long)ih * g.W + iw) * g.C + t.c;
  }
};

// ConvFwdA for C % 64 == 0 (every conv but the stem): a 64-deep K step never leaves one
// (kh, kw) tap, so the K cursor is wave-uniform (kUniformK: SGPRs) and the address of a chunk is
// the row's pixel pointer at tap (0, 0) plus the cursor's tap offset; the padding test is one
// bit of a per-row mask of in-bounds taps (built once).  No 64-bit multiplies, divisions or
// branches per DMA (ConvFwdA: ~25 vector instructions per chunk, this: ~6).
template <typename T>
struct ConvFwdAU {  // A(m = n,oh,ow ; k = kh,kw,ci)
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  const T* x;
  Geom g;
  int M, K;
  struct Ctx { const T* base; unsigned mask; };
  struct KCur { int c0, t, kh, kw, off; };     // off = (kh d W + kw d) C + c0 (elements)
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    Ctx c;
    const bool ok = r < M;
    const int rr = ok ? r : 0;
    const int hw = g.OH * g.OW;
    const int n = rr / hw, rem = rr - n * hw;
    const int oh = rem / g.OW, ow = rem - oh * g.OW;
    const int ihb = oh * g.s - g.p, iwb = ow * g.s - g.p;
    c.base = x + (((long)n * g.H + ihb) * g.W + iwb) * g.C + coff;
    unsigned m = 0;
    if (ok) {
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw)
          if ((unsigned)(ihb + kh * g.d) < (unsigned)g.H &&
              (unsigned)(iwb + kw * g.d) < (unsigned)g.W)
            m |= 1u << (kh * g.KW + kw);
    }
    c.mask = m;
    return c;
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE void set_off(KCur& t) const { t.off = (t.kh * g.d * g.W + t.kw * g.d) * g.C + t.c0; }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.t = k / g.C;
    t.c0 = k - t.t * g.C;
    t.kh = t.t / g.KW;
    t.kw = t.t - t.kh * g.KW;
    set_off(t);
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.c0 += d;
    if (t.c0 >= g.C) {                 // d <= 64 <= C: at most one tap per step
      t.c0 -= g.C;
      ++t.t;
      if (++t.kw == g.KW) {
        t.kw = 0;
        ++t.kh;
      }
    }
    set_off(t);
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!((c.mask >> t.t) & 1u)) return nullptr;   // padding, rows >= M, taps past K
    return c.base + t.off;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& t, const void* fb) const {
    return ((c.mask >> t.t) & 1u) ? (const void*)(c.base + t.off) : fb;
  }
};

template <typename T>
struct ConvDgradA {  // A(m = n,ih,iw ; k = kh,kw,co) = G[n, (ih+p-kh d)/s, (iw+p-kw d)/s, co]
  static constexpr bool kContig = true;
  const T* gr;
  Geom g;
  int M, K;
  struct Ctx { const T* img; int ihp, iwp; bool ok; };
  using KCur = TapCur;
  RETR_DEVICE Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < M;
    int rr = c.ok ? r : 0;
    int hw = g.H * g.W;
    int n = rr / hw, rem = rr - n * hw;
    int ih = rem / g.W, iw = rem - ih * g.W;
    c.img = gr + (long)n * g.OH * g.OW * g.Co;
    c.ihp = ih + g.p;
    c.iwp = iw + g.p;
    return c;
  }
  RETR_DEVICE KCur kcur(int k) const { return tap_cur(k, g.Co, g.KW, g.d); }
  RETR_DEVICE void advance(KCur& t, int d) const { tap_advance(t, d, g.Co, g.KW, g.d); }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!c.ok || t.k >= K) return nullptr;
    int th = c.ihp - t.khd, tw = c.iwp - t.kwd;
    if (th < 0 || tw < 0) return nullptr;
    int oh = th, ow = tw;
    if (g.s != 1) {
      oh = th / g.s;
      ow = tw / g.s;
      if (oh * g.s != th || ow * g.s != tw) return nullptr;
    }
    if (oh >= g.OH || ow >= g.OW) return nullptr;
    return c.img + ((long)oh * g.OW + ow) * g.Co + t.c;
  }
};

// ConvDgradA for stride 1 with Co % 64 == 0: as ConvFwdAU, the tap of a 64-deep K step is
// wave-uniform; chunk address = the pixel pointer of G at (ih + p, iw + p) minus the tap offset
// (kh d OW + kw d) Co, padding test = one bit of the row's in-bounds-tap mask.
template <typename T>
struct ConvDgradAU {  // A(m = n,ih,iw ; k = kh,kw,co) = G[n, ih+p-kh d, iw+p-kw d, co]
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  const T* gr;
  Geom g;
  int M, K;
  struct Ctx { const T* base; unsigned mask; };
  struct KCur { int c0, t, kh, kw, off; };     // off = c0 - (kh d OW + kw d) Co
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    Ctx c;
    const bool ok = r < M;
    const int rr = ok ? r : 0;
    const int hw = g.H * g.W;
    const int n = rr / hw, rem = rr - n * hw;
    const int ih = rem / g.W, iw = rem - ih * g.W;
    const int ihp = ih + g.p, iwp = iw + g.p;
    c.base = gr + (((long)n * g.OH + ihp) * g.OW + iwp) * g.Co + coff;
    unsigned m = 0;
    if (ok) {
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw)
          if ((unsigned)(ihp - kh * g.d) < (unsigned)g.OH &&
              (unsigned)(iwp - kw * g.d) < (unsigned)g.OW)
            m |= 1u << (kh * g.KW + kw);
    }
    c.mask = m;
    return c;
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE void set_off(KCur& t) const {
    t.off = t.c0 - (t.kh * g.d * g.OW + t.kw * g.d) * g.Co;
  }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.t = k / g.Co;
    t.c0 = k - t.t * g.Co;
    t.kh = t.t / g.KW;
    t.kw = t.t - t.kh * g.KW;
    set_off(t);
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.c0 += d;
    if (t.c0 >= g.Co) {
      t.c0 -= g.Co;
      ++t.t;
      if (++t.kw == g.KW) {
        t.kw = 0;
        ++t.kh;
      }
    }
    set_off(t);
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!((c.mask >> t.t) & 1u)) return nullptr;
    return c.base + t.off;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& t, const void* fb) const {
    return ((c.mask >> t.t) & 1u) ? (const void*)(c.base + t.off) : fb;
  }
};

template <typename T>
struct ConvWgradB {  // B(row = kh,kw,ci ; k = pixel n,oh,ow) = X[n, oh*s-p+kh d, ow*s-p+kw d, ci]
  static constexpr bool kContig = false;
  const T* x;
  Geom g;
  int rows, M;
  int adv_q, adv_r;   // one K-step (Elem<T>::BK pixels) = adv_q output rows + adv_r columns
  struct Ctx { int khd, kwd; long off; bool ok; };
  // the cursor keeps the output pixel (n, oh, ow) and the element offset of the input pixel
  // (n, oh*s, ow*s): advancing one K-step is adds and at most a wrap or two, no divisions
  struct KCur { int m, oh, ow; long base; };
  RETR_DEVICE Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < rows;
    int rr = c.ok ? r : 0;
    int khw = rr / g.C;
    const int ci = rr - khw * g.C;
    int kh = khw / g.KW, kw = khw - kh * g.KW;
    c.khd = kh * g.d - g.p;
    c.kwd = kw * g.d - g.p;
    c.off = ((long)c.khd * g.W + c.kwd) * g.C + ci;
    return c;
  }
  RETR_DEVICE KCur kcur(int m) const {
    KCur k;
    k.m = m;
    int hw = g.OH * g.OW;
    const int n = m / hw;
    int rem = m - n * hw;
    k.oh = rem / g.OW;
    k.ow = rem - k.oh * g.OW;
    k.base = (((long)n * g.H + k.oh * g.s) * g.W + k.ow * g.s) * g.C;
    return k;
  }
  RETR_DEVICE void advance(KCur& k, int d) const {
    k.m += d;
    if (d != Elem<T>::BK) {   // generic step (not used by the GEMM cores)
      k = kcur(k.m);
      return;
    }
    const long rowC = (long)g.s * g.W * g.C;          // one output row down
    k.ow += adv_r;
    k.oh += adv_q;
    k.base += (long)adv_q * rowC + (long)adv_r * g.s * g.C;
    if (k.ow >= g.OW) {
      k.ow -= g.OW;
      k.oh += 1;
      k.base += rowC - (long)g.OW * g.s * g.C;
    }
    while (k.oh >= g.OH) {                            // next image
      k.oh -= g.OH;
      k.base += ((long)g.H - (long)g.OH * g.s) * g.W * g.C;
    }
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    if (!c.ok || k.m >= M) return nullptr;
    int ih = k.oh * g.s + c.khd, iw = k.ow * g.s + c.kwd;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return nullptr;
    return x + k.base + c.off;
  }
};

// ConvWgradB with 32-bit element offsets (inputs under 2^31 elements) and at most one output-row
// and one image wrap per K-step (OH * OW >= BK): the cursor advance is four 32-bit adds and two
// conditional ones, the chunk test and address one compare chain and one 64-bit add -- the
// 64-bit cursor arithmetic, its selects and the image-wrap loop of ConvWgradB were most of the
// weight-gradient loop's vector instructions (82 per K-step beside 16 MFMAs).
template <typename T>
struct ConvWgradB32 {  // B(row = kh,kw,ci ; k = pixel n,oh,ow) = X[n, oh*s-p+kh d, ow*s-p+kw d, ci]
  static constexpr bool kContig = false;
  const T* x;
  Geom g;
  int rows, M;
  int adv_q, adv_r;          // one K-step = adv_q output rows + adv_r columns
  int d_step, d_row, d_img;  // element-offset deltas: a K-step, an output-row wrap, an image wrap
  struct Ctx { int khd, kwd, off; bool ok; };
  struct KCur { int m, oh, ow, base; };
  RETR_DEVICE Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < rows;
    const int rr = c.ok ? r : 0;
    const int khw = rr / g.C;
    const int ci = rr - khw * g.C;
    const int kh = khw / g.KW, kw = khw - kh * g.KW;
    c.khd = kh * g.d - g.p;
    c.kwd = kw * g.d - g.p;
    c.off = (c.khd * g.W + c.kwd) * g.C + ci;
    return c;
  }
  RETR_DEVICE KCur kcur(int m) const {
    KCur k;
    k.m = m;
    const int hw = g.OH * g.OW;
    const int n = m / hw;
    const int rem = m - n * hw;
    k.oh = rem / g.OW;
    k.ow = rem - k.oh * g.OW;
    k.base = ((n * g.H + k.oh * g.s) * g.W + k.ow * g.s) * g.C;
    return k;
  }
  RETR_DEVICE void advance(KCur& k, int d) const {
    if (d != Elem<T>::BK) {   // generic step (not used by the GEMM cores)
      k = kcur(k.m + d);
      return;
    }
    k.m += d;
    k.ow += adv_r;
    k.oh += adv_q;
    k.base += d_step;
    if (k.ow >= g.OW) {
      k.ow -= g.OW;
      k.oh += 1;
      k.base += d_row;
    }
    if (k.oh >= g.OH) {
      k.oh -= g.OH;
      k.base += d_img;
    }
  }
  RETR_DEVICE bool ok(const Ctx& c, const KCur& k) const {
    const int ih = k.oh * g.s + c.khd, iw = k.ow * g.s + c.kwd;
    return c.ok & (k.m < M) & ((unsigned)ih < (unsigned)g.H) & ((unsigned)iw < (unsigned)g.W);
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    return ok(c, k) ? (const void*)(x + (unsigned)(k.base + c.off)) : nullptr;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& k, const void* fb) const {
    return ok(c, k) ? (const void*)(x + (unsigned)(k.base + c.off)) : fb;
  }
};

// ---- stride-2 data gradient by output phase ------------------------------------------------
// For stride 2 (dilation 1) only taps kh == (ih + p) mod 2 reach an input row ih, so the
// dgrad of each of the four (ih, iw) parity classes is a dense implicit GEMM over its own tap
// subset: no MFMA work on the structurally zero (tap, pixel) pairs that the generic
// ConvDgradA loader multiplies (3/4 of them for 1x1 and ~5/9 for 3x3 stride-2 convs).
struct Phase {
  int a, b;          // parity class of (ih + p, iw + p)
  int ih0, iw0;      // first input row / column of the class
  int Hp, Wp;        // rows / columns of the class
  int nkh, nkw;      // taps of the class: kh = a + 2 ti, kw = b + 2 tj
};

template <typename T>
struct ConvDgradPhaseA {  // A(m = n,i',j' ; k = ti,tj,co) = G[n, i' + ch(ti), j' + cw(tj), co]
  static constexpr bool kContig = true;
  const T* gr;
  Geom g;
  Phase ph;
  int M, K;
  struct Ctx { const T* img; int i, j; bool ok; };
  struct KCur { int k, c, ti, tj; };
  RETR_DEVICE Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < M;
    const int rr = c.ok ? r : 0;
    const int hw = ph.Hp * ph.Wp;
    const int n = rr / hw, rem = rr - n * hw;
    c.i = rem / ph.Wp;
    c.j = rem - c.i * ph.Wp;
    c.img = gr + (long)n * g.OH * g.OW * g.Co;
    return c;
  }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.k = k;
    const int tap = k / g.Co;
    t.c = k - tap * g.Co;
    t.ti = tap / ph.nkw;
    t.tj = tap - t.ti * ph.nkw;
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.k += d;
    t.c += d;
    while (t.c >= g.Co) {
      t.c -= g.Co;
      if (++t.tj == ph.nkw) {
        t.tj = 0;
        ++t.ti;
      }
    }
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!c.ok || t.k >= K) return nullptr;
    // oh = (ih + p - kh) / 2 with ih = ih0 + 2 i, kh = a + 2 ti
    const int oh = c.i + ((ph.ih0 + g.p - ph.a) >> 1) - t.ti;
    const int ow = c.j + ((ph.iw0 + g.p - ph.b) >> 1) - t.tj;
    if ((unsigned)oh >= (unsigned)g.OH || (unsigned)ow >= (unsigned)g.OW) return nullptr;
    return c.img + ((long)oh * g.OW + ow) * g.Co + t.c;
  }
};

// Uniform-K versions of the two phase loaders (Co % 64 == 0): tap (ti, tj) and channel base
// in SGPRs; A's chunk = the row's G pointer at (i + ch0, j + cw0) minus (ti OW + tj) Co, with a
// per-row mask of in-bounds taps (nkh * nkw <= 32).
template <typename T>
struct ConvDgradPhaseAU {
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  const T* gr;
  Geom g;
  Phase ph;
  int M, K;
  struct Ctx { const T* base; unsigned mask; };
  struct KCur { int c0, t, ti, tj, off; };
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    Ctx c;
    const bool ok = r < M;
    const int rr = ok ? r : 0;
    const int hw = ph.Hp * ph.Wp;
    const int n = rr / hw, rem = rr - n * hw;
    const int i = rem / ph.Wp, j = rem - i * ph.Wp;
    const int oh0 = i + ((ph.ih0 + g.p - ph.a) >> 1), ow0 = j + ((ph.iw0 + g.p - ph.b) >> 1);
    c.base = gr + (((long)n * g.OH + oh0) * g.OW + ow0) * g.Co + coff;
    unsigned m = 0;
    if (ok) {
      for (int ti = 0; ti < ph.nkh; ++ti)
        for (int tj = 0; tj < ph.nkw; ++tj)
          if ((unsigned)(oh0 - ti) < (unsigned)g.OH && (unsigned)(ow0 - tj) < (unsigned)g.OW)
            m |= 1u << (ti * ph.nkw + tj);
    }
    c.mask = m;
    return c;
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE void set_off(KCur& t) const { t.off = t.c0 - (t.ti * g.OW + t.tj) * g.Co; }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.t = k / g.Co;
    t.c0 = k - t.t * g.Co;
    t.ti = t.t / ph.nkw;
    t.tj = t.t - t.ti * ph.nkw;
    set_off(t);
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.c0 += d;
    if (t.c0 >= g.Co) {
      t.c0 -= g.Co;
      ++t.t;
      if (++t.tj == ph.nkw) {
        t.tj = 0;
        ++t.ti;
      }
    }
    set_off(t);
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!((c.mask >> t.t) & 1u)) return nullptr;
    return c.base + t.off;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& t, const void* fb) const {
    return ((c.mask >> t.t) & 1u) ? (const void*)(c.base + t.off) : fb;
  }
};

template <typename T>
struct DgradPhaseWU {  // B(row = ci ; k = ti,tj,co) = Wt[ci][a + 2ti][b + 2tj][co]
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  const T* wt;
  Geom g;
  Phase ph;
  int rows, K;
  struct Ctx { const T* row; int klim; };
  struct KCur { int k, c0, ti, tj, off; };
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    return Ctx{wt + (long)(r < rows ? r : 0) * g.KH * g.KW * g.Co + coff, r < rows ? K : 0};
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE void set_off(KCur& t) const {
    t.off = ((ph.a + 2 * t.ti) * g.KW + ph.b + 2 * t.tj) * g.Co + t.c0;
  }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.k = k;
    const int tap = k / g.Co;
    t.c0 = k - tap * g.Co;
    t.ti = tap / ph.nkw;
    t.tj = tap - t.ti * ph.nkw;
    set_off(t);
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.k += d;
    t.c0 += d;
    if (t.c0 >= g.Co) {
      t.c0 -= g.Co;
      if (++t.tj == ph.nkw) {
        t.tj = 0;
        ++t.ti;
      }
    }
    set_off(t);
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    return t.k < c.klim ? (const void*)(c.row + t.off) : nullptr;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& t, const void* fb) const {
    return t.k < c.klim ? (const void*)(c.row + t.off) : fb;
  }
};

template <typename T>
struct DgradPhaseW {  // B(row = ci ; k = ti,tj,co) = Wt[ci][a + 2ti][b + 2tj][co]
  static constexpr bool kContig = true;
  const T* wt;
  Geom g;
  Phase ph;
  int rows, K;
  struct Ctx { const T* row; bool ok; };
  struct KCur { int k, c, ti, tj; };
  RETR_DEVICE Ctx row_ctx(int r) const {
    return Ctx{wt + (long)(r < rows ? r : 0) * g.KH * g.KW * g.Co, r < rows};
  }
  RETR_DEVICE KCur kcur(int k) const {
    KCur t;
    t.k = k;
    const int tap = k / g.Co;
    t.c = k - tap * g.Co;
    t.ti = tap / ph.nkw;
    t.tj = tap - t.ti * ph.nkw;
    return t;
  }
  RETR_DEVICE void advance(KCur& t, int d) const {
    t.k += d;
    t.c += d;
    while (t.c >= g.Co) {
      t.c -= g.Co;
      if (++t.tj == ph.nkw) {
        t.tj = 0;
        ++t.ti;
      }
    }
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& t) const {
    if (!c.ok || t.k >= K) return nullptr;
    const int kh = ph.a + 2 * t.ti, kw = ph.b + 2 * t.tj;
    return c.row + ((long)kh * g.KW + kw) * g.Co + t.c;
  }
};

// epilogue adaptor: phase-local GEMM row -> NHWC pixel row of dx
template <class EP>
struct EpiPhaseRows {
  EP ep;
  int Hp, Wp, H, W, ih0, iw0;
  static constexpr bool kRowSum = false;
  float* rowsum = nullptr;
  RETR_DEVICE int map(int m) const {
    const int hw = Hp * Wp;
    const int n = m / hw, rem = m - n * hw;
    const int i = rem / Wp, j = rem - i * Wp;
    return (n * H + ih0 + 2 * i) * W + iw0 + 2 * j;
  }
  RETR_DEVICE void apply(int m, int n, float v) const { ep.apply(map(m), n, v); }
  RETR_DEVICE void apply8(int m, int n, float (&v)[8]) const { ep.apply8(map(m), n, v); }
  using Pre = typename EP::Pre;
  RETR_DEVICE void fetch8(int m, int n, Pre& p) const { ep.fetch8(map(m), n, p); }
  RETR_DEVICE void apply8p(int m, int n, float (&v)[8], const Pre& p) const {
    ep.apply8p(map(m), n, v, p);
  }
  RETR_DEVICE void empty_split(int, int) const {}
  RETR_DEVICE bool lane_contiguous() const { return false; }
};

// Forward / data-gradient convs that run faster on the 64x64 two-stage tile than on the
// 128x128 ones (tools/conv_micro.py r50, profiles/r2_conv_tiles.txt): every GEMM over <= 8192
// output pixels (layer 4 at cfg2, incl. stride-2 dgrad phases) unless both N and K exceed 512,
// and 1x1 stride-1 convs into >= 1024 channels from <= 512 (40x40 maps).  A retr_tune
// RETR_TUNE_BIG_TILE override still wins.
inline bool prefer_tile64(int M, int N, int K, bool dense1x1, bool res_small_k) {
  if (retr_tune_get(RETR_TUNE_BIG_TILE) != 0) return false;
  if (res_small_k) return true;   // 1x1 K <= 64 with a residual (layer 1): 117 -> 106 us
  if (M <= 8192 && (N <= 512 || K <= 512)) return true;
  return dense1x1 && N >= 1024 && K <= 512 && M <= 32768;
}

template <int FAM, typename T, class LA, class LB, class EP>
int launch_auto(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits,
                hipStream_t st, const char* what, bool dense1x1 = false,
                bool res_small_k = false) {
  if constexpr (sizeof(T) == 2) {
    return launch_big<FAM>(la, lb, ep, M, N, K, splits, st, what,
                           prefer_tile64(M, N, K, dense1x1, res_small_k));
  } else {
    if (N >= 128 && M >= 4096) return launch_gemm<FAM, T, 128, 128>(la, lb, ep, M, N, K, splits, st, what);
    return launch_gemm<FAM, T, 64, 64>(la, lb, ep, M, N, K, splits, st, what);
  }
}

// Weight-gradient GEMM (fp32 target, split over the pixel reduction).  Split-K slices write
// partial slabs ws[s] with plain stores (no fp32 atomics: atomics run at ~1.3 TB/s chip-wide
// and made split-K the cost of these GEMMs); retr_conv_wgrad_unpack adds the slabs in order
// while it re-lays the gradient out to OIHW, so the result is deterministic.
struct WgradPlan {
  int tile;     // 128: gemm2 128x128 (LDS-DMA), 65: gemm2 64x64, 129: reg-staged 128x128,
                // 64: reg-staged 64x64
  int splits;
};

template <typename T>
WgradPlan wgrad_plan(int R, int Ncols, int Mp, bool dense1x1) {
  constexpr int BK = Elem<T>::BK;
  WgradPlan p{64, 1};
  if (R >= 128 && Ncols >= 128) p.tile = sizeof(T) == 2 ? 128 : 129;
  // 64x64 LDS-DMA tile for the 1x1 stride-1 weight gradients with a <= 128-wide side or
  // <= 8192 pixels (tools/conv_micro.py wtile, profiles/r2_conv_wgrad_tiles.txt: 3-14 % faster;
  // 3x3, strided and 256 x 512 ones are faster on 128x128); knob 1 forces it, 2 forbids it
  const int tt = retr_tune_get(RETR_TUNE_CONV_WGRAD_TILE);
  if (sizeof(T) == 2 && R >= 64 && Ncols >= 64 &&
      (tt == 1 || (tt == 0 && dense1x1 && (R <= 128 || Ncols <= 128 || Mp <= 8192))))
    p.tile = 65;
  // knob 3: the single-stage 64x64 tile (8 blocks per CU) wherever the 64x64 one is chosen
  if (p.tile == 65 && tt == 3) p.tile = 66;
  const int bm = (p.tile == 64 || p.tile == 65 || p.tile == 66) ? 64 : 128;
  const int bn = bm;
  const long tiles = (long)cdiv(R, bm) * cdiv(Ncols, bn);
  const int ksteps = cdiv(Mp, BK);
  // <= 128 slabs, >= 8 K-steps per slice.  The 128x128 kernel runs two blocks per CU (512
  // slots): pick the slice count by a cost model, rounds x K-steps per slice (a grid of 540
  // blocks runs two rounds, so 14 slices of 29 K-steps beat 15 of 27) plus the slab traffic of
  // the extra slices (tiles x 64 KB written + read per slice, ~0.016 K-step-times per tile).
  const int tune = retr_tune_get(RETR_TUNE_CONV_WGRAD_SPLITS);
  long smax = ksteps / 8;
  if (smax > 128) smax = 128;
  if (smax < 1) smax = 1;
  long s;
  if (tune >= 2) {
    s = tune < smax ? tune : smax;
  } else if (tune == 1 || (p.tile != 128 && p.tile != 65 && p.tile != 66)) {
    s = (512 + tiles - 1) / tiles;
    if (s > smax) s = smax;
  } else {
    // (the 64x64 tile: ~4 blocks per CU, a quarter of the slab bytes per tile)
    const long slots = p.tile == 66 ? 2048 : p.tile == 65 ? 1024 : 512;
    const double slab_cost = p.tile == 128 ? 0.016 : 0.004;
    s = 1;
    double best = 1e30;
    for (long c = 1; c <= smax; ++c) {
      const long kc = cdiv(ksteps, (int)c);
      const long rounds = (tiles * cdiv(ksteps, (int)kc) + slots - 1) / slots;
      const double cost = (double)rounds * (kc + 2) + slab_cost * (double)tiles * c;
      if (cost < best) { best = cost; s = c; }
    }
  }
  if (s < 1) s = 1;
  // the launcher rounds the slice length up to whole K-steps: report the slices it will use
  const int kchunk = cdiv(ksteps, (int)s) * BK;
  p.splits = cdiv(Mp, kchunk);
  return p;
}

template <int FAM, typename T, class LA, class LB>
int launch_wgrad(const LA& la, const LB& lb, float* ws, long ldws, int R, int Ncols, int Mp,
                 hipStream_t st, const char* what, bool dense1x1) {
  const WgradPlan p = wgrad_plan<T>(R, Ncols, Mp, dense1x1);
  const int s = p.splits;
  EpiAccF32 ep{ws, ldws, 0, 0, 1, nullptr};
  ep.split_stride = s > 1 ? (long)R * ldws : 0;
  ep.set_vec();
  if constexpr (sizeof(T) == 2) {
    // 8 waves (4 x 2) for the 3x3 / strided weight gradients, 4 waves (2 x 2) for the dense
    // 1x1 ones with long split-K plans (tools/conv_micro.py wtile, profiles/r3_gemm_depth.txt)
    if (p.tile == 128 && !dense1x1)
      return launch_gemm2<FAM, 128, 128, 4, 2, 2>(la, lb, ep, R, Ncols, Mp, s, st, what);
    if (p.tile == 128) return launch_gemm2<FAM, 128, 128, 2, 2, 2>(la, lb, ep, R, Ncols, Mp, s, st, what);
    if (p.tile == 65) return launch_gemm2<FAM, 64, 64, 2, 2, 2>(la, lb, ep, R, Ncols, Mp, s, st, what);
    if (p.tile == 66) return launch_gemm2<FAM, 64, 64, 2, 2, 1>(la, lb, ep, R, Ncols, Mp, s, st, what);
  } else {
    if (p.tile == 129) return launch_gemm<FAM, T, 128, 128>(la, lb, ep, R, Ncols, Mp, s, st, what);
  }
  return launch_gemm<FAM, T, 64, 64>(la, lb, ep, R, Ncols, Mp, s, st, what);
}

template <typename T>
int conv_fwd_t(const void* x, Geom g, const void* w, const float* bias, const void* res, void* y,
               int relu, hipStream_t st) {
  int M = g.Nb * g.OH * g.OW, N = g.Co, K = g.KH * g.KW * g.C;
  DenseK<T> lb{(const T*)w, (long)K, N, K};
  EpiFwd<T, T> ep{(T*)y, (long)N, bias, (const T*)res, (long)N, relu ? 2 : 0, DropoutParams{0, 0, 1.f}, 0};
  ep.set_vec();
  if (g.KH == 1 && g.KW == 1 && g.s == 1 && g.p == 0) {
    DenseK<T> la{(const T*)x, (long)g.C, M, K};
    // short reductions into >= 1024 channels: the resident-A panel kernel (panel.hpp)
    if constexpr (sizeof(T) == 2) {
      if (K <= 256 && K % 64 == 0 && N >= 1024 && retr_tune_get(RETR_TUNE_PANEL) == 1 &&
          retr_tune_get(RETR_TUNE_PANEL_CONV) == 1)
        return launch_panel<kFamConvFwd>(la, lb, ep, M, N, K, st, "conv_fwd_1x1");
    }
    return launch_auto<kFamConvFwd, T>(la, lb, ep, M, N, K, 1, st, "conv_fwd_1x1", true,
                                       res != nullptr && K <= 64);
  }
  // 3x3 stride-1 pad-1: the direct kernel, input halo resident in LDS (conv3x3.hip)
  if constexpr (sizeof(T) == 2) {
    if (g.KH == 3 && g.KW == 3 && g.s == 1 && g.p == 1 && g.d == 1 && !res && relu &&
        conv3x3_direct_ok(g.H, g.W, g.C, g.Co))
      return conv3x3_fwd_direct((const bf16*)x, (const bf16*)w, bias, (bf16*)y, relu, g.Nb, g.H,
                                g.W, g.C, g.Co, st);
  }
  // (1x1 strided convs keep ConvFwdA: a single tap gains nothing and measured slower)
  if (sizeof(T) == 2 && g.C % 64 == 0 && g.KH * g.KW > 1 && g.KH * g.KW <= 32) {
    ConvFwdAU<T> la{(const T*)x, g, M, K};
    return launch_auto<kFamConvFwd, T>(la, lb, ep, M, N, K, 1, st, "conv_fwd");
  }
  ConvFwdA<T> la{(const T*)x, g, M, K};
  return launch_auto<kFamConvFwd, T>(la, lb, ep, M, N, K, 1, st, "conv_fwd");
}

// dx = gate(addend) (or 0) at the pixels of the tap-less stride-2 phases in `zmask`
// (bit (ih % 2) * 2 + iw % 2); 8 channels per thread
__global__ void dgrad_phase_fill_kernel(bf16* dx, const bf16* addend, const bf16* gate, int H,
                                        int W, int C, long chunks, int zmask) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= chunks) return;
  const int cpp = C / 8;
  const long p = i / cpp;
  const int c = (int)(i - p * cpp) * 8;
  const int iw = (int)(p % W), ih = (int)((p / W) % H);
  if (!((zmask >> ((ih & 1) * 2 + (iw & 1))) & 1)) return;
  const long off = p * C + c;
  bf16x8 v;
  if (addend) {
    v = *(const bf16x8*)(addend + off);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (bf16)0.f;
  }
  if (gate) {
    const bf16x8 gg = *(const bf16x8*)(gate + off);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!((float)gg[e] > 0.f)) v[e] = (bf16)0.f;
  }
  *(bf16x8*)(dx + off) = v;
}

template <typename T>
int conv_dgrad_t(const void* dy, Geom g, const void* wt, void* dx, const void* addend,
                 const void* gate, hipStream_t st) {
  int M = g.Nb * g.H * g.W, N = g.C, K = g.KH * g.KW * g.Co;
  DenseK<T> lb{(const T*)wt, (long)K, N, K};
  EpiDgrad<T, T, T> ep{(T*)dx, (long)N, (const T*)addend, (long)N, (const T*)gate, (long)N};
  ep.set_vec();
  if (g.KH == 1 && g.KW == 1 && g.s == 1 && g.p == 0) {
    DenseK<T> la{(const T*)dy, (long)g.Co, M, K};
    if constexpr (sizeof(T) == 2) {
      if (K <= 256 && K % 64 == 0 && N >= 1024 && retr_tune_get(RETR_TUNE_PANEL) == 1 &&
          retr_tune_get(RETR_TUNE_PANEL_CONV) == 1)
        return launch_panel<kFamConvDgrad>(la, lb, ep, M, N, K, st, "conv_dgrad_1x1");
    }
    return launch_auto<kFamConvDgrad, T>(la, lb, ep, M, N, K, 1, st, "conv_dgrad_1x1", true);
  }
  if (g.s == 2 && g.d == 1) {
    // phases with no taps (a 1x1 stride-2 kernel reaches one pixel in four): dx = gate(addend)
    // there, written by one elementwise pass instead of K = 0 GEMM launches
    int zmask = 0;
    for (int a = 0; a < 2; ++a)
      for (int bb = 0; bb < 2; ++bb) {
        const int nkh = g.KH > a ? (g.KH - a + 1) / 2 : 0;
        const int nkw = g.KW > bb ? (g.KW - bb + 1) / 2 : 0;
        if (nkh * nkw == 0) {
          const int ih0 = ((a - g.p) % 2 + 2) % 2, iw0 = ((bb - g.p) % 2 + 2) % 2;
          zmask |= 1 << (ih0 * 2 + iw0);
        }
      }
    // dx == addend (in place): the caller has written gate(addend) at every pixel already (the
    // block's other branch, ResNet first blocks: resnet.py), so the tap-less phases are final
    // and only the phases with taps are rewritten -- no fill pass over 3/4 of the map
    const bool inplace = addend != nullptr && addend == dx;
    if (zmask && (inplace || (sizeof(T) == 2 && N % 8 == 0))) {
      if (!inplace) {
        const long chunks = (long)M * (N / 8);
        hipLaunchKernelGGL(dgrad_phase_fill_kernel, dim3((unsigned)cdiv(chunks, 256)), dim3(256),
                           0, st, (bf16*)dx, (const bf16*)addend, (const bf16*)gate, g.H, g.W, N,
                           chunks, zmask);
        if (int e = retr_check_launch("conv_dgrad_phase_fill")) return e;
      }
    } else {
      zmask = 0;
    }
    for (int a = 0; a < 2; ++a)
      for (int bb = 0; bb < 2; ++bb) {
        Phase ph;
        ph.a = a;
        ph.b = bb;
        ph.ih0 = ((a - g.p) % 2 + 2) % 2;
        ph.iw0 = ((bb - g.p) % 2 + 2) % 2;
        ph.Hp = g.H > ph.ih0 ? (g.H - ph.ih0 + 1) / 2 : 0;
        ph.Wp = g.W > ph.iw0 ? (g.W - ph.iw0 + 1) / 2 : 0;
        ph.nkh = g.KH > a ? (g.KH - a + 1) / 2 : 0;
        ph.nkw = g.KW > bb ? (g.KW - bb + 1) / 2 : 0;
        const int Mp = g.Nb * ph.Hp * ph.Wp, Kp = ph.nkh * ph.nkw * g.Co;
        if (Mp == 0) continue;
        if (Kp == 0 && (zmask >> (ph.ih0 * 2 + ph.iw0) & 1)) continue;
        EpiPhaseRows<EpiDgrad<T, T, T>> pe{ep, ph.Hp, ph.Wp, g.H, g.W, ph.ih0, ph.iw0};
        if (sizeof(T) == 2 && g.Co % 64 == 0 && ph.nkh * ph.nkw <= 32) {
          ConvDgradPhaseAU<T> pa{(const T*)dy, g, ph, Mp, Kp};
          DgradPhaseWU<T> pb{(const T*)wt, g, ph, N, Kp};
          // <= 128 input channels over >= 64k phase pixels (layer2.0's 3x3 stride-2 at cfg2):
          // the single-stage 64x128 tile, more blocks in flight (tools/conv_micro.py r50,
          // profiles/r3_shortk_s1.txt: 160x160x128 <- 128 k3s2 120 -> 99 us)
          if constexpr (sizeof(T) == 2) {
            if (N <= 128 && Mp >= 65536 && retr_tune_get(RETR_TUNE_BIG_TILE) == 0 &&
                retr_tune_get(RETR_TUNE_SHORTK) != 1) {
              if (int e = launch_gemm2<kFamConvDgrad, 64, 128, 2, 2, 1>(pa, pb, pe, Mp, N, Kp, 1,
                                                                          st, "conv_dgrad_s2"))
                return e;
              continue;
            }
          }
          if (int e = launch_auto<kFamConvDgrad, T>(pa, pb, pe, Mp, N, Kp, 1, st, "conv_dgrad_s2"))
            return e;
          continue;
        }
        ConvDgradPhaseA<T> pa{(const T*)dy, g, ph, Mp, Kp};
        DgradPhaseW<T> pb{(const T*)wt, g, ph, N, Kp};
        if (int e = launch_auto<kFamConvDgrad, T>(pa, pb, pe, Mp, N, Kp, 1, st, "conv_dgrad_s2"))
          return e;
      }
    return 0;
  }
  if constexpr (sizeof(T) == 2) {
    if (g.KH == 3 && g.KW == 3 && g.s == 1 && g.p == 1 && g.d == 1 &&
        conv3x3_direct_ok(g.H, g.W, g.Co, g.C))
      return conv3x3_dgrad_direct((const bf16*)dy, (const bf16*)wt, (bf16*)dx,
                                  (const bf16*)addend, (const bf16*)gate, g.Nb, g.H, g.W, g.Co,
                                  g.C, st);
  }
  if (sizeof(T) == 2 && g.s == 1 && g.Co % 64 == 0 && g.KH * g.KW <= 32) {
    ConvDgradAU<T> la{(const T*)dy, g, M, K};
    return launch_auto<kFamConvDgrad, T>(la, lb, ep, M, N, K, 1, st, "conv_dgrad");
  }
  ConvDgradA<T> la{(const T*)dy, g, M, K};
  return launch_auto<kFamConvDgrad, T>(la, lb, ep, M, N, K, 1, st, "conv_dgrad");
}

template <typename T>
int conv_wgrad_t(const void* dy, const void* x, Geom g, float* ws, hipStream_t st) {
  int Mp = g.Nb * g.OH * g.OW;          // reduction length (pixels)
  int R = g.Co, Ncols = g.KH * g.KW * g.C;
  DenseT<T> la{(const T*)dy, (long)g.Co, R, Mp};
  if (g.KH == 1 && g.KW == 1 && g.s == 1 && g.p == 0) {
    DenseT<T> lb{(const T*)x, (long)g.C, Ncols, Mp};
    return launch_wgrad<kFamConvWgrad, T>(la, lb, ws, (long)Ncols, R, Ncols, Mp, st, "conv_wgrad_1x1",
                                          true);
  }
  constexpr int BK = Elem<T>::BK;
  if constexpr (sizeof(T) == 2) {
    if ((long)g.Nb * g.H * g.W * g.C < (1L << 31) && g.OH * g.OW >= BK &&
        retr_tune_get(RETR_TUNE_WGRAD_B32) != 1) {
      const int q = BK / g.OW, r = BK % g.OW;
      ConvWgradB32<T> lb{(const T*)x, g, Ncols, Mp, q, r,
                         (q * g.s * g.W + r * g.s) * g.C,
                         g.s * g.W * g.C - g.OW * g.s * g.C,
                         (g.H - g.OH * g.s) * g.W * g.C};
      return launch_wgrad<kFamConvWgrad, T>(la, lb, ws, (long)Ncols, R, Ncols, Mp, st,
                                            "conv_wgrad", false);
    }
  }
  ConvWgradB<T> lb{(const T*)x, g, Ncols, Mp, BK / g.OW, BK % g.OW};
  return launch_wgrad<kFamConvWgrad, T>(la, lb, ws, (long)Ncols, R, Ncols, Mp, st, "conv_wgrad", false);
}

// ---- weight packing: fp32 OIHW (+ FrozenBN buffers) -> folded [Co][KH][KW][Cp] and the
//      dgrad image [Cp][KH][KW][Co]; also beff/scale for the epilogues.
template <typename T>
__global__ void conv_pack_kernel(const float* w, const float* bnw, const float* bnb,
                                 const float* bnrm, const float* bnrv, const float* conv_bias,
                                 int Co, int Ci, int KH, int KW, int Cp, T* wout, T* wtout,
                                 float* bias_out, float* scale_out) {
  long total = (long)Co * KH * KW * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int ci = i % Cp;
    long t = i / Cp;
    int kw = t % KW;
    t /= KW;
    int kh = t % KH;
    int co = (int)(t / KH);
    float scale = 1.f;
    if (bnw) scale = bnw[co] * (1.0f / sqrtf(bnrv[co] + 1e-5f));
    float v = ci < Ci ? w[(((long)co * Ci + ci) * KH + kh) * KW + kw] * scale : 0.f;
    wout[i] = from_f<T>(v);
    if (wtout) wtout[(((long)ci * KH + kh) * KW + kw) * Co + co] = from_f<T>(v);
    if (ci == 0 && kh == 0 && kw == 0) {
      float b;
      if (bnw) b = bnb[co] - bnrm[co] * scale;
      else b = conv_bias ? conv_bias[co] : 0.f;
      if (bias_out) bias_out[co] = b;
      if (scale_out) scale_out[co] = scale;
    }
  }
}

// grad[co][ci][kh][kw] (=|+=) scale[co] * sum_s ws[s][co][kh][kw][ci]: threads walk the slabs
// in their own order (4 consecutive input channels per thread, 16-byte loads, eight slabs in
// flight, added in slice order) and scatter into the OIHW parameter layout
__global__ void wgrad_unpack4_kernel(const float* ws, const float* scale, float* grad, int Co,
                                     int Ci, int Cp, int KHW, int accumulate, int splits) {
  const int c4 = Ci / 4;
  const long total = (long)Co * KHW * c4;
  const long slab = (long)Co * KHW * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % c4) * 4;
    const long t = i / c4;
    const int tap = (int)(t % KHW), co = (int)(t / KHW);
    const float* src = ws + ((long)co * KHW + tap) * Cp + ci;
    f32x4 v = *(const f32x4*)src;
    int s = 1;
    for (; s + 7 < splits; s += 8) {
      f32x4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *(const f32x4*)(src + (s + k) * slab);
#pragma unroll
      for (int k = 0; k < 8; ++k) v += u[k];
    }
    for (; s < splits; ++s) v += *(const f32x4*)(src + s * slab);
    const float sc = scale ? scale[co] : 1.f;
    float* dst = grad + ((long)co * Ci + ci) * KHW + tap;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = v[e] * sc;
      dst[(long)e * KHW] = accumulate ? dst[(long)e * KHW] + x : x;
    }
  }
}

// Same sum with the slices spread over NW waves: the 64 lanes of a wave take 64 consecutive
// 4-channel chunks (coalesced 1 KB per load), wave w adds slices w, w + NW, ... (up to 8 loads in
// flight), and wave 0 adds the NW partial sums in wave order -- a fixed order, so still
// deterministic.  (One thread per chunk walking all slices left the 3x3 / 56-slice and 1x1 /
// 124-slice unpacks at ~150 blocks, latency-bound at ~10 us.)
template <int NW>
__global__ void __launch_bounds__(NW * 64)
wgrad_unpack4w_kernel(const float* ws, const float* scale, float* grad, int Co, int Ci, int Cp,
                      int KHW, int accumulate, int splits) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c4 = Ci / 4;
  const long total = (long)Co * KHW * c4;
  const long slab = (long)Co * KHW * Cp;
  const long i = (long)blockIdx.x * 64 + lane;
  int ci = 0, tap = 0, co = 0;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    ci = (int)(i % c4) * 4;
    const long t = i / c4;
    tap = (int)(t % KHW);
    co = (int)(t / KHW);
    const float* src = ws + ((long)co * KHW + tap) * Cp + ci;
    int s = w;
    for (; s + 7 * NW < splits; s += 8 * NW) {
      f32x4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *(const f32x4*)(src + (long)(s + k * NW) * slab);
#pragma unroll
      for (int k = 0; k < 8; ++k) v += u[k];
    }
    for (; s < splits; s += NW) v += *(const f32x4*)(src + (long)s * slab);
  }
  if constexpr (NW > 1) {
    red[w][lane] = v;
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int k = 1; k < NW; ++k) v += red[k][lane];
  }
  if (i >= total) return;
  const float sc = scale ? scale[co] : 1.f;
  float* dst = grad + ((long)co * Ci + ci) * KHW + tap;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = v[e] * sc;
    dst[(long)e * KHW] = accumulate ? dst[(long)e * KHW] + x : x;
  }
}

__global__ void wgrad_unpack_kernel(const float* ws, const float* scale, float* grad, int Co,
                                    int Ci, int Cp, int KH, int KW, int accumulate, int splits) {
  const long total = (long)Co * Ci * KH * KW;
  const long slab = (long)Co * KH * KW * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int kw = i % KW;
    long t = i / KW;
    int kh = t % KH;
    t /= KH;
    int ci = t % Ci;
    int co = (int)(t / Ci);
    const long src = ((long)co * KH * KW + kh * KW + kw) * Cp + ci;
    float v = ws[src];
    int s = 1;
    for (; s + 7 < splits; s += 8) {           // eight slab loads in flight, added in order
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = ws[src + (s + u) * slab];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += t[u];
    }
    for (; s < splits; ++s) v += ws[src + s * slab];
    if (scale) v *= scale[co];
    grad[i] = accumulate ? grad[i] + v : v;
  }
}

// Grouped weight packing: every conv of the backbone in one launch (the per-conv launches were
// ~42 small, latency-bound kernels per training step).  Block ranges per descriptor (block-
// uniform descriptor lookup); the per-element arithmetic of conv_pack_kernel.
constexpr int kPackGroup = 16;
constexpr int kPackPerThread = 4;

struct PackGroup {
  retr_conv_pack_desc d[kPackGroup];
  int blk0[kPackGroup + 1];
  int n;
};

template <typename T>
__global__ void __launch_bounds__(256) conv_pack_group_kernel(PackGroup g) {
  const int bid = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int i = 1; i < kPackGroup; ++i)
    if (i < g.n && bid >= g.blk0[i]) p = i;
  const retr_conv_pack_desc& d = g.d[p];
  const int Co = d.Co, Ci = d.Ci, KH = d.KH, KW = d.KW, Cp = d.Cp;
  const long total = (long)Co * KH * KW * Cp;
  const long base = ((long)(bid - g.blk0[p]) * 256 + threadIdx.x) * kPackPerThread;
  const float* bnw = d.bn_w;
#pragma unroll
  for (int u = 0; u < kPackPerThread; ++u) {
    const long i = base + u;
    if (i >= total) break;
    const int ci = (int)(i % Cp);
    long t = i / Cp;
    const int kw = (int)(t % KW);
    t /= KW;
    const int kh = (int)(t % KH);
    const int co = (int)(t / KH);
    float scale = 1.f;
    if (bnw) scale = bnw[co] * (1.0f / sqrtf(d.bn_rv[co] + 1e-5f));
    const float v = ci < Ci ? d.w[(((long)co * Ci + ci) * KH + kh) * KW + kw] * scale : 0.f;
    ((T*)d.w_out)[i] = from_f<T>(v);
    if (d.wt_out) ((T*)d.wt_out)[(((long)ci * KH + kh) * KW + kw) * Co + co] = from_f<T>(v);
    if (ci == 0 && kh == 0 && kw == 0) {
      float b;
      if (bnw) b = d.bn_b[co] - d.bn_rm[co] * scale;
      else b = d.conv_bias ? d.conv_bias[co] : 0.f;
      if (d.bias_out) d.bias_out[co] = b;
      if (d.scale_out) d.scale_out[co] = scale;
    }
  }
}

// Tiled grouped packing for convs with Ci == Cp and 64 | Co, Cp: one block per (desc, 64 output
// channels, 64 input channels, all KHW taps): the fp32 rows [co][ci0 .. ci0+63][taps] are read as
// contiguous runs, folded and rounded into an LDS tile, and both images are written as 128-byte
// runs ([co][tap][Cp] with ci fastest, [ci][tap][Co] with co fastest).
template <typename T, int KHW>
__global__ void __launch_bounds__(256) conv_pack_tiled_group_kernel(PackGroup g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* tile = (T*)smem;                            // [64 co][64 ci][KHW] (+2 pad per co)
  __shared__ float sc[64];
  const int bid = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int i = 1; i < kPackGroup; ++i)
    if (i < g.n && bid >= g.blk0[i]) p = i;
  const retr_conv_pack_desc& d = g.d[p];
  const int Co = d.Co, Cp = d.Cp;
  const int t = bid - g.blk0[p], tn = Cp / 64;
  const int co0 = (t / tn) * 64, ci0 = (t % tn) * 64;
  const int tid = threadIdx.x;
  if (tid < 64) {
    const int co = co0 + tid;
    float scale = 1.f;
    if (d.bn_w) scale = d.bn_w[co] * (1.0f / sqrtf(d.bn_rv[co] + 1e-5f));
    sc[tid] = scale;
    if (ci0 == 0) {
      float b;
      if (d.bn_w) b = d.bn_b[co] - d.bn_rm[co] * scale;
      else b = d.conv_bias ? d.conv_bias[co] : 0.f;
      if (d.bias_out) d.bias_out[co] = b;
      if (d.scale_out) d.scale_out[co] = scale;
    }
  }
  __syncthreads();
  constexpr int ROW = 64 * KHW;                  // one co row of the tile
  constexpr int LDR = ROW + 2;                   // odd dword stride: the co-fastest reads below
  constexpr int TOT = 64 * ROW;                  // hit 64 distinct banks
  // fp32 rows in 16-byte loads (a row's 64 KHW floats are contiguous and 16-byte aligned)
  constexpr int R4 = ROW / 4;
  static_assert(ROW % 4 == 0, "pack row");
#pragma unroll 4
  for (int f = tid; f < 64 * R4; f += 256) {
    const int r = f / R4, j = 4 * (f - r * R4);
    const float4 v = *(const float4*)(d.w + ((long)(co0 + r) * Cp + ci0) * KHW + j);
    const float s = sc[r];
    tile[r * LDR + j] = from_f<T>(v.x * s);
    tile[r * LDR + j + 1] = from_f<T>(v.y * s);
    tile[r * LDR + j + 2] = from_f<T>(v.z * s);
    tile[r * LDR + j + 3] = from_f<T>(v.w * s);
  }
  __syncthreads();
  // both images in 16-byte stores: VEC consecutive ci (image 1) / co (image 2) per store
  constexpr int VEC = 16 / sizeof(T), NV = 64 / VEC;
  typedef __attribute__((ext_vector_type(4))) unsigned int u4;
  T* wout = (T*)d.w_out;
#pragma unroll 4
  for (int e = tid; e < 64 * KHW * NV; e += 256) {
    const int cc = e % NV, q = e / NV;
    const int tap = q % KHW, r = q / KHW;
    T v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = tile[r * LDR + (cc * VEC + k) * KHW + tap];
    *(u4*)(wout + ((long)(co0 + r) * KHW + tap) * Cp + ci0 + cc * VEC) = *(const u4*)v;
  }
  if (!d.wt_out) return;
  T* wt = (T*)d.wt_out;
#pragma unroll 4
  for (int e = tid; e < 64 * KHW * NV; e += 256) {
    const int rc = e % NV, q = e / NV;
    const int tap = q % KHW, ci = q / KHW;
    T v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = tile[(rc * VEC + k) * LDR + ci * KHW + tap];
    *(u4*)(wt + ((long)(ci0 + ci) * KHW + tap) * Co + co0 + rc * VEC) = *(const u4*)v;
  }
}

Geom make_geom(int Nb, int H, int W, int C, int Co, int KH, int KW, int s, int p, int d) {
  Geom g{Nb, H, W, C, Co, KH, KW, s, p, d, 0, 0};
  g.OH = (H + 2 * p - d * (KH - 1) - 1) / s + 1;
  g.OW = (W + 2 * p - d * (KW - 1) - 1) / s + 1;
  return g;
}


// ---- grouped weight gradients of many convolutions (retr_conv2d_wgrad_group) -----------------
// The weight gradients of a whole backbone backward in two launches (dense 1x1 stride-1 convs;
// 3x3 / strided convs on the ConvWgradB32 loader) instead of one split-K GEMM + one slab-sum
// unpack per conv.  One K-slice length for the whole group (about two blocks per slot over all
// problems' tiles) replaces each conv's own slice count, which had to fill the chip from 9-144
// tiles alone: layer 3 / 4 3x3 convs drop from 14 / 3 slices to 2 / 1, the slab bytes written and
// re-read by the unpacks fall ~5x.  Problems live in a device table (put by table_put launches in
// stream order); logical blocks go to the XCDs in runs of kCWChunk, the XCDs taking turns, with
// the longest blocks first.
//
// (Round 5's slice-affine order -- every tile of one K-slice on one XCD, from a host-built piece
// table -- was measured 0.17 ms/step slower and has been removed: DESIGN.md §4.)
struct CWProb {
  const bf16* dy;
  const bf16* x;
  float* ws;
  Geom g;
  int splits, kchunk, tiles_n, tiles, blk0, vec;
};
struct CWHead {
  int nprob, total, pad0, pad1;
};
static_assert(sizeof(CWProb) == 96 && sizeof(CWHead) == 16, "conv wgrad table");
constexpr int kCWChunk = 4;

template <int KIND, int NW, int BN = 128>
__global__ void __launch_bounds__(NW * 64) conv_wgrad_group_kernel(const char* __restrict__ table,
                                                                   int chunk) {
  const CWHead& h = *(const CWHead*)table;
  const CWProb* P = (const CWProb*)(table + sizeof(CWHead));
  const int hw = blockIdx.x, xc = hw & 7, q = hw >> 3;
  const int nprob = h.nprob;
  int lo = 0, split, tile;
  // runs of `chunk` logical blocks per XCD turn
  const int L = (q / chunk) * (8 * chunk) + xc * chunk + q % chunk;
  if (L >= h.total) return;
  int hi = nprob - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (P[mid].blk0 <= L) lo = mid;
    else hi = mid - 1;
  }
  const int local = L - P[lo].blk0;
  split = local / P[lo].tiles;
  tile = local - split * P[lo].tiles;
  if (lo >= nprob || split >= P[lo].splits || tile >= P[lo].tiles) return;   // table guard
  const CWProb d = P[lo];
  const Geom& g = d.g;
  const int Mp = g.Nb * g.OH * g.OW, R = g.Co, Ncols = g.KH * g.KW * g.C;
  const DenseT<bf16> la{d.dy, (long)g.Co, R, Mp};
  EpiAccF32 ep{d.ws, (long)Ncols, 0, d.vec, 1, nullptr};
  ep.split_stride = (long)R * Ncols;
  ep.split = split;
  // 128 x 128: 4 waves (2 x 2) or 8 (4 x 2); 128 x 256 (opt-in): 8 waves (2 x 4) of 64 x 64, the
  // dY panel re-read by half as many column tiles, fp32 epilogue in two row bands
  constexpr int WM = BN == 256 ? 2 : (NW == 8 ? 4 : 2), WN = NW / WM;
  constexpr int EPB = BN == 256 ? 2 : 0;
  if constexpr (KIND == 0) {
    const DenseT<bf16> lb{d.x, (long)g.C, Ncols, Mp};
    gemm2_tile<kFamConvWgrad, 128, BN, WM, WN, 2, EPB>(la, lb, ep, R, Ncols, Mp, d.kchunk,
                                                       d.tiles_n, tile, split);
  } else {
    constexpr int BK = 64;
    const int qq = BK / g.OW, rr = BK % g.OW;
    const ConvWgradB32<bf16> lb{d.x, g, Ncols, Mp, qq, rr, (qq * g.s * g.W + rr * g.s) * g.C,
                                g.s * g.W * g.C - g.OW * g.s * g.C, (g.H - g.OH * g.s) * g.W * g.C};
    gemm2_tile<kFamConvWgrad, 128, BN, WM, WN, 2, EPB>(la, lb, ep, R, Ncols, Mp, d.kchunk,
                                                       d.tiles_n, tile, split);
  }
}

struct CWPut {
  unsigned w[640];
  int off, n;
};

__global__ void __launch_bounds__(256) cw_table_put_kernel(CWPut c, unsigned* dst) {
  for (int i = threadIdx.x; i < c.n; i += 256) dst[c.off + i] = c.w[i];
}

// Every grouped conv's slab sum + OIHW re-layout (+ FrozenBN scale) in ONE launch: 64 chunks of 4
// input channels per block, the 4 waves take every fourth slice (8 loads in flight) and wave 0
// adds the 4 partial sums in wave order (wgrad_unpack4w_kernel's arithmetic) -- instead of one
// unpack launch per conv.
struct UPJob {
  const float* ws;
  const float* scale;
  float* grad;
  int Co, Ci, Cp, KHW, splits, accumulate, blk0, pad;   // pad: grad 16-byte aligned
};
static_assert(sizeof(UPJob) == 56, "unpack table");

__global__ void __launch_bounds__(256) wgrad_unpack_group_kernel(const char* __restrict__ table) {
  __shared__ f32x4 red[4][64];
  const CWHead h = *(const CWHead*)table;
  const UPJob* J = (const UPJob*)(table + sizeof(CWHead));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // a block walks 64-chunk groups bid, bid + gridDim.x, ... (the grid is capped: ~90 k tiny
  // blocks spent their time in dispatch); every group is summed exactly as before
  for (int bid = blockIdx.x; bid < h.total; bid += gridDim.x) {
    int lo = 0, hi = h.nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (J[mid].blk0 <= bid) lo = mid;
      else hi = mid - 1;
    }
    const UPJob d = J[lo];
    const int c4 = d.Ci / 4;
    const long total = (long)d.Co * d.KHW * c4;
    const long slab = (long)d.Co * d.KHW * d.Cp;
    const long i = (long)(bid - d.blk0) * 64 + lane;
    int ci = 0, tap = 0, co = 0;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (i < total) {
      ci = (int)(i % c4) * 4;
      const long t = i / c4;
      tap = (int)(t % d.KHW);
      co = (int)(t / d.KHW);
      const float* src = d.ws + ((long)co * d.KHW + tap) * d.Cp + ci;
      int s = w;
      for (; s + 28 < d.splits; s += 32) {
        f32x4 u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = *(const f32x4*)(src + (long)(s + 4 * k) * slab);
#pragma unroll
        for (int k = 0; k < 8; ++k) v += u[k];
      }
      for (; s < d.splits; s += 4) v += *(const f32x4*)(src + (long)s * slab);
    }
    red[w][lane] = v;
    __syncthreads();
    if (w == 0 && i < total) {
      v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
      const float sc = d.scale ? d.scale[co] : 1.f;
      float* dst = d.grad + ((long)co * d.Ci + ci) * d.KHW + tap;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = v[e] * sc;
        dst[(long)e * d.KHW] = d.accumulate ? dst[(long)e * d.KHW] + x : x;
      }
    }
    __syncthreads();                             // red[] is rewritten by the next group
  }
}

// Round 6: one block per output-channel row (co) of one problem instead of one per 64 chunks.
// A thread owns a 16-byte chunk (4 input channels at one tap) and forms the same four partial
// sums as wgrad_unpack_group_kernel's four waves (slices s = w mod 4, ascending) in registers,
// eight slices in flight, then ((p0 + p1) + p2) + p3 -- bitwise the same values, without the LDS
// reduction and its two barriers per group.  The row's KHW x Ci outputs go through LDS in OIHW
// order, so the gradient is written in contiguous runs (the 64-chunk kernel wrote each 3x3
// value as a 4-byte store KHW floats from its neighbour).  ~92 k tiny blocks -> ~20 k rows.
constexpr int kUnpackRowMax = 9 * 1024;           // floats of LDS: KHW x Ci of one row

__global__ void __launch_bounds__(256) wgrad_unpack_rows_kernel(const char* __restrict__ table) {
  extern __shared__ __attribute__((aligned(16))) float rowbuf[];
  const CWHead h = *(const CWHead*)table;
  const UPJob* J = (const UPJob*)(table + sizeof(CWHead));
  const int bid = blockIdx.x;
  int lo = 0, hi = h.nprob - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (J[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const UPJob d = J[lo];
  const int co = bid - d.blk0;
  if (co >= d.Co) return;                          // table guard
  const int c4 = d.Ci / 4, nch = d.KHW * c4;
  const long slab = (long)d.Co * d.KHW * d.Cp;
  const float sc = d.scale ? d.scale[co] : 1.f;
  const float* rowp = d.ws + (long)co * d.KHW * d.Cp;
  float* grow = d.grad + (long)co * d.Ci * d.KHW;
  const bool staged = d.KHW > 1 && d.KHW * d.Ci <= kUnpackRowMax;
  for (int q = threadIdx.x; q < nch; q += 256) {
    const int tap = q / c4, ci = (q - tap * c4) * 4;
    const float* src = rowp + (long)tap * d.Cp + ci;
    f32x4 p[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) p[w] = f32x4{0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 8 <= d.splits; s += 8) {
      f32x4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *(const f32x4*)(src + (long)(s + k) * slab);
#pragma unroll
      for (int k = 0; k < 8; ++k) p[k & 3] += u[k];
    }
    {
      f32x4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (s + k < d.splits) u[k] = *(const f32x4*)(src + (long)(s + k) * slab);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (s + k < d.splits) p[k & 3] += u[k];
    }
    const f32x4 v = ((p[0] + p[1]) + p[2]) + p[3];
    if (staged) {
#pragma unroll
      for (int e = 0; e < 4; ++e) rowbuf[(ci + e) * d.KHW + tap] = v[e] * sc;
    } else if (d.KHW == 1 && d.pad) {
      f32x4 x = v * sc;
      if (d.accumulate) x += *(const f32x4*)(grow + ci);
      *(f32x4*)(grow + ci) = x;
    } else {
      float* dst = grow + (long)ci * d.KHW + tap;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = v[e] * sc;
        dst[(long)e * d.KHW] = d.accumulate ? dst[(long)e * d.KHW] + x : x;
      }
    }
  }
  if (!staged) return;
  __syncthreads();
  const int n = d.KHW * d.Ci;
  for (int t = threadIdx.x; t < n; t += 256) {
    const float x = rowbuf[t];
    grow[t] = d.accumulate ? grow[t] + x : x;
  }
}

// 0: dense 1x1 stride-1, 1: ConvWgradB32 (3x3 / strided), -1: not groupable
int cw_kind(const Geom& g) {
  if (g.KH == 1 && g.KW == 1 && g.s == 1 && g.p == 0) return 0;
  if ((long)g.Nb * g.H * g.W * g.C < (1L << 31) && g.OH * g.OW >= 64 && g.C % 8 == 0 &&
      g.Co % 8 == 0)
    return 1;
  return -1;
}

}  // namespace

extern "C" {

int retr_conv2d_fwd(int dtype, const void* x, int Nb, int H, int W, int C, const void* w,
                    const float* bias, const void* residual, void* y, int Co, int KH, int KW,
                    int stride, int pad, int dil, int relu, void* stream) {
  Geom g = make_geom(Nb, H, W, C, Co, KH, KW, stride, pad, dil);
  int epc = dtype == RETR_BF16 ? 8 : 4;
  RETR_REQUIRE(C % epc == 0, "conv2d_fwd: C=%d must be a multiple of %d", C, epc);
  RETR_REQUIRE(g.OH > 0 && g.OW > 0, "conv2d_fwd: empty output");
  if (dtype == RETR_BF16) return conv_fwd_t<bf16>(x, g, w, bias, residual, y, relu, (hipStream_t)stream);
  return conv_fwd_t<float>(x, g, w, bias, residual, y, relu, (hipStream_t)stream);
}

int retr_conv2d_fwd_out(int dtype, const void* x, int Nb, int H, int W, int C, const void* w,
                        const float* bias, const void* residual, void* y, int Co, int KH, int KW,
                        int stride, int pad, int dil, int OH, int OW, int relu, void* stream) {
  Geom g = make_geom(Nb, H, W, C, Co, KH, KW, stride, pad, dil);
  int epc = dtype == RETR_BF16 ? 8 : 4;
  RETR_REQUIRE(C % epc == 0, "conv2d_fwd_out: C=%d must be a multiple of %d", C, epc);
  RETR_REQUIRE(OH > 0 && OW > 0 && OH <= g.OH && OW <= g.OW,
               "conv2d_fwd_out: output %dx%d outside the conv's %dx%d", OH, OW, g.OH, g.OW);
  g.OH = OH;
  g.OW = OW;
  if (dtype == RETR_BF16) return conv_fwd_t<bf16>(x, g, w, bias, residual, y, relu, (hipStream_t)stream);
  return conv_fwd_t<float>(x, g, w, bias, residual, y, relu, (hipStream_t)stream);
}

int retr_conv1x1_fwd_cat(int dtype, const void* x1, int C1, const void* x2, int C2, int Nb,
                         int OH, int OW, int H2, int W2, int stride2, const void* w,
                         const float* bias, void* y, int Co, int relu, void* stream) {
  RETR_REQUIRE(dtype == RETR_BF16, "conv1x1_fwd_cat: bf16 only");
  RETR_REQUIRE(C1 % 8 == 0 && C2 % 8 == 0 && C1 > 0 && C2 > 0 && Co % 8 == 0,
               "conv1x1_fwd_cat: C1=%d C2=%d Co=%d must be positive multiples of 8", C1, C2, Co);
  RETR_REQUIRE(Nb > 0 && OH > 0 && OW > 0 && stride2 >= 1 && (OH - 1) * stride2 < H2 &&
               (OW - 1) * stride2 < W2 && (stride2 != 1 || (H2 == OH && W2 == OW)),
               "conv1x1_fwd_cat: %dx%d output of a stride-%d 1x1 conv over %dx%d", OH, OW,
               stride2, H2, W2);
  const int K = C1 + C2, M = Nb * OH * OW;
  DenseK2<bf16> la{(const bf16*)x1, (long)C1, (const bf16*)x2, (long)C2, C1, M, K,
                   OH, OW, H2, W2, stride2};
  DenseK<bf16> lb{(const bf16*)w, (long)K, Co, K};
  EpiFwd<bf16, bf16> ep{(bf16*)y, (long)Co, bias, nullptr, (long)Co, relu ? 2 : 0,
                        DropoutParams{0, 0, 1.f}, 0};
  ep.set_vec();
  // built-in tile rule without the residual-conv 64x64 preference: at layer 1 (K = 128) the
  // single-stage 128x128 tile runs 105 us vs 145 us for 64x64 (tools/cat_micro.py,
  // profiles/r2_cat_micro.txt; unfused pair 212 us)
  return launch_auto<kFamConvFwd, bf16>(la, lb, ep, M, Co, K, 1, (hipStream_t)stream,
                                        "conv_fwd_1x1_cat", true, false);
}

int retr_conv2d_dgrad(int dtype, const void* dy, int Nb, int H, int W, int C, const void* wt,
                      void* dx, int Co, int KH, int KW, int stride, int pad, int dil,
                      const void* addend, const void* gate, void* stream) {
  Geom g = make_geom(Nb, H, W, C, Co, KH, KW, stride, pad, dil);
  int epc = dtype == RETR_BF16 ? 8 : 4;
  RETR_REQUIRE(C % epc == 0 && Co % epc == 0, "conv2d_dgrad: channels must be %%%d", epc);
  if (dtype == RETR_BF16) return conv_dgrad_t<bf16>(dy, g, wt, dx, addend, gate, (hipStream_t)stream);
  return conv_dgrad_t<float>(dy, g, wt, dx, addend, gate, (hipStream_t)stream);
}

int retr_conv2d_wgrad(int dtype, const void* dy, const void* x, int Nb, int H, int W, int C,
                      float* ws, int Co, int KH, int KW, int stride, int pad, int dil,
                      void* stream) {
  Geom g = make_geom(Nb, H, W, C, Co, KH, KW, stride, pad, dil);
  int epc = dtype == RETR_BF16 ? 8 : 4;
  RETR_REQUIRE(C % epc == 0 && Co % epc == 0, "conv2d_wgrad: channels must be %%%d", epc);
  if (dtype == RETR_BF16) return conv_wgrad_t<bf16>(dy, x, g, ws, (hipStream_t)stream);
  return conv_wgrad_t<float>(dy, x, g, ws, (hipStream_t)stream);
}

int retr_conv_pack(int dtype, const float* w, const float* bn_w, const float* bn_b,
                   const float* bn_rm, const float* bn_rv, const float* conv_bias, int Co, int Ci,
                   int KH, int KW, int Cp, void* w_out, void* wt_out, float* bias_out,
                   float* scale_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long total = (long)Co * KH * KW * Cp;
  int grid = (int)(total / 256 + 1 < 4096 ? total / 256 + 1 : 4096);
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(conv_pack_kernel<bf16>, dim3(grid), dim3(256), 0, st, w, bn_w, bn_b, bn_rm,
                       bn_rv, conv_bias, Co, Ci, KH, KW, Cp, (bf16*)w_out, (bf16*)wt_out, bias_out, scale_out);
  else
    hipLaunchKernelGGL(conv_pack_kernel<float>, dim3(grid), dim3(256), 0, st, w, bn_w, bn_b, bn_rm,
                       bn_rv, conv_bias, Co, Ci, KH, KW, Cp, (float*)w_out, (float*)wt_out, bias_out, scale_out);
  return retr_check_launch("conv_pack");
}

}  // extern "C"

namespace {
// launch one class of descriptors (tiled kernel with KHW taps, or the elementwise one: KHW = 0)
template <typename T, int KHW>
int pack_class(const retr_conv_pack_desc* const* d, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += kPackGroup) {
    PackGroup g{};
    int blocks = 0;
    for (int i = i0; i < n && g.n < kPackGroup; ++i) {
      const retr_conv_pack_desc& q = *d[i];
      g.d[g.n] = q;
      g.blk0[g.n] = blocks;
      if constexpr (KHW > 0) blocks += (q.Co / 64) * (q.Cp / 64);
      else blocks += (int)cdiv((long)q.Co * q.KH * q.KW * q.Cp, 256L * kPackPerThread);
      ++g.n;
    }
    g.blk0[g.n] = blocks;
    if (blocks == 0) continue;
    if constexpr (KHW > 0) {
      constexpr size_t lds = (size_t)64 * (64 * KHW + 2) * sizeof(T);
      auto kern = conv_pack_tiled_group_kernel<T, KHW>;
      static bool attr = false;
      if (lds > 65536 && !attr) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr = true;
      }
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, st, g);
    } else {
      hipLaunchKernelGGL(conv_pack_group_kernel<T>, dim3(blocks), dim3(256), 0, st, g);
    }
    if (int e = retr_check_launch("conv_pack_group")) return e;
  }
  return 0;
}

template <typename T>
int pack_all(int n, const retr_conv_pack_desc* d, hipStream_t st) {
  // classes: 3x3 / 1x1 tiled (Ci == Cp, 64 | Co, 64 | Cp, 16-byte aligned w / w_out / wt_out:
  // the tiled kernel moves float4 / 16-byte chunks), everything else elementwise
  const retr_conv_pack_desc* c9[256];
  const retr_conv_pack_desc* c1[256];
  const retr_conv_pack_desc* ce[256];
  int n9 = 0, n1 = 0, ne = 0;
  for (int i = 0; i < n; ++i) {
    const retr_conv_pack_desc& q = d[i];
    const bool aligned =
        (((uintptr_t)q.w | (uintptr_t)q.w_out | (uintptr_t)q.wt_out) & 15) == 0;
    const bool tiled = q.Ci == q.Cp && q.Co % 64 == 0 && q.Cp % 64 == 0 && aligned;
    if (tiled && q.KH * q.KW == 9) c9[n9++] = &q;
    else if (tiled && q.KH * q.KW == 1) c1[n1++] = &q;
    else ce[ne++] = &q;
  }
  if (int e = pack_class<T, 9>(c9, n9, st)) return e;
  if (int e = pack_class<T, 1>(c1, n1, st)) return e;
  return pack_class<T, 0>(ce, ne, st);
}
}  // namespace

extern "C" {

// [W3eff | Wdseff] rows and b3 + bds of every fused bottleneck tail in one launch (one thread
// per 16-byte chunk of a destination row; each problem owns a block range)
struct CatGroup {
  retr_cat_rows_desc d[8];
  int blk0[9];
  int n;
};

__global__ void __launch_bounds__(256) cat_rows_group_kernel(CatGroup g) {
  int p = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i)
    if (i < g.n && (int)blockIdx.x >= g.blk0[i]) p = i;
  const retr_cat_rows_desc& d = g.d[p];
  const long i = (long)(blockIdx.x - g.blk0[p]) * 256 + threadIdx.x;
  const int ca = d.ka / 8, cb = d.kb / 8, c = ca + cb;
  if (i < (long)d.rows * c) {
    const int r = (int)(i / c), j = (int)(i % c);
    const u32x4 v = j < ca ? ((const u32x4*)d.a)[(long)r * ca + j]
                           : ((const u32x4*)d.b)[(long)r * cb + (j - ca)];
    ((u32x4*)d.dst)[i] = v;
  }
  if (i < d.rows) d.bias_dst[i] = d.bias_a[i] + d.bias_b[i];
}

int retr_cat_rows_group(int n, const retr_cat_rows_desc* d, void* stream) {
  RETR_REQUIRE(n >= 0 && n <= 8, "cat_rows_group: n=%d (0..8)", n);
  if (n == 0) return 0;
  CatGroup g{};
  g.n = n;
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    RETR_REQUIRE(d[i].ka % 8 == 0 && d[i].kb % 8 == 0 && d[i].rows > 0,
                 "cat_rows_group[%d]: ka=%d kb=%d rows=%d", i, d[i].ka, d[i].kb, d[i].rows);
    RETR_REQUIRE((((uintptr_t)d[i].a | (uintptr_t)d[i].b | (uintptr_t)d[i].dst) & 15) == 0,
                 "cat_rows_group[%d]: 16-byte alignment", i);
    g.d[i] = d[i];
    g.blk0[i] = blocks;
    const long chunks = (long)d[i].rows * ((d[i].ka + d[i].kb) / 8);
    blocks += (int)cdiv(chunks > d[i].rows ? chunks : (long)d[i].rows, 256L);
  }
  g.blk0[n] = blocks;
  hipLaunchKernelGGL(cat_rows_group_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, g);
  return retr_check_launch("cat_rows_group");
}

int retr_conv_pack_group(int dtype, int n, const retr_conv_pack_desc* d, void* stream) {
  RETR_REQUIRE(n >= 0 && n <= 256, "conv_pack_group: n=%d (0..256)", n);
  hipStream_t st = (hipStream_t)stream;
  return dtype == RETR_BF16 ? pack_all<bf16>(n, d, st) : pack_all<float>(n, d, st);
}

int retr_conv2d_wgrad_splits(int dtype, int Nb, int H, int W, int C, int Co, int KH, int KW,
                             int stride, int pad, int dil) {
  Geom g = make_geom(Nb, H, W, C, Co, KH, KW, stride, pad, dil);
  const int Mp = g.Nb * g.OH * g.OW, Ncols = g.KH * g.KW * g.C;
  const bool d1 = g.KH == 1 && g.KW == 1 && g.s == 1 && g.p == 0;
  return dtype == RETR_BF16 ? wgrad_plan<bf16>(g.Co, Ncols, Mp, d1).splits
                            : wgrad_plan<float>(g.Co, Ncols, Mp, d1).splits;
}

size_t retr_conv2d_wgrad_group_table_bytes(int n) {
  // two kinds, each header + problems, each start 256-byte aligned
  return n < 0 ? 0 : 2 * (sizeof(CWHead) + 256) + (size_t)n * sizeof(CWProb);
}

int retr_conv2d_wgrad_group_plan(int dtype, int n, retr_conv_wgrad_desc* d) {
  RETR_REQUIRE(n >= 0 && (n == 0 || d), "conv2d_wgrad_group_plan: n=%d", n);
  // one K-slice length per kind: ~2 blocks per slot (512 slots: two 64 KB-LDS blocks per CU)
  // over all of the kind's tiles
  long work[2] = {0, 0};
  for (int i = 0; i < n; ++i) {
    retr_conv_wgrad_desc& q = d[i];
    const Geom g = make_geom(q.Nb, q.H, q.W, q.C, q.Co, q.KH, q.KW, q.stride, q.pad, q.dil);
    q.kind = dtype == RETR_BF16 ? cw_kind(g) : -1;
    q.splits = 0;
    if (q.kind < 0) continue;
    const long tiles = (long)cdiv(g.Co, 128) * cdiv(g.KH * g.KW * g.C, 128);
    work[q.kind] += tiles * cdiv(g.Nb * g.OH * g.OW, 64);
  }
  for (int i = 0; i < n; ++i) {
    retr_conv_wgrad_desc& q = d[i];
    if (q.kind < 0) continue;
    const Geom g = make_geom(q.Nb, q.H, q.W, q.C, q.Co, q.KH, q.KW, q.stride, q.pad, q.dil);
    const int ksteps = cdiv(g.Nb * g.OH * g.OW, 64);
    long chunk = (work[q.kind] + 1023) / 1024;
    if (retr_tune_get(RETR_TUNE_CONV_WGRAD_SPLITS) >= 2) chunk = retr_tune_get(RETR_TUNE_CONV_WGRAD_SPLITS);
    if (chunk < 8) chunk = 8;
    long s = (ksteps + chunk - 1) / chunk;
    if (s > 128) s = 128;
    if (s < 1) s = 1;
    const int kchunk = cdiv(ksteps, (int)s) * 64;   // whole K-steps; no empty slices
    q.splits = cdiv(g.Nb * g.OH * g.OW, kchunk);
  }
  return 0;
}

int retr_conv2d_wgrad_group(int dtype, int n, const retr_conv_wgrad_desc* d, void* table,
                            size_t table_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(dtype == RETR_BF16, "conv2d_wgrad_group: bf16 only");
  RETR_REQUIRE(n >= 0 && (n == 0 || d) && n <= 4096, "conv2d_wgrad_group: n=%d", n);
  RETR_REQUIRE(table && table_bytes >= retr_conv2d_wgrad_group_table_bytes(n) &&
                   ((uintptr_t)table & 15) == 0,
               "conv2d_wgrad_group: table of %zu bytes (need %zu, 16-byte aligned)", table_bytes,
               retr_conv2d_wgrad_group_table_bytes(n));
  for (int kind = 0; kind < 2; ++kind) {
    // this kind's problems, longest blocks first (stable)
    std::vector<int> ord;
    for (int i = 0; i < n; ++i)
      if (d[i].kind == kind) {
        RETR_REQUIRE(d[i].splits >= 1 && d[i].ws && d[i].dy && d[i].x,
                     "conv2d_wgrad_group[%d]: unplanned problem", i);
        ord.push_back(i);
      }
    if (ord.empty()) continue;
    // RETR_TUNE_CW_WAVES 3: the 128 x 256 tile for this kind (sweeps)
    const int wl = retr_tune_get(RETR_TUNE_CW_WAVES);
    const int bn = wl == 3 ? 256 : 128;
    auto blk_len = [&](int i) {
      const Geom g = make_geom(d[i].Nb, d[i].H, d[i].W, d[i].C, d[i].Co, d[i].KH, d[i].KW,
                               d[i].stride, d[i].pad, d[i].dil);
      return cdiv(g.Nb * g.OH * g.OW, d[i].splits);
    };
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return blk_len(a) > blk_len(b); });
    std::vector<char> buf(sizeof(CWHead) + ord.size() * sizeof(CWProb) + 16, 0);
    CWHead* h = (CWHead*)buf.data();
    CWProb* P = (CWProb*)(buf.data() + sizeof(CWHead));
    int blocks = 0;
    for (size_t j = 0; j < ord.size(); ++j) {
      const retr_conv_wgrad_desc& q = d[ord[j]];
      const Geom g = make_geom(q.Nb, q.H, q.W, q.C, q.Co, q.KH, q.KW, q.stride, q.pad, q.dil);
      RETR_REQUIRE(cw_kind(g) == kind, "conv2d_wgrad_group[%d]: kind %d does not fit", ord[j], kind);
      CWProb& p = P[j];
      p.dy = (const bf16*)q.dy;
      p.x = (const bf16*)q.x;
      p.ws = q.ws;
      p.g = g;
      const int Mp = g.Nb * g.OH * g.OW, Ncols = g.KH * g.KW * g.C;
      p.kchunk = cdiv(cdiv(Mp, 64), q.splits) * 64;
      p.splits = cdiv(Mp, p.kchunk);
      RETR_REQUIRE(p.splits == q.splits, "conv2d_wgrad_group[%d]: splits %d != plan %d", ord[j],
                   p.splits, q.splits);
      p.tiles_n = cdiv(Ncols, bn);
      p.tiles = cdiv(g.Co, 128) * p.tiles_n;
      p.blk0 = blocks;
      p.vec = vec8_ok<float>(q.ws, (long)Ncols) ? 1 : 0;
      blocks += p.tiles * p.splits;
    }
    h->nprob = (int)ord.size();
    h->total = blocks;
    const size_t used = sizeof(CWHead) + ord.size() * sizeof(CWProb);
    const int words = (int)((used + 3) / 4);
    const unsigned* src = (const unsigned*)buf.data();
    for (int off = 0; off < words; off += 640) {
      CWPut c;
      c.off = off;
      c.n = words - off < 640 ? words - off : 640;
      memcpy(c.w, src + off, (size_t)c.n * 4);
      hipLaunchKernelGGL(cw_table_put_kernel, dim3(1), dim3(256), 0, st, c, (unsigned*)table);
      if (int e = retr_check_launch("conv2d_wgrad_group table")) return e;
    }
    // RETR_TUNE_CW_CHUNK > 0: runs of that many logical blocks per XCD turn (sweeps); else kCWChunk
    int chunk = retr_tune_get(RETR_TUNE_CW_CHUNK);
    chunk = chunk > 0 ? chunk : kCWChunk;
    const int grid = cdiv(blocks, 8 * chunk) * 8 * chunk;
    const int nw = wl == 1 ? 4 : wl == 2 ? 8 : (kind == 0 ? 4 : 8);
    auto launch = [&](auto kern, int threads, size_t lds) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, st, (const char*)table, chunk);
    };
    constexpr size_t lds = gemm2_lds_bytes<128, 128, 2, 0>();
    constexpr size_t lds256 = gemm2_lds_bytes<128, 256, 2, 2>();
    if (bn == 256) {
      if (kind == 0) launch(conv_wgrad_group_kernel<0, 8, 256>, 512, lds256);
      else launch(conv_wgrad_group_kernel<1, 8, 256>, 512, lds256);
    } else if (kind == 0) {
      if (nw == 4) launch(conv_wgrad_group_kernel<0, 4>, 256, lds);
      else launch(conv_wgrad_group_kernel<0, 8>, 512, lds);
    } else {
      if (nw == 4) launch(conv_wgrad_group_kernel<1, 4>, 256, lds);
      else launch(conv_wgrad_group_kernel<1, 8>, 512, lds);
    }
    if (int e = retr_check_launch(kind == 0 ? "conv2d_wgrad_group 1x1" : "conv2d_wgrad_group")) return e;
    // the next kind's table must not overwrite this one before the launch has read it: use
    // the second half of the caller's table for kind 1
    table = (char*)table + (used + 255) / 256 * 256;
    table_bytes -= (used + 255) / 256 * 256;
  }
  return 0;
}

size_t retr_conv_wgrad_unpack_group_table_bytes(int n) {
  return n < 0 ? 0 : sizeof(CWHead) + (size_t)n * sizeof(UPJob);
}

int retr_conv_wgrad_unpack_group(int n, const retr_conv_unpack_desc* d, void* table,
                                 size_t table_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && (n == 0 || d), "conv_wgrad_unpack_group: n=%d", n);
  RETR_REQUIRE(table && table_bytes >= retr_conv_wgrad_unpack_group_table_bytes(n) &&
                   ((uintptr_t)table & 15) == 0,
               "conv_wgrad_unpack_group: table of %zu bytes (need %zu, 16-byte aligned)",
               table_bytes, retr_conv_wgrad_unpack_group_table_bytes(n));
  if (n == 0) return 0;
  std::vector<char> buf(retr_conv_wgrad_unpack_group_table_bytes(n) + 16, 0);
  CWHead* h = (CWHead*)buf.data();
  UPJob* J = (UPJob*)(buf.data() + sizeof(CWHead));
  // RETR_TUNE_UNPACK_GRID: 0 = one block per output-channel row (wgrad_unpack_rows_kernel);
  // -1 = round 5's block per 64 chunks, > 0 = that kernel with its grid capped (A/B)
  const int knob = retr_tune_get(RETR_TUNE_UNPACK_GRID);
  const bool rows = knob == 0;
  int blocks = 0;
  size_t lds = 0;
  for (int i = 0; i < n; ++i) {
    const retr_conv_unpack_desc& q = d[i];
    RETR_REQUIRE(q.ws && q.grad && q.Ci % 4 == 0 && q.Cp % 4 == 0 && q.Cp >= q.Ci &&
                     q.splits >= 1 && ((uintptr_t)q.ws & 15) == 0,
                 "conv_wgrad_unpack_group[%d]: Co=%d Ci=%d Cp=%d splits=%d", i, q.Co, q.Ci,
                 q.Cp, q.splits);
    UPJob& j = J[i];
    j.ws = q.ws;
    j.scale = q.scale;
    j.grad = q.grad;
    j.Co = q.Co;
    j.Ci = q.Ci;
    j.Cp = q.Cp;
    j.KHW = q.KH * q.KW;
    j.splits = q.splits;
    j.accumulate = q.accumulate;
    j.blk0 = blocks;
    j.pad = ((uintptr_t)q.grad & 15) == 0;        // 16-byte rows for the 1x1 store
    if (rows) {
      blocks += q.Co;
      if (j.KHW > 1 && j.KHW * q.Ci <= kUnpackRowMax)
        lds = std::max(lds, (size_t)j.KHW * q.Ci * sizeof(float));
    } else {
      blocks += (int)cdiv((long)q.Co * j.KHW * (q.Ci / 4), 64);
    }
  }
  h->nprob = n;
  h->total = blocks;
  const int words = (int)((retr_conv_wgrad_unpack_group_table_bytes(n) + 3) / 4);
  const unsigned* src = (const unsigned*)buf.data();
  for (int off = 0; off < words; off += 640) {
    CWPut c;
    c.off = off;
    c.n = words - off < 640 ? words - off : 640;
    memcpy(c.w, src + off, (size_t)c.n * 4);
    hipLaunchKernelGGL(cw_table_put_kernel, dim3(1), dim3(256), 0, st, c, (unsigned*)table);
    if (int e = retr_check_launch("conv_wgrad_unpack_group table")) return e;
  }
  if (blocks == 0) return 0;
  if (rows) {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)wgrad_unpack_rows_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(wgrad_unpack_rows_kernel, dim3(blocks), dim3(256), lds, st,
                       (const char*)table);
    return retr_check_launch("conv_wgrad_unpack_group");
  }
  int grid = blocks;
  if (knob > 0 && grid > knob) grid = knob;
  hipLaunchKernelGGL(wgrad_unpack_group_kernel, dim3(grid), dim3(256), 0, st,
                     (const char*)table);
  return retr_check_launch("conv_wgrad_unpack_group");
}

int retr_conv_wgrad_unpack(const float* ws, const float* scale, float* grad, int Co, int Ci,
                           int Cp, int KH, int KW, int accumulate, int splits, void* stream) {
  RETR_REQUIRE(splits >= 1, "conv_wgrad_unpack: splits=%d", splits);
  if (Ci % 4 == 0 && Cp % 4 == 0 && ((uintptr_t)ws & 15) == 0) {
    const long total = (long)Co * KH * KW * (Ci / 4);
    if (splits >= 8) {
      const dim3 grid((unsigned)cdiv(total, 64));
      hipStream_t st = (hipStream_t)stream;
#define UNPW(NW) hipLaunchKernelGGL(wgrad_unpack4w_kernel<NW>, grid, dim3(NW * 64), 0, st, ws, \
                                    scale, grad, Co, Ci, Cp, KH * KW, accumulate, splits)
      if (splits >= 64) UNPW(16);
      else if (splits >= 24) UNPW(8);
      else UNPW(4);
#undef UNPW
      return retr_check_launch("conv_wgrad_unpack4w");
    }
    const int grid = (int)(total / 256 + 1 < 8192 ? total / 256 + 1 : 8192);
    hipLaunchKernelGGL(wgrad_unpack4_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws,
                       scale, grad, Co, Ci, Cp, KH * KW, accumulate, splits);
    return retr_check_launch("conv_wgrad_unpack4");
  }
  long total = (long)Co * Ci * KH * KW;
  int grid = (int)(total / 256 + 1 < 4096 ? total / 256 + 1 : 4096);
  hipLaunchKernelGGL(wgrad_unpack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, scale,
                     grad, Co, Ci, Cp, KH, KW, accumulate, splits);
  return retr_check_launch("conv_wgrad_unpack");
}

}  // extern "C"
