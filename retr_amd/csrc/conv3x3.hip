// Direct 3x3 stride-1 convolution (forward and data gradient) with the input halo resident in
// LDS: the ResNet bottleneck's 3x3 convs (torchvision Bottleneck.conv2 via
// models/backbone.py:65,69) and their data gradients, bf16 NHWC, fp32 accumulation.
//
// The implicit GEMM (conv.hip ConvFwdAU / ConvDgradAU) fetches the A operand -- the input row
// of every (pixel, tap) -- from L2 once per tap: each input pixel crosses the L2 -> CU fabric
// nine times, and a 128x128 tile at 64 channels per K-step needs 32 KB per step, the CU's whole
// fabric bandwidth at full MFMA rate.  Here a block owns a TH x TW output
// tile x BN output channels; per 64-channel input chunk it stages the (TH+2) x (TW+2) halo ONCE
// (global loads -> VGPRs -> LDS, 160-byte padded pixel rows) and runs the chunk's nine taps as
// nine K-steps whose A fragments are LDS reads of the halo at a compile-time offset per tap.
// Only the weights stream per K-step (BN x 64 channels by LDS-DMA, the gemm2.hpp stager and
// swizzle): 16 KB + 1/9 of a halo per step instead of 32 KB.
//
// K order: chunk-major, tap-minor ((c, 0), (c, 1), ... (c, 8), (c + 1, 0) ...), so an output's
// MFMA chain differs from the implicit GEMM's tap-major order: the same products, summed in
// another fixed order (results within fp32 rounding of the implicit GEMM, deterministic).
//
// Data gradient (stride 1, pad 1): dx[ih, iw, ci] = sum dy[ih + 1 - kh, iw + 1 - kw, co]
// W[co][kh][kw][ci] -- a 3x3 convolution of dy with the flipped kernel; the weights come from
// the dgrad pack [Cp][3][3][Co] with the tap index reversed.
#include <cstring>

#include "gemm2.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

using namespace retr;

namespace {

// B operand: row n (output channel), K-step s = (chunk c, tap t): W[n][tap'][c * 64 .. + 64) of a
// [rows][9][CP] pack, tap' = t (forward) or 8 - t (data gradient: flipped kernel)
template <bool FLIP>
struct TapW {
  static constexpr bool kContig = true;
  static constexpr bool kUniformK = true;
  const bf16* p;
  int rows, CP;
  struct Ctx { const bf16* row; bool ok; };
  struct KCur { int t, c64, off; };
  RETR_DEVICE Ctx row_ctx_c(int r, int coff) const {
    return Ctx{p + (long)(r < rows ? r : 0) * 9 * CP + coff, r < rows};
  }
  RETR_DEVICE Ctx row_ctx(int r) const { return row_ctx_c(r, 0); }
  RETR_DEVICE KCur kcur(int) const { return KCur{0, 0, (FLIP ? 8 : 0) * CP}; }
  RETR_DEVICE void advance(KCur& k, int) const {
    if (++k.t == 9) {
      k.t = 0;
      k.c64 += 64;
    }
    k.off = (FLIP ? 8 - k.t : k.t) * CP + k.c64;
  }
  RETR_DEVICE const void* addr_or(const Ctx& c, const KCur& k, const void* fb) const {
    return c.ok ? (const void*)(c.row + k.off) : fb;
  }
  RETR_DEVICE const void* addr(const Ctx& c, const KCur& k) const {
    return c.ok ? (const void*)(c.row + k.off) : nullptr;
  }
};

// Halo pixel rows are RB bytes: 64 bf16 channels + padding.  A fragment read (ds_read_b128) is
// serviced in four 16-lane groups, each mixing two 16-byte k chunks of 8 pixels; with 144-byte
// rows (36 dwords, 9 x 4) pixel r of chunk 1 and pixel r + 7 of chunk 0 share a bank slot -- every
// read of a whole 16-pixel line is a 2-way conflict.  160-byte rows (40 dwords) put a group's 16
// slots on 16 distinct bank slots (the 20-pixel tiles' wrapped lines: 6.4 instead of 10.4 LDS
// cycles per read).  The 4 x 20 four-wave tile keeps 144: at 160 its LDS no longer fits three
// blocks per CU, which costs more than the conflicts (tools/c3_micro.py, profiles/r6_c3_rb.txt);
// the default tiles no longer use it.
template <int TH, int TW, int BN, int RB, int S>
constexpr size_t c3_main_lds() {
  return ((size_t)(TH + 2) * (TW + 2) * RB + 255) / 256 * 256 + (size_t)S * BN * kBKBytes;
}
// epilogue bands: as few as keep the fp32 staging tile within the main loop's LDS footprint
template <int TH, int TW, int BN, int WM, int RB, int S>
constexpr int epi_passes() {
  int p = 1;
  while (p < WM && (size_t)TH * TW * (BN + 4) * 4 / p > c3_main_lds<TH, TW, BN, RB, S>()) p *= 2;
  return p;
}

// S: weight stages in the ring (2: one step of look-ahead; 3: two, counted waits)
template <int TH, int TW, int BN, int WM, int WN, int RB, int S, bool DGRAD, class EP>
__global__ void __launch_bounds__(WM * WN * 64, 2)
conv3x3_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, EP ep, int H, int W,
               int CI, int CO, int tiles_x, int tiles_y, int tiles_n) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = TH * TW;                   // output pixels per block
  constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  constexpr int HALO_BYTES = (HP * RB + 255) / 256 * 256;
  static_assert(RB % 16 == 0 && RB >= 128, "halo row");
  constexpr int WST = BN * kBKBytes;            // one weight stage
  static_assert(S == 2 || S == 3, "weight ring");
  constexpr int HCH = (HP * 8 + NT - 1) / NT;   // 16-byte halo chunks per thread per channel chunk
  using LB = TapW<DGRAD>;
  using SB = GStager<BN, NT, LB>;
  constexpr int LPT = SB::NCH;                  // weight DMA instructions per thread per step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  char* wst = smem + HALO_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // block -> (channel tile, image, tile row, tile column); consecutive blocks share an image
  // region (halo overlap) and all blocks of a channel tile share its weights
  const int nblk = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nblk);
  const int tpi = tiles_x * tiles_y;
  const int nt = bid % tiles_n;
  const int rest = bid / tiles_n;
  const int img = rest / tpi, tt = rest % tpi;
  const int y0 = (tt / tiles_x) * TH, x0 = (tt % tiles_x) * TW;
  const int n0 = nt * BN;
  const int nchunks = CI / 64;
  const int nsteps = nchunks * 9;

  // halo chunk loader: thread q-slots (pixel hp, 16-byte piece j)
  const bf16* xin = x + (long)img * H * W * CI;
  // Every thread issues exactly HCH loads: slots past the halo and pixels outside the image read
  // the zero page.  (The wait at t == 1 below counts HCH halo loads behind the step-1 weight
  // DMA; a predicated load became a branch the compiler skips when a whole wave is masked --
  // waves past the halo's last slots always were -- and vmcnt(HCH) then let that wave's weight
  // chunks still be in flight at the barrier: other waves could read the previous step's
  // weights.  Seen as a rare 1-ulp-scale loss difference in test_gpu_ddp's bitwise check.)
  auto halo_load = [&](int c, u32x4 (&r)[HCH]) {
#pragma unroll
    for (int i = 0; i < HCH; ++i) {
      const int q = tid + NT * i;
      const int hp = q >> 3, j = q & 7;
      const int gy = y0 + hp / HW - 1, gx = x0 + hp % HW - 1;
      const bool ok = q < HP * 8 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      const bf16* src = ok ? xin + ((long)gy * W + gx) * CI + c * 64 + j * 8
                           : (const bf16*)g_zero_page;
      r[i] = *(const u32x4*)src;
    }
  };
  auto halo_store = [&](const u32x4 (&r)[HCH]) {
#pragma unroll
    for (int i = 0; i < HCH; ++i) {
      const int q = tid + NT * i;
      if (q < HP * 8) *(u32x4*)(halo + (q >> 3) * RB + (q & 7) * 16) = r[i];
    }
  };

  // per-lane A base: output pixel p of fragment i at tap (0, 0) = halo pixel (py, px)
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wm * WTM + 16 * i + (lane & 15);
    abase[i] = ((p / TW) * HW + p % TW) * RB + (lane >> 4) * 16;
  }

  SB sb;
  const LB lb{w, CO, CI};
  sb.init(lb, n0, tid, 0);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 hr[HCH];
  halo_load(0, hr);
  sb.issue(lb, wst, wave);                      // weights of step 0 (and 1)
  if (S == 3 && nsteps > 1) sb.issue(lb, wst + WST, wave);
  halo_store(hr);

  int s = 0;
  for (int c = 0; c < nchunks; ++c) {
    if (c > 0) {
      // every wave is done with chunk c - 1's halo: overwrite it with chunk c's
      raw_barrier();
      halo_store(hr);
    }
    const bool more = c + 1 < nchunks;
#pragma unroll
    for (int t = 0; t < 9; ++t, ++s) {
      // weights of step s landed.  In flight behind them may be: the halo loads of chunk
      // c + 1 (issued at t = 0 after the weights of step s0 + S - 1: still allowed at t = 1, and
      // at t = 2 with three stages) and, with three stages, the weights of step s + 1
      const bool nx = S == 3 && s + 1 < nsteps;
      const bool hh = more && (t == 1 || (S == 3 && t == 2));
      if (nx && hh) wait_vmcnt_lgkm0<LPT + HCH>();
      else if (nx) wait_vmcnt_lgkm0<LPT>();
      else if (hh) wait_vmcnt_lgkm0<HCH>();
      else wait_vmcnt_lgkm0<0>();
      raw_barrier();
      if (s + S - 1 < nsteps) sb.issue(lb, wst + ((s + S - 1) % S) * WST, wave);
      if (t == 0 && more) halo_load(c + 1, hr);
      const char* B = wst + (s % S) * WST;
      const int tapoff = ((t / 3) * HW + t % 3) * RB;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *(const u32x4*)(halo + abase[i] + tapoff + ks * 64);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = Stager<bf16, BN, LB>::frag(B, wn * WTN + 16 * j, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mfma_step<bf16>(acc[i][j], af[i], bfr[j]);
      }
    }
  }
  (void)LPT;
  __syncthreads();

  // epilogue through LDS: fp32 tile [BM][BN + 4], 8 consecutive channels per thread, in EPB
  // bands of wave rows when the whole tile does not fit under the main-loop footprint
  constexpr int CS = BN + 4;
  constexpr int EPB = epi_passes<TH, TW, BN, WM, RB, S>();
  constexpr int BAND = BM / EPB;
  constexpr int CH = BN / 8;
  float* ct = (float*)smem;
#pragma unroll
  for (int pass = 0; pass < EPB; ++pass) {
    if (pass > 0) __syncthreads();
    if (wm / (WM / EPB) == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            ct[(wm * WTM - pass * BAND + 16 * i + 4 * (lane >> 4) + e) * CS + wn * WTN + 16 * j +
               (lane & 15)] = acc[i][j][e];
    }
    __syncthreads();
    for (int q = tid; q < BAND * CH; q += NT) {
      const int mb = q / CH, cc = (q % CH) * 8;
      const int m = pass * BAND + mb;
      const int y = y0 + m / TW, xx = x0 + m % TW;
      if (y >= H || xx >= W || n0 + cc >= CO) continue;
      const int row = (img * H + y) * W + xx;
      const f32x4 lo = *(const f32x4*)(ct + mb * CS + cc);
      const f32x4 hi = *(const f32x4*)(ct + mb * CS + cc + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      ep.apply8(row, n0 + cc, v);
    }
  }
}

template <int TH, int TW, int BN, int WM, int WN, int RB, int S>
constexpr size_t c3_lds() {
  constexpr size_t main = c3_main_lds<TH, TW, BN, RB, S>();
  constexpr size_t epi = (size_t)TH * TW * (BN + 4) * 4 / epi_passes<TH, TW, BN, WM, RB, S>();
  return main > epi ? main : epi;
}

template <int TH, int TW, int BN, int WM, int WN, int RB, bool DGRAD, int S = 2, class EP>
int launch_c3(const bf16* x, const bf16* w, const EP& ep, int Nb, int H, int W, int CI, int CO,
              hipStream_t st, const char* what) {
  const int tiles_x = cdiv(W, TW), tiles_y = cdiv(H, TH), tiles_n = cdiv(CO, BN);
  const long blocks = (long)Nb * tiles_x * tiles_y * tiles_n;
  constexpr size_t lds = c3_lds<TH, TW, BN, WM, WN, RB, S>();
  auto kern = conv3x3_kernel<TH, TW, BN, WM, WN, RB, S, DGRAD, EP>;
  if constexpr (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(WM * WN * 64), lds, st, x, w, ep, H, W,
                     CI, CO, tiles_x, tiles_y, tiles_n);
  return retr_check_launch(what);
}

// tile per map width (the cfg2 / cfg4 maps: 80 (layer 2), 40 (layer 3), 20 (layer 4)): rows of
// whole 16- or 20-pixel lines, 8 waves over 128 channels.  RETR_TUNE_C3_TILE (sweeps,
// tools/c3_micro.py) forces one of the variants.
template <bool DGRAD, class EP>
int run_c3(const bf16* x, const bf16* w, const EP& ep, int Nb, int H, int W, int CI, int CO,
           hipStream_t st, const char* what) {
  switch (retr_tune_get(RETR_TUNE_C3_TILE)) {
    case 1: return launch_c3<8, 16, 128, 4, 2, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 2: return launch_c3<8, 20, 128, 2, 4, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 3: return launch_c3<4, 16, 128, 2, 4, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 4: return launch_c3<8, 16, 64, 4, 2, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 5: return launch_c3<16, 16, 128, 4, 2, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 6:
      if (CO % 256 == 0) return launch_c3<8, 20, 256, 2, 4, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
      break;
    case 7: return launch_c3<4, 20, 128, 1, 4, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 8: return launch_c3<8, 16, 128, 2, 2, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    // the 144-byte-row layout of rounds 3-5 (A/B)
    case 9: return launch_c3<4, 20, 128, 1, 4, 144, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 10: return launch_c3<8, 16, 128, 4, 2, 144, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 11: return launch_c3<8, 20, 128, 2, 4, 144, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
    // three weight stages (two steps of look-ahead): within 1-3 % of two, either way
    // (profiles/r6_c3_rb.txt) -- the weight DMA latency is hidden by the second block per CU
    case 12: return launch_c3<8, 16, 128, 4, 2, 160, DGRAD, 3>(x, w, ep, Nb, H, W, CI, CO, st, what);
    case 13: return launch_c3<8, 20, 128, 2, 4, 160, DGRAD, 3>(x, w, ep, Nb, H, W, CI, CO, st, what);
    default: break;
  }
  // tools/c3_micro.py --rounds 3 (profiles/r6_c3_rb.txt, interleaved in one process): with
  // 160-byte halo rows the 8 x 16 eight-wave tile is the fastest on the 80- and 40-wide maps
  // (80x80x128 fwd 38.4 / dgrad 39.3 us vs 38.7 / 40.0 for round 5's 4 x 20 tile; 40x40x256
  // 35.5 / 36.1 vs 36.0 / 36.8 at 144-byte rows), and the 8 x 20 tile now beats the implicit GEMM
  // on the 20x20x512 maps of layer 4 (48.2 / 49.1 vs 51.6 / 52.0 us; at 144-byte rows it lost:
  // 54.4 / 54.7)
  if (W == 20) return launch_c3<8, 20, 128, 2, 4, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
  return launch_c3<8, 16, 128, 4, 2, 160, DGRAD>(x, w, ep, Nb, H, W, CI, CO, st, what);
}

}  // namespace

// used by conv.hip (retr_conv2d_fwd / retr_conv2d_dgrad) for bf16 3x3 stride-1 pad-1 convs
namespace retr {

bool conv3x3_direct_ok(int H, int W, int CI, int CO) {
  const int mode = retr_tune_get(RETR_TUNE_CONV3X3);
  if (mode == 1) return false;
  if (mode == 2) return CI % 64 == 0 && CO % 128 == 0 && H >= 8 && W >= 16;   // sweeps
  return CI % 64 == 0 && CO % 128 == 0 && H >= 8 && (W >= 32 || W == 20);
}

int conv3x3_fwd_direct(const bf16* x, const bf16* w, const float* bias, bf16* y, int relu, int Nb,
                       int H, int W, int CI, int CO, hipStream_t st) {
  EpiFwd<bf16, bf16> ep{y, (long)CO, bias, (const bf16*)nullptr, (long)CO, relu ? 2 : 0,
                        DropoutParams{0, 0, 1.f}, 0};
  ep.set_vec();
  return run_c3<false>(x, w, ep, Nb, H, W, CI, CO, st, "conv3x3_fwd");
}

int conv3x3_dgrad_direct(const bf16* dy, const bf16* wt, bf16* dx, const bf16* addend,
                         const bf16* gate, int Nb, int H, int W, int CI_out, int CO_in,
                         hipStream_t st) {
  // output channels = the conv's input channels (CO_in here); reduction over its outputs
  EpiDgrad<bf16, bf16, bf16> ep{dx, (long)CO_in, addend, (long)CO_in, gate, (long)CO_in};
  ep.set_vec();
  return run_c3<true>(dy, wt, ep, Nb, H, W, CI_out, CO_in, st, "conv3x3_dgrad");
}

}  // namespace retr
