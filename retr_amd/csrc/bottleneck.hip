// Fused stride-1 ResNet bottleneck forward for the frozen layer1 of ResNet-50/101
// (torchvision Bottleneck via models/backbone.py:65, frozen by models/backbone.py:58-60, so no
// activation of it is ever needed by backward):
//
//   h1 = relu(x W1^T + b1)                     1x1, Cin -> 64        (FrozenBN folded)
//   h2 = relu(conv3x3(h1, W2) + b2)            3x3, pad 1, 64 -> 64
//   y  = relu(h2 W3^T + b3 + x)                1x1, 64 -> 256, identity residual (Cin = 256)
//   y  = relu([h2 | x] [W3 | Wds]^T + b3 + bds)  first block: 1x1 downsample folded in (Cin 64)
//
// One 512-thread block (8 waves, 2 blocks per CU) per 8 x 16 output tile of one image.  h1 (on
// the tile's 10 x 18 halo) and h2 never leave LDS: the unfused path wrote and re-read both
// (2 x 2 x 52 MB per block at cfg2) and read x twice (conv1 and the residual, 2 x 210 MB).
// Every product runs the same v_mfma_f32_16x16x32_bf16 chain over K in the same order as the
// unfused implicit-GEMM kernels (K ascending in 32-deep steps; conv2's K is tap-major
// (kh, kw, ci) like the packed weights [Co][3][3][Ci]), with the same bf16 roundings of h1 / h2
// and the same epilogue order (acc + bias (+ residual), ReLU, bf16), so the result equals the
// three-launch path bitwise.
//
//   phase A  h1 on the halo: 12 position tiles (192 >= 180) x 4 channel tiles.  x goes through
//            LDS in 64-channel stages by LDS-DMA (coalesced 128-byte lines, source-side
//            swizzle, zero page for rows outside the image), two stages in flight; W1
//            fragments from L2.  Positions outside the image are written as 0 (conv2's zero
//            padding applies to h1).  With the downsample (Cin 64, one stage) the stage stays
//            resident and phase C reads the tile pixels' rows from it.
//   phase B  h2: B fragments of tap (kh, kw) are the halo rows (py + kh) * 18 + kw + px of h1
//            (padded 144-byte rows: immediate LDS offsets); the W2 fragments are loaded
//            before the barrier that ends phase A.
//   phase C  y: 64 output channels x 4 output rows per wave; acc + b3 staged in fp32 through
//            LDS so the residual read and the store are 128-byte runs per pixel.
// Products are computed transposed (weights = A operand): a lane holds 4 consecutive channels
// of one position, so the h1 / h2 / stage writes are 8- and 16-byte runs.  Biases are copied
// to LDS once per block.  Measured with tools/bn_micro.py / bn_phase.py
// (profiles/r3_bottleneck_ab.txt).
#include "common.hpp"
#include "../../include/retr_hip.h"

#ifndef BN_DIAG
#define BN_DIAG 0        // A/B diagnostics only (tools/bn_micro.sh)
#endif
#ifndef BN_XCD_REMAP
#define BN_XCD_REMAP 1   // tools/bn_micro.sh builds the A/B variant with 0
#endif

namespace {

constexpr int TH = 8, TW = 16;                    // output tile
constexpr int HH = TH + 2, HW = TW + 2;           // halo
constexpr int NHALO = HH * HW;                    // 180 (12 position tiles of 16, 192 rows)
constexpr int P = 64;                             // bottleneck width (planes)
constexpr int CO = 256;                           // block output channels
constexpr int NT = 512;                           // 8 waves

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// Every product is computed transposed: the weights are the A operand (rows = output channels)
// and the activations the B operand (columns = positions), so a lane's accumulator holds 4
// consecutive channels of one position and the epilogues write 8-byte runs (LDS and global)
// instead of single bf16 values.  C[c][p] = sum_k W[c][k] X[p][k] is the same sum as the
// unfused C[p][c], the MFMA reduces over k in the same order for either operand placement.
RETR_DEVICE f32x4 mfma(const u32x4& w, const u32x4& x, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w),
                                                 __builtin_bit_cast(bf16x8, x), acc, 0, 0, 0);
}

// [rows][64] bf16 image with 144-byte rows (16 bytes of padding): a row offset is a compile-time
// constant times the stride, so the conv2 tap walk reads LDS at immediate offsets from one
// per-lane base.  (A ds_read_b128 lane group mixes two k chunks of 8 rows, which 144-byte rows
// put 2-way on some bank slots; 160-byte rows remove that and measured no faster -- phases B / C
// are not LDS-bound: profiles/r6_ab_bn_rs160_rejected.txt.)
constexpr int RS = 144;
constexpr int SST = 68;                           // phase C stage: [8 waves][16 px][64 + 4] fp32
constexpr int H2OFF = 8 * 16 * SST * 4;           // 34816 >= the 192 x 144 of h1s
static_assert(H2OFF >= 192 * RS, "h1s / stage region");
constexpr int XST = 192 * 128;                    // one 64-channel x stage
RETR_DEVICE int soff(int r, int c) { return r * RS + c * 16; }

// read by the halo positions outside the image instead of a predicated load (a branch around
// each load makes the compiler drain the load counter at every join); >= the 8 x 64 + 48 bytes
// a position's k walk spans
static __device__ __attribute__((aligned(64))) unsigned int g_bn_zero[256];

#if BN_DIAG == 9
// per-wave phase time stamps (s_memrealtime, 100 MHz) of the first 4096 blocks: A/B tooling
__device__ unsigned long long g_bn_prof[4096 * 8 * 8];
#define BN_T(k)                                                                          \
  if (lane == 0 && blockIdx.x < 4096)                                                    \
    g_bn_prof[(blockIdx.x * 8 + wave) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define BN_T(k)
#endif

RETR_DEVICE void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                   0, 0);
}

RETR_DEVICE u32x2 pack4(float a, float b, float c, float d) {
  return __builtin_bit_cast(u32x2, bf16x4{(bf16)a, (bf16)b, (bf16)c, (bf16)d});
}

template <bool DS>
constexpr int lds_main() { return H2OFF + 128 * RS + (DS ? XST : 0); }   // h1s | h2s (| x)
static_assert(2 * XST <= H2OFF + 128 * RS, "two x stages under h1s + h2s");

template <int CIN, bool DS>
__global__ void __launch_bounds__(NT, 4)
bottleneck_s1_kernel(const bf16* __restrict__ x, int H, int W, const bf16* __restrict__ w1,
                     const float* __restrict__ b1, const bf16* __restrict__ w2,
                     const float* __restrict__ b2, const bf16* __restrict__ w3,
                     const float* __restrict__ b3, bf16* __restrict__ y) {
  static_assert(CIN % 32 == 0 && (DS ? CIN == 64 : CIN == CO), "shape");
  constexpr int K3 = P + (DS ? CIN : 0);          // conv3 (+ downsample) reduction
  constexpr int KS3 = K3 / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* h1s = smem;                               // [192][64] bf16 (halo positions)
  char* h2s = smem + H2OFF;                       // [128][64] bf16 (tile pixels)
  // x stages: [192][128 B] swizzled; with the downsample (one stage) past h2s, where phase C
  // reads the tile pixels' rows as the downsample operand; else two stages under h1s
  char* xst = DS ? smem + H2OFF + 128 * RS : smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;      // fragment row, 8-element k chunk
  const int tiles_w = W / TW, tiles_h = H / TH;
  // XCD-aware order: hardware deals blocks round-robin over the 8 XCDs; consecutive tiles
  // (which share halo rows of x) land on one XCD's L2
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if (BN_XCD_REMAP && (nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int n = bid / (tiles_h * tiles_w);
  const int rem = bid - n * tiles_h * tiles_w;
  const int y0 = (rem / tiles_w) * TH, x0 = (rem % tiles_w) * TW;
  const bf16* ximg = x + (long)n * H * W * CIN;
  BN_T(0);
  // b1 | b2 | b3 (384 floats) into LDS once; read back by the epilogues (first use is behind
  // phase A's barriers)
  float* bias_s = (float*)(smem + lds_main<DS>());
  if (tid < 96) {                                  // LDS-DMA: no register round trip
    const float* src = tid < 16 ? b1 + 4 * tid : tid < 32 ? b2 + 4 * (tid - 16) : b3 + 4 * (tid - 32);
    glds16(src, (char*)bias_s + wave * 1024);
  }

  // ---- phase A: h1 on the halo ------------------------------------------------------------
  // x goes through LDS in 64-channel stages (2 k-steps): the halo's 192 rows x 128 bytes by
  // LDS-DMA, each wave-instruction 8 positions x one 128-byte line (coalesced), rows
  // XOR-swizzled on the source side (slot s of row r holds chunk s ^ ((r >> 1) & 7)); rows past
  // the halo and positions outside the image read the zero page.  Two stages, one barrier per
  // stage: stage kk + 1 is issued right after the barrier that starts stage kk.
  // MFMA split: wave -> channel tiles 2 (w & 1) + {0, 1} x position tiles 3 (w >> 1) + {0..2};
  // W1 fragments from L2, one stage ahead in registers.
  constexpr int KK = CIN / 64;
  const bf16* lsrc[3];
  {
    const int lc = (tid & 7) ^ ((tid >> 4) & 7);   // (row >> 1) & 7 == (tid >> 4) & 7
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int r = (tid >> 3) + 64 * i;
      const int hy = r / HW, hx = r - hy * HW;
      const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
      bool ok = r < NHALO && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
#if BN_DIAG == 1
      ok = false;
#endif
      lsrc[i] = (ok ? ximg + ((long)iy * W + ix) * CIN : (const bf16*)g_bn_zero) + 8 * lc;
    }
  }
  auto issue_x = [&](int kk) {
#pragma unroll
    for (int i = 0; i < 3; ++i) glds16(lsrc[i] + 64 * kk, xst + (kk & 1) * XST + (512 * i + wave * 64) * 16);
  };
  const int hc = wave & 1, pg = wave >> 1;
  bool aok[3];
  int apos[3], xoff[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int p = 16 * (3 * pg + i) + r16;
    const int hy = p / HW, hx = p - hy * HW;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    apos[i] = p;
    aok[i] = p < NHALO && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) xoff[i][ks] = p * 128 + (((kq + 4 * ks) ^ ((p >> 1) & 7)) << 4);
  }
  const bf16* w1row = w1 + (long)(32 * hc + r16) * CIN + 8 * kq;
  const int ct = wave & 3, rg = wave >> 2;
  const bf16* wrow2 = w2 + (long)(16 * ct + r16) * 9 * P + 8 * kq;
  u32x4 w2f[9][2];
  {
    f32x4 acc[3][2];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // two stages, one barrier per stage: stage kk + 1 (x DMA + the W1 fragments) is issued
    // right after the barrier that starts stage kk.  (A third stage in flight measured no
    // faster: with every block in phase A at once the x reads run at ~5 TB/s.)
    issue_x(0);
    u32x4 wa[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) wa[ks][j] = *(const u32x4*)(w1row + (long)16 * j * CIN + 32 * ks);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      __syncthreads();                             // stage kk landed (every wave's DMA), and
                                                   // stage kk - 1 is no longer read
      u32x4 wn[2][2];
      if (kk + 1 < KK) {
        issue_x(kk + 1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            wn[ks][j] = *(const u32x4*)(w1row + (long)16 * j * CIN + 64 * (kk + 1) + 32 * ks);
      }
      const char* st = xst + (kk & 1) * XST;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const u32x4 a = *(const u32x4*)(st + xoff[i][ks]);
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma(wa[ks][j], a, acc[i][j]);
        }
      if (kk + 1 < KK) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 2; ++j) wa[ks][j] = wn[ks][j];
      }
    }
    BN_T(1);
    if constexpr (!DS) __syncthreads();            // h1s overlays the x stages
    // epilogue: relu(acc + b1) -> bf16, 0 outside the image (conv2 pads h1 with zeros);
    // lane: channels 32 hc + 16 j + 4 kq + e of position apos[i]
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 32 * hc + 16 * j + 4 * kq;
        const f32x4 b1v = *(const f32x4*)(bias_s + c);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = aok[i] ? fmaxf(acc[i][j][e] + b1v[e], 0.f) : 0.f;
        *(u32x2*)(h1s + soff(apos[i], c >> 3) + (c & 7) * 2) = pack4(v[0], v[1], v[2], v[3]);
      }
  }
  // conv2 weights for this wave's channel tile: the first 5 taps' fragments in flight across
  // the barrier, the last 4 taps' issued behind
  // the first tap's products
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) w2f[t][ks] = *(const u32x4*)(wrow2 + t * P + 32 * ks);
  __syncthreads();
  BN_T(2);

  // ---- phase B: h2 = relu(conv3x3(h1) + b2); wave -> channel tile w & 3 x output rows
  //      4 (w >> 2) + {0..3} -----------------------------------------------------------------
  {
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int hr = (4 * rg + i + kh) * HW + kw + r16;
          const u32x4 a = *(const u32x4*)(h1s + soff(hr, kq + 4 * ks));
          acc[i] = mfma(w2f[tap][ks], a, acc[i]);
        }
      }
      if (tap == 0) {
#pragma unroll
        for (int t = 5; t < 9; ++t)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) w2f[t][ks] = *(const u32x4*)(wrow2 + t * P + 32 * ks);
      }
    }
    BN_T(3);
    const int c = 16 * ct + 4 * kq;
    const f32x4 bc = *(const f32x4*)(bias_s + 64 + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * (4 * rg + i) + r16;
      *(u32x2*)(h2s + soff(m, c >> 3) + (c & 7) * 2) =
          pack4(fmaxf(acc[i][0] + bc[0], 0.f), fmaxf(acc[i][1] + bc[1], 0.f),
                fmaxf(acc[i][2] + bc[2], 0.f), fmaxf(acc[i][3] + bc[3], 0.f));
    }
  }
  // conv3 weights, first two k-steps, in flight across the barrier
  const int co0 = 64 * (wave & 3), pr = wave >> 2;
  const bf16* w3row = w3 + (long)(co0 + r16) * K3 + 8 * kq;
  u32x4 w3f[KS3][4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j) w3f[ks][j] = *(const u32x4*)(w3row + (long)16 * j * K3 + 32 * ks);
  __syncthreads();
  BN_T(4);

  // ---- phase C: y = relu([h2 (| x)] W3^T + b3 (+ x)); wave -> output channels 64 (w & 3) ..
  //      + 63 x output rows 4 (w >> 2) + {0..3}: each lane stores 8-byte runs, each pixel's
  //      128-byte channel range comes from one wave ---------------------------------------------
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS3; ++ks) {
    if (ks >= 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w3f[ks][j] = *(const u32x4*)(w3row + (long)16 * j * K3 + 32 * ks);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * (4 * pr + i) + r16;
      u32x4 a;
      if (ks < 2) {
        a = *(const u32x4*)(h2s + soff(m, kq + 4 * ks));
      } else {                                     // x at pixel (4 pr + i, r16): halo row
        const int hr = (4 * pr + i + 1) * HW + r16 + 1;
        a = *(const u32x4*)(xst + hr * 128 + (((kq + 4 * (ks - 2)) ^ ((hr >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(w3f[ks][j], a, acc[i][j]);
    }
  }
  BN_T(5);
  // epilogue, one output row (16 pixels x 64 channels) at a time: acc + b3 in fp32 through
  // this wave's LDS stage (h1s is dead), then 8 lanes per pixel read 8 channels each, add the
  // residual and store, so every global access is a 128-byte run per pixel
  float* stg = (float*)smem + wave * 16 * SST;
  f32x4 bj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bj[j] = *(const f32x4*)(bias_s + 128 + co0 + 16 * j + 4 * kq);
  const int pp0 = lane >> 3, c8 = (lane & 7) * 8;
  // the residual rows of all four output rows in flight at once (one exposed memory latency
  // instead of one per row: the MFMA registers of conv3 are dead here)
  u32x4 resv[4][2];
  if constexpr (!DS && BN_DIAG != 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long pix0 = ((long)n * H + y0 + 4 * pr + i) * W + x0;
#pragma unroll
      for (int it = 0; it < 2; ++it)
        resv[i][it] = *(const u32x4*)(x + (pix0 + pp0 + 8 * it) * CIN + co0 + c8);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long pix0 = ((long)n * H + y0 + 4 * pr + i) * W + x0;
    u32x4 res[2];
    if constexpr (!DS && BN_DIAG != 2) {
      res[0] = resv[i][0];
      res[1] = resv[i][1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bj[j][e];
      *(f32x4*)(stg + r16 * SST + 16 * j + 4 * kq) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's stage writes landed
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int pp = pp0 + 8 * it;
      const f32x4 lo = *(const f32x4*)(stg + pp * SST + c8);
      const f32x4 hi = *(const f32x4*)(stg + pp * SST + c8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (!DS && BN_DIAG != 2) {
        const bf16x8 r = __builtin_bit_cast(bf16x8, res[it]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)fmaxf(v[e], 0.f);
      *(bf16x8*)(y + (pix0 + pp) * CO + co0 + c8) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // stage reads done before reuse
  }
  BN_T(6);
}

template <bool DS>
constexpr size_t lds_bytes() { return lds_main<DS>() + 384 * 4; }   // + biases

template <int CIN, bool DS>
int launch(const void* x, int N, int H, int W, const void* w1, const float* b1, const void* w2,
           const float* b2, const void* w3, const float* b3, void* y, hipStream_t st) {
  auto kern = bottleneck_s1_kernel<CIN, DS>;
  constexpr size_t lds = lds_bytes<DS>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  const int blocks = N * (H / TH) * (W / TW);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(NT), lds, st, (const bf16*)x, H, W,
                     (const bf16*)w1, b1, (const bf16*)w2, b2, (const bf16*)w3, b3, (bf16*)y);
  return retr_check_launch("bottleneck_s1");
}

}  // namespace

#if BN_DIAG == 9
extern "C" int retr_bn_prof(void* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bn_prof), sizeof(g_bn_prof)) != hipSuccess;
}
#endif

extern "C" int retr_bottleneck_s1_fwd(int dtype, const void* x, int N, int H, int W, int Cin,
                                      const void* w1, const float* b1, const void* w2,
                                      const float* b2, const void* w3, const float* b3, int ds,
                                      void* y, void* stream) {
  RETR_REQUIRE(dtype == RETR_DTYPE_BF16, "bottleneck_s1: bf16 only");
  RETR_REQUIRE(H % TH == 0 && W % TW == 0, "bottleneck_s1: H %% 8, W %% 16 (H=%d W=%d)", H, W);
  RETR_REQUIRE((ds && Cin == 64) || (!ds && Cin == CO),
               "bottleneck_s1: Cin=%d ds=%d (64 with downsample | 256 identity)", Cin, ds);
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (ds) return launch<64, true>(x, N, H, W, w1, b1, w2, b2, w3, b3, y, st);
  return launch<256, false>(x, N, H, W, w1, b1, w2, b2, w3, b3, y, st);
}
