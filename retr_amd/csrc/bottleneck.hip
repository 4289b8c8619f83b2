// Fused stride-1 ResNet bottleneck forward for the frozen layer1 of ResNet-50/101
// (torchvision Bottleneck via models/backbone.py:65, frozen by models/backbone.py:58-60, so no
// activation of it is ever needed by backward):
//
//   h1 = relu(x W1^T + b1)                     1x1, Cin -> 64        (FrozenBN folded)
//   h2 = relu(conv3x3(h1, W2) + b2)            3x3, pad 1, 64 -> 64
//   y  = relu(h2 W3^T + b3 + x)                1x1, 64 -> 256, identity residual (Cin = 256)
//   y  = relu([h2 | x] [W3 | Wds]^T + b3 + bds)  first block: 1x1 downsample folded in (Cin 64)
//
// One 256-thread block per 8 x 16 output tile of one image.  h1 (on the tile's 10 x 18 halo)
// and h2 never leave LDS: the unfused path wrote and re-read both (2 x 2 x 52 MB per block at
// cfg2) and read x twice (conv1 and the residual, 2 x 210 MB).  Every product runs the same
// v_mfma_f32_16x16x32_bf16 chain over K in the same order as the unfused implicit-GEMM
// kernels (K ascending in 32-deep steps; conv2's K is tap-major (kh, kw, ci) like the packed
// weights [Co][3][3][Ci]), with the same bf16 roundings of h1 / h2 and the same epilogue order
// (acc + bias (+ residual), ReLU, bf16), so the result equals the three-launch path bitwise.
//
//   phase A  h1 on the halo: 12 row tiles (192 >= 180 positions) x 4 column tiles, wave w owns
//            row tiles 3w..3w+2; x fragments straight from global memory (each position is
//            read by one wave only), W1 fragments from L2; positions outside the image are
//            written as 0 (conv2's zero padding applies to h1, not relu(b1)).
//   phase B  h2: wave w owns output channels 16w..16w+15 over all 128 pixels; A fragments of
//            tap (kh, kw) are the halo rows (py + kh) * 18 + kw + px of h1.
//   phase C  y: wave w owns output channels 64w..64w+63; fp32 (acc + bias) staged through LDS
//            so the residual load, ReLU, bf16 conversion and store run 8 channels (16 bytes)
//            per lane.
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

constexpr int TH = 8, TW = 16;                    // output tile
constexpr int HH = TH + 2, HW = TW + 2;           // halo
constexpr int NHALO = HH * HW;                    // 180
constexpr int P = 64;                             // bottleneck width (planes)
constexpr int CO = 256;                           // block output channels

RETR_DEVICE f32x4 mfma(const u32x4& a, const u32x4& b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}

// [rows][64] bf16 image, 128-byte rows, 16-byte chunk c of row r at chunk c ^ ((r >> 1) & 7)
// (the gemm.hpp swizzle: the 16 rows x 4 chunks of a fragment read hit distinct banks)
RETR_DEVICE int soff(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

RETR_DEVICE u32x4 ld16g(const bf16* p, bool ok) {
  return ok ? *(const u32x4*)p : u32x4{0u, 0u, 0u, 0u};
}

template <int CIN, bool DS>
__global__ void __launch_bounds__(256, 2)
bottleneck_s1_kernel(const bf16* __restrict__ x, int H, int W, const bf16* __restrict__ w1,
                     const float* __restrict__ b1, const bf16* __restrict__ w2,
                     const float* __restrict__ b2, const bf16* __restrict__ w3,
                     const float* __restrict__ b3, bf16* __restrict__ y) {
  static_assert(CIN % 32 == 0 && (DS ? CIN == 64 : CIN == CO), "shape");
  constexpr int K3 = P + (DS ? CIN : 0);          // conv3 (+ downsample) reduction
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* h1s = smem;                               // [192][64] bf16
  char* h2s = smem + 192 * 128;                   // [128][64] bf16
  float* stg = (float*)smem;                      // phase C: [4 waves][64][64] fp32 (aliases)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;      // fragment row, 8-element k chunk
  const int tiles_w = W / TW, tiles_h = H / TH;
  const int bid = blockIdx.x;
  const int n = bid / (tiles_h * tiles_w);
  const int rem = bid - n * tiles_h * tiles_w;
  const int y0 = (rem / tiles_w) * TH, x0 = (rem % tiles_w) * TW;
  const bf16* ximg = x + (long)n * H * W * CIN;

  // ---- phase A: h1 on the halo ------------------------------------------------------------
  {
    f32x4 acc[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* arow[3];
    bool aok[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = 16 * (3 * wave + i) + r16;
      const int hy = p / HW, hx = p - hy * HW;
      const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
      aok[i] = p < NHALO && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      arow[i] = ximg + ((long)(aok[i] ? iy : 0) * W + (aok[i] ? ix : 0)) * CIN + 8 * kq;
    }
#pragma unroll
    for (int ks = 0; ks < CIN / 32; ++ks) {
      u32x4 a[3], b[4];
#pragma unroll
      for (int i = 0; i < 3; ++i) a[i] = ld16g(arow[i] + 32 * ks, aok[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *(const u32x4*)(w1 + (long)(16 * j + r16) * CIN + 32 * ks + 8 * kq);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
    // epilogue: relu(acc + b1) -> bf16, 0 outside the image; C layout: row 4 kq + e, col r16
    float bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = b1[16 * j + r16];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = 16 * (3 * wave + i) + 4 * kq + e;
        const int hy = p / HW, hx = p - hy * HW;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool ok = p < NHALO && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 16 * j + r16;
          const float v = ok ? fmaxf(acc[i][j][e] + bj[j], 0.f) : 0.f;
          *(bf16*)(h1s + soff(p, c >> 3) + (c & 7) * 2) = (bf16)v;
        }
      }
  }
  __syncthreads();

  // ---- phase B: h2 = relu(conv3x3(h1) + b2), wave w -> channels 16w .. 16w+15 ---------------
  {
    f32x4 acc[TH];
#pragma unroll
    for (int i = 0; i < TH; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* wrow = w2 + (long)(16 * wave + r16) * 9 * P + 8 * kq;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const u32x4 b = *(const u32x4*)(wrow + tap * P + 32 * ks);
#pragma unroll
        for (int i = 0; i < TH; ++i) {
          const int hr = (i + kh) * HW + kw + r16;
          const u32x4 a = *(const u32x4*)(h1s + soff(hr, kq + 4 * ks));
          acc[i] = mfma(a, b, acc[i]);
        }
      }
    }
    const int c = 16 * wave + r16;
    const float bc = b2[c];
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = 16 * i + 4 * kq + e;
        *(bf16*)(h2s + soff(m, c >> 3) + (c & 7) * 2) = (bf16)fmaxf(acc[i][e] + bc, 0.f);
      }
  }
  __syncthreads();

  // ---- phase C: y = relu([h2 (| x)] W3^T + b3 (+ x)), wave w -> channels 64w .. 64w+63 --------
  f32x4 acc[TH][4];
#pragma unroll
  for (int i = 0; i < TH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int cw = 64 * wave;
#pragma unroll
  for (int ks = 0; ks < K3 / 32; ++ks) {
    u32x4 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *(const u32x4*)(w3 + (long)(cw + 16 * j + r16) * K3 + 32 * ks + 8 * kq);
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      u32x4 a;
      if (ks < P / 32) {
        a = *(const u32x4*)(h2s + soff(16 * i + r16, kq + 4 * ks));
      } else {                                   // downsample operand: x at the output pixel
        a = *(const u32x4*)(ximg + ((long)(y0 + i) * W + x0 + r16) * CIN + 32 * (ks - P / 32) + 8 * kq);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(a, b[j], acc[i][j]);
    }
  }
  __syncthreads();                               // every wave is done reading h2s: reuse LDS
  float bj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bj[j] = b3[cw + 16 * j + r16];
  float* ws = stg + wave * 64 * 68;              // this wave's [64 rows][64 (+4 pad)] fp32
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    // rows 64 half .. 64 half + 63 of the tile (output rows py = 4 half .. 4 half + 3)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ws[(16 * i + 4 * kq + e) * 68 + 16 * j + r16] = acc[4 * half + i][j][e] + bj[j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS writes landed
    // 64 rows x 8 chunks of 8 channels = 512 chunks, 8 per lane
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int q = lane + 64 * it;
      const int rr = q >> 3, c8 = (q & 7) * 8;
      const int m = 64 * half + rr;
      const int py = m >> 4, px = m & 15;
      const long pix = ((long)n * H + y0 + py) * W + x0 + px;
      const f32x4 lo = *(const f32x4*)(ws + rr * 68 + c8);
      const f32x4 hi = *(const f32x4*)(ws + rr * 68 + c8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (!DS) {
        const bf16x8 r = *(const bf16x8*)(x + pix * CIN + cw + c8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)fmaxf(v[e], 0.f);
      *(bf16x8*)(y + pix * CO + cw + c8) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next half
  }
}

constexpr size_t kLds = 4 * 64 * 68 * 4;          // 69632 B (phase C staging >= h1s + h2s)
static_assert(kLds >= 192 * 128 + 128 * 128, "LDS regions");

template <int CIN, bool DS>
int launch(const void* x, int N, int H, int W, const void* w1, const float* b1, const void* w2,
           const float* b2, const void* w3, const float* b3, void* y, hipStream_t st) {
  auto kern = bottleneck_s1_kernel<CIN, DS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kLds);
    attr = true;
  }
  const int blocks = N * (H / TH) * (W / TW);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), kLds, st, (const bf16*)x, H, W,
                     (const bf16*)w1, b1, (const bf16*)w2, b2, (const bf16*)w3, b3, (bf16*)y);
  return retr_check_launch("bottleneck_s1");
}

}  // namespace

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
