// Fused ResNet stem forward for the frozen stem of the bf16 backbone (torchvision conv1 + bn1 +
// relu + maxpool, models/backbone.py:85-95 via IntermediateLayerGetter; frozen by
// models/backbone.py:58-60, so backward never needs the conv1 output):
//
//   s = relu(conv4x4_s1_p2(x_s2d, W2) + b)      the space-to-depth form of the 7x7 stride-2 conv
//                                                (misc.hip nchw_to_s2d16 / stem_s2d_weights)
//   y = maxpool3x3_s2_p1(s)                      [N, ceil(H2/2), ceil(W2/2), 64]
//
// The unfused path wrote s (N x H2 x W2 x 64 bf16: 210 MB at cfg2) and read it back for the
// pool; here s lives only in LDS.  One 512-thread block (8 waves, 2 blocks per CU) per 8 x 16
// pooled tile of one image: the tile's pooling windows cover 17 x 33 conv pixels (561, 36
// position tiles of 16), which read a 20 x 36 pixel patch of the 32-byte s2d input, loaded once
// into LDS by LDS-DMA (zero page outside the image = the conv's zero padding).
//
// Numerics: every conv pixel runs the same v_mfma_f32_16x16x32_bf16 chain over K = (tap, ch)
// ascending in 32-deep steps (two taps per step) as the implicit-GEMM conv kernel, from a zero
// accumulator, then acc + bias, ReLU, bf16 -- the unfused conv's epilogue -- and the pool takes
// the max of those bf16 values over the window's in-image pixels (maxpool8_kernel), so the
// output equals the two-launch path bitwise.  Products are computed transposed (weights = A
// operand, positions = B): a lane's accumulator holds 4 consecutive output channels of one
// position, written to the LDS staging image as one 8-byte run.
//
// The 64 output channels go in two passes of 32 (staging 561 x 80 B = 44.9 KB, so the block
// fits twice per CU next to the 24 KB patch): per pass each wave computes 4 position tiles x 2
// channel tiles + one (position, channel) tile of the 4 left over (72 units / 8 waves), then the
// block pools its 128 pooled pixels x 32 channels (one 16-byte chunk per thread).
#include "common.hpp"
#include "../../include/retr_hip.h"

#ifndef STEM_DIAG
#define STEM_DIAG 0      // 9: per-wave phase stamps (A/B tooling only: tools/stem_micro.sh)
#endif

namespace {

#if STEM_DIAG == 9
__device__ unsigned long long g_stem_prof[4096 * 8 * 8];
#define STEM_T(k)                                                                        \
  if (lane == 0 && blockIdx.x < 4096)                                                    \
    g_stem_prof[(blockIdx.x * 8 + wave) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define STEM_T(k)
#endif

constexpr int TPH = 8, TPW = 16;                  // pooled tile
constexpr int CR = 2 * TPH + 1, CC = 2 * TPW + 1; // conv pixels under the tile's windows
constexpr int NPX = CR * CC;                      // 561
constexpr int NTILE = (NPX + 15) / 16;            // 36 position tiles
constexpr int IR = CR + 3, IC = CC + 3;           // 20 x 36 input pixels (4x4 taps)
constexpr int NCHUNK = IR * IC * 2;               // 1440 16-byte chunks
constexpr int NT = 512;
constexpr int ROUNDS = (NCHUNK + NT - 1) / NT;    // 3 DMA instructions per lane
constexpr int PATCH = ROUNDS * NT * 16;           // 24576 B (tail chunks land past the patch)
constexpr int SROW = 80;                          // staging row: 32 channels + 16 B pad
constexpr int LDS = PATCH + NPX * SROW;           // 69456 B
constexpr int CO = 64, K = 256;
static_assert(NTILE == 36 && NCHUNK <= ROUNDS * NT, "tile geometry");

static __device__ __attribute__((aligned(64))) unsigned int g_stem_zero[16];

RETR_DEVICE f32x4 mfma(const u32x4& w, const u32x4& x, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w),
                                                 __builtin_bit_cast(bf16x8, x), acc, 0, 0, 0);
}

RETR_DEVICE void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                   0, 0);
}

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// one (position tile, channel tile) product: 8 K-steps, the B fragment of step s = taps
// (2s, 2s + 1) of the lane's position (lanes 32-63 take the odd tap: +32 B in the patch row)
template <int NCT>
RETR_DEVICE void tile_mma(const char* patch, int base, const u32x4 (&wf)[2][8], int ct0,
                          f32x4 (&acc)[NCT]) {
#pragma unroll
  for (int j = 0; j < NCT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int off = ((s >> 1) * IC + 2 * (s & 1)) * 32;
    const u32x4 b = *(const u32x4*)(patch + base + off);
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[j] = mfma(wf[ct0 + j][s], b, acc[j]);
  }
}

__global__ void __launch_bounds__(NT, 4)
stem_pool_kernel(const bf16* __restrict__ x, int H2, int W2, const bf16* __restrict__ w,
                 const float* __restrict__ bias, bf16* __restrict__ y, int PH, int PW,
                 int tiles_h, int tiles_w) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* patch = smem;
  char* stg = smem + PATCH;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  // XCD-aware order: consecutive tiles (sharing patch rows) on one XCD's L2
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int per_img = tiles_h * tiles_w;
  const int n = bid / per_img;
  const int rem = bid - n * per_img;
  const int p0 = (rem / tiles_w) * TPH, q0 = (rem % tiles_w) * TPW;
  const int r0 = 2 * p0 - 1, c0 = 2 * q0 - 1;     // conv pixel (0, 0) of the tile
  const bf16* ximg = x + (long)n * H2 * W2 * 16;
  STEM_T(0);

  // ---- patch: input rows r0 - 2 .. r0 + CR, cols c0 - 2 .. c0 + CC, [IR][IC][32 B] ----------
#pragma unroll
  for (int k = 0; k < ROUNDS; ++k) {
    const int c = k * NT + tid;
    const int prow = c / (IC * 2), rc = c - prow * (IC * 2);
    const int gr = r0 - 2 + prow, gc = c0 - 2 + (rc >> 1);
    const bool ok = c < NCHUNK && (unsigned)gr < (unsigned)H2 && (unsigned)gc < (unsigned)W2;
    const void* src = ok ? (const void*)(ximg + ((long)gr * W2 + gc) * 16 + 8 * (rc & 1))
                         : (const void*)g_stem_zero;
    glds16(src, patch + (k * NT + wave * 64) * 16);
  }

  // unit split: tiles wave + 8 i (i < 4) with both channel tiles of the pass, plus the single
  // (tile 32 + wave / 2, channel tile wave & 1)
  int base[5], pix[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int t = i < 4 ? wave + 8 * i : 32 + (wave >> 1);
    const int p = 16 * t + r16;
    pix[i] = p;
    const int pc = p < NPX ? p : NPX - 1;
    const int r = pc / CC, cc = pc - r * CC;
    base[i] = (r * IC + cc) * 32 + (kq & 1) * 16 + (kq >> 1) * 32;
  }

#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // W2 fragments of the pass's two channel tiles (A operand: row = channel, 8 K at 8 kq)
    u32x4 wf[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 8; ++s)
        wf[j][s] = *(const u32x4*)(w + (long)(32 * h + 16 * j + r16) * K + 32 * s + 8 * kq);
    float bv[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[j][e] = bias[32 * h + 16 * j + 4 * kq + e];
    __syncthreads();       // pass 0: the patch landed; pass 1: pass 0's pool read the staging
    STEM_T(1 + 3 * h);

    auto emit = [&](int p, int j, const f32x4& a) {
      if (p < NPX) {
        *(u32x2*)(stg + p * SROW + (16 * j + 4 * kq) * 2) = __builtin_bit_cast(
            u32x2, bf16x4{(bf16)fmaxf(a[0] + bv[j][0], 0.f), (bf16)fmaxf(a[1] + bv[j][1], 0.f),
                          (bf16)fmaxf(a[2] + bv[j][2], 0.f), (bf16)fmaxf(a[3] + bv[j][3], 0.f)});
      }
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 acc[2];
      tile_mma<2>(patch, base[i], wf, 0, acc);
      emit(pix[i], 0, acc[0]);
      emit(pix[i], 1, acc[1]);
    }
    {
      f32x4 acc[1];
      if (wave & 1) {
        tile_mma<1>(patch, base[4], wf, 1, acc);
        emit(pix[4], 1, acc[0]);
      } else {
        tile_mma<1>(patch, base[4], wf, 0, acc);
        emit(pix[4], 0, acc[0]);
      }
    }
    STEM_T(2 + 3 * h);
    __syncthreads();

    // ---- pool: pooled pixel tid / 4 of the tile, channels 32 h + 8 (tid & 3) .. + 8 ---------
    {
      const int pp = tid >> 2, ch = tid & 3;
      const int pl = pp >> 4, ql = pp & 15;
      const int p = p0 + pl, q = q0 + ql;
      if (p < PH && q < PW) {
        float m[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
        for (int dr = 0; dr < 3; ++dr) {
          const int r = 2 * pl + dr;
          if ((unsigned)(r0 + r) >= (unsigned)H2) continue;
#pragma unroll
          for (int dc = 0; dc < 3; ++dc) {
            const int c = 2 * ql + dc;
            if ((unsigned)(c0 + c) >= (unsigned)W2) continue;
            const bf16x8 v = *(const bf16x8*)(stg + (r * CC + c) * SROW + ch * 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
          }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
        *(bf16x8*)(y + (((long)n * PH + p) * PW + q) * CO + 32 * h + 8 * ch) = o;
      }
    }
    STEM_T(3 + 3 * h);
  }
}

}  // namespace

extern "C" {

int retr_stem_pool_fwd(int dtype, const void* x, int N, int H2, int W2, const void* w,
                       const float* bias, void* y, int Co, void* stream) {
  RETR_REQUIRE(dtype == RETR_DTYPE_BF16, "stem_pool_fwd: bf16 only");
  RETR_REQUIRE(Co == CO, "stem_pool_fwd: Co=%d (64)", Co);
  RETR_REQUIRE(N > 0 && H2 > 0 && W2 > 0, "stem_pool_fwd: empty input %dx%dx%d", N, H2, W2);
  const int PH = (H2 - 1) / 2 + 1, PW = (W2 - 1) / 2 + 1;
  const int tiles_h = (PH + TPH - 1) / TPH, tiles_w = (PW + TPW - 1) / TPW;
  const long blocks = (long)N * tiles_h * tiles_w;
  RETR_REQUIRE(blocks < (1L << 31), "stem_pool_fwd: grid too large");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)stem_pool_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL(stem_pool_kernel, dim3((unsigned)blocks), dim3(NT), LDS,
                     (hipStream_t)stream, (const bf16*)x, H2, W2, (const bf16*)w, bias, (bf16*)y,
                     PH, PW, tiles_h, tiles_w);
  return retr_check_launch("stem_pool_fwd");
}

#if STEM_DIAG == 9
int retr_stem_prof(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stem_prof), sizeof(g_stem_prof));
}
#endif

}  // extern "C"
