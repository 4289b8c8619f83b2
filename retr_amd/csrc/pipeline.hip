// RefCOCO encoder-input pipeline on the GPU: bbox crop / context masking,
// pad-to-square, antialiased bilinear resize, ColorJitter, ToTensor + Normalize, mask resize.
//
// Replaces the per-item PIL / torchvision path of RefCocoCaption.__getitem__
// (data_utils/refcoco.py:131-178) with the helpers of data_utils/utils.py:161-252 and the
// transforms of refcoco.py:14-46.  Host code (retr_amd/data_pipeline.py) decodes nothing on the
// GPU: it uploads the raw uint8 RGB images of a batch in one copy, plus per-item descriptors and
// the resampling coefficient tables it computes exactly as Pillow does (double precision ->
// 22-bit fixed point, libImaging/Resample.c); the kernels then reproduce Pillow's integer
// arithmetic bit for bit:
//   1. pipe_hpass: horizontal pass of the padded square image (never materialised: a pixel of
//      the D x D canvas is the crop / context pixel or 0), uint8 [D][S][3] per item;
//   2. pipe_vpass: vertical pass -> uint8 [S][S][3];
//   3. pipe_finish: one block per item applies the jitter ops in the drawn order (Pillow
//      ImageEnhance blends in float32, truncated / clipped to uint8; contrast blends towards the
//      rounded mean luma, a block reduction), then ToTensor + Normalize -> fp32 [3][S][S];
//   4. pipe_mask: the padded bool mask after torchvision's antialiased bilinear resize is True
//      wherever a nonzero filter tap covers a True pixel: evaluated per output pixel from the
//      tap windows and the (pad / context box) rectangles.
// HBM traffic: the raw images once, the [D][S][3] intermediate written + read, [S][S][3] u8 and
// the fp32 output; all byte / integer work (no MFMA).
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

constexpr int kPrec = 22;   // Pillow PRECISION_BITS for 8-bit images (32 - 8 - 2)

RETR_DEVICE unsigned char clip8(int v) {
  v >>= kPrec;
  return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pixel (r, c) of item it's padded D x D canvas (0 outside the pasted region / inside the
// zeroed context box), channel by channel
RETR_DEVICE void canvas_px(const unsigned char* src, const retr_pipe_item& it, int r, int c,
                           int (&px)[3]) {
  const int rr = r - it.oy, cc = c - it.ox;
  px[0] = px[1] = px[2] = 0;
  if ((unsigned)rr >= (unsigned)it.rh || (unsigned)cc >= (unsigned)it.rw) return;
  if (it.bw > 0 && rr >= it.by && rr < it.by + it.bh && cc >= it.bx && cc < it.bx + it.bw) return;
  const unsigned char* p = src + it.src_off + ((long)(it.y0 + rr) * it.W + (it.x0 + cc)) * 3;
  px[0] = p[0];
  px[1] = p[1];
  px[2] = p[2];
}

__global__ void __launch_bounds__(256)
pipe_hpass_kernel(const unsigned char* src, const retr_pipe_item* items, const int* coef,
                  unsigned char* tmp, int S) {
  const retr_pipe_item it = items[blockIdx.y];
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)it.D * S) return;
  const int r = (int)(idx / S), xx = (int)(idx - (long)r * S);
  const int* bounds = coef + it.coef_off;
  const int* kk = bounds + 2 * S + xx * it.ksize;
  const int xmin = bounds[2 * xx], n = bounds[2 * xx + 1];
  int acc[3] = {1 << (kPrec - 1), 1 << (kPrec - 1), 1 << (kPrec - 1)};
  if (r >= it.oy && r < it.oy + it.rh) {      // rows of the pad band are all zero
    for (int k = 0; k < n; ++k) {
      int px[3];
      canvas_px(src, it, r, xmin + k, px);
      const int w = kk[k];
      acc[0] += px[0] * w;
      acc[1] += px[1] * w;
      acc[2] += px[2] * w;
    }
  }
  unsigned char* o = tmp + it.tmp_off + idx * 3;
  o[0] = clip8(acc[0]);
  o[1] = clip8(acc[1]);
  o[2] = clip8(acc[2]);
}

__global__ void __launch_bounds__(256)
pipe_vpass_kernel(const retr_pipe_item* items, const int* coef, const unsigned char* tmp,
                  unsigned char* out, int S) {
  const retr_pipe_item it = items[blockIdx.y];
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)S * S) return;
  const int yy = (int)(idx / S), xx = (int)(idx - (long)yy * S);
  const int* bounds = coef + it.coef_off;
  const int* kk = bounds + 2 * S + yy * it.ksize;
  const int ymin = bounds[2 * yy], n = bounds[2 * yy + 1];
  int acc[3] = {1 << (kPrec - 1), 1 << (kPrec - 1), 1 << (kPrec - 1)};
  const unsigned char* t = tmp + it.tmp_off + ((long)ymin * S + xx) * 3;
  for (int k = 0; k < n; ++k) {
    const int w = kk[k];
    acc[0] += t[0] * w;
    acc[1] += t[1] * w;
    acc[2] += t[2] * w;
    t += (long)S * 3;
  }
  unsigned char* o = out + ((long)blockIdx.y * S * S + idx) * 3;
  o[0] = clip8(acc[0]);
  o[1] = clip8(acc[1]);
  o[2] = clip8(acc[2]);
}

// Pillow L = (R 19595 + G 38470 + B 7471 + 0x8000) >> 16
RETR_DEVICE int luma(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

// ImagingBlend(in1 = degenerate, in2 = image, alpha): float32 multiply then add, each rounded
// (no FMA contraction: HIP's __fmul_rn / __fadd_rn are plain operators that clang would fuse,
// and the fused result truncates to one less wherever d + a (v - d) lands just on an integer),
// truncated to uint8 for alpha in [0, 1], clipped otherwise
RETR_DEVICE int blend(int d, int v, float a) {
#pragma clang fp contract(off)
  const float t = (float)d + a * (float)(v - d);
  if (a >= 0.f && a <= 1.f) return (int)t;
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)t);
}

constexpr int kFinThreads = 1024;

__global__ void __launch_bounds__(kFinThreads)
pipe_finish_kernel(const retr_pipe_item* items, unsigned char* u8, float* out, int S,
                   float m0, float m1, float m2, float s0, float s1, float s2) {
  __shared__ long long red[kFinThreads / 64];
  const retr_pipe_item it = items[blockIdx.x];
  const long P = (long)S * S;
  unsigned char* img = u8 + (long)blockIdx.x * P * 3;
  const int tid = threadIdx.x;
  for (int slot = 0; slot < 3; ++slot) {
    const int op = (it.ops >> (4 * slot)) & 15;
    if (op == 0) break;
    const float f = it.f[slot];
    int mean = 0;
    if (op == 2) {   // contrast: int(mean(L) + 0.5) over the whole image
      long long s = 0;
      for (long p = tid; p < P; p += kFinThreads) {
        const unsigned char* q = img + p * 3;
        s += luma(q[0], q[1], q[2]);
      }
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if ((tid & 63) == 0) red[tid >> 6] = s;
      __syncthreads();
      long long tot = 0;
      for (int w = 0; w < kFinThreads / 64; ++w) tot += red[w];
      mean = (int)((double)tot / (double)P + 0.5);
      __syncthreads();
    }
    // every thread rewrites only its own pixels (p = tid + k * 1024), so the ops chain needs no
    // cross-thread visibility beyond the contrast reduction above
    for (long p = tid; p < P; p += kFinThreads) {
      unsigned char* q = img + p * 3;
      const int r = q[0], g = q[1], b = q[2];
      int d0 = 0, d1 = 0, d2 = 0;
      if (op == 2) d0 = d1 = d2 = mean;
      if (op == 3) d0 = d1 = d2 = luma(r, g, b);
      q[0] = (unsigned char)blend(d0, r, f);
      q[1] = (unsigned char)blend(d1, g, f);
      q[2] = (unsigned char)blend(d2, b, f);
    }
  }
  // ToTensor (/ 255) + Normalize((x - mean) / std), fp32 NCHW
  float* o = out + (long)blockIdx.x * 3 * P;
  for (long p = tid; p < P; p += kFinThreads) {
    const unsigned char* q = img + p * 3;
    o[p] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)q[0], 255.f), m0), s0);
    o[P + p] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)q[1], 255.f), m1), s1);
    o[2 * P + p] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)q[2], 255.f), m2), s2);
  }
}

__global__ void __launch_bounds__(256)
pipe_mask_kernel(const retr_pipe_item* items, const int* win, unsigned char* mask, int S) {
  const retr_pipe_item it = items[blockIdx.y];
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)S * S) return;
  const int yy = (int)(idx / S), xx = (int)(idx - (long)yy * S);
  const int* w = win + it.win_off;
  const int ylo = w[2 * yy], yhi = w[2 * yy + 1], xlo = w[2 * xx], xhi = w[2 * xx + 1];
  bool m = false;
  if (yhi > ylo && xhi > xlo) {
    // pad band: the window leaves the pasted region [my, my + rh) x [mx, mx + rw)
    m = ylo < it.my || yhi > it.my + it.rh || xlo < it.mx || xhi > it.mx + it.rw;
    // context: the window meets the masked box
    if (!m && it.bw > 0) {
      const int by0 = it.my + it.by, bx0 = it.mx + it.bx;
      m = ylo < by0 + it.bh && yhi > by0 && xlo < bx0 + it.bw && xhi > bx0;
    }
  }
  mask[(long)blockIdx.y * S * S + idx] = m ? 1 : 0;
}

}  // namespace

extern "C" {

int retr_pipe_run(const unsigned char* src, const retr_pipe_item* items, int n, const int* coef,
                  const int* win, unsigned char* tmp, int max_d, unsigned char* u8, float* out,
                  unsigned char* mask, int S, const float* mean, const float* std_,
                  void* stream) {
  if (n == 0) return 0;
  RETR_REQUIRE(S > 0 && max_d > 0, "pipe_run: S=%d max_d=%d", S, max_d);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(pipe_hpass_kernel, dim3((unsigned)cdiv((long)max_d * S, 256), n), dim3(256),
                     0, st, src, items, coef, tmp, S);
  if (int e = retr_check_launch("pipe_hpass")) return e;
  hipLaunchKernelGGL(pipe_vpass_kernel, dim3((unsigned)cdiv((long)S * S, 256), n), dim3(256), 0,
                     st, items, coef, tmp, u8, S);
  if (int e = retr_check_launch("pipe_vpass")) return e;
  hipLaunchKernelGGL(pipe_finish_kernel, dim3(n), dim3(kFinThreads), 0, st, items, u8, out, S,
                     mean[0], mean[1], mean[2], std_[0], std_[1], std_[2]);
  if (int e = retr_check_launch("pipe_finish")) return e;
  if (mask) {
    hipLaunchKernelGGL(pipe_mask_kernel, dim3((unsigned)cdiv((long)S * S, 256), n), dim3(256), 0,
                       st, items, win, mask, S);
    if (int e = retr_check_launch("pipe_mask")) return e;
  }
  return 0;
}

}  // extern "C"
