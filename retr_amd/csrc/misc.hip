// Small streaming kernels around the hot path: image layout change, stem max-pool, mask
// down-sampling, dropout backward, casts and position-embedding gradient reduction.
#include "common.hpp"
#include "epilogues.hpp"
#include "../../include/retr_hip.h"

namespace {

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* x, T* y, int N, int C, int H, int W, int Cp) {
  long total = (long)N * H * W * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = i % Cp;
    long pix = i / Cp;
    int w = pix % W;
    long t = pix / W;
    int h = t % H;
    int n = (int)(t / H);
    float v = c < C ? x[(((long)n * C + c) * H + h) * W + w] : 0.f;
    y[i] = from_f<T>(v);
  }
}

// bf16, Cp == 8: one thread per pixel reads its C (<= 8) channel planes (coalesced along w) and
// writes the pixel's 16-byte chunk
__global__ void nchw_to_nhwc8_kernel(const float* x, bf16* y, int N, int C, int H, int W) {
  const long HW = (long)H * W, total = (long)N * HW;
  for (long pix = blockIdx.x * (long)blockDim.x + threadIdx.x; pix < total;
       pix += (long)gridDim.x * blockDim.x) {
    const long n = pix / HW, hw = pix - n * HW;
    bf16x8 o;
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = (bf16)(c < C ? x[(n * C + c) * HW + hw] : 0.f);
    *(bf16x8*)(y + pix * 8) = o;
  }
}

// bf16 space-to-depth stem input: y[n][Y][X][(dy * 2 + dx) * 3 + c] = x[n][c][2Y + dy][2X + dx]
// (12 channels, 4 zero pad channels -> one 32-byte pixel).  The 7x7 stride-2 stem becomes a 4x4
// stride-1 conv over 16 channels (K = 256 instead of 7 * 7 * 8 = 392) on half the input bytes.
__global__ void nchw_to_s2d16_kernel(const float* x, bf16* y, int N, int H, int W) {
  constexpr int C = 3;
  const int H2 = H / 2, W2 = W / 2;
  const long HW = (long)H * W, P2 = (long)H2 * W2, total = (long)N * P2;
  for (long pix = blockIdx.x * (long)blockDim.x + threadIdx.x; pix < total;
       pix += (long)gridDim.x * blockDim.x) {
    const long n = pix / P2, rem = pix - n * P2;
    const int Y = (int)(rem / W2), X = (int)(rem - (long)Y * W2);
    bf16x8 o[2];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[1][e] = (bf16)0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const float2 v = *(const float2*)(x + (n * C + c) * HW + (long)(2 * Y + dy) * W + 2 * X);
        const int q0 = (dy * 2) * C + c, q1 = (dy * 2 + 1) * C + c;
        o[q0 >> 3][q0 & 7] = (bf16)v.x;
        o[q1 >> 3][q1 & 7] = (bf16)v.y;
      }
    bf16x8* dst = (bf16x8*)(y + pix * 16);
    dst[0] = o[0];
    dst[1] = o[1];
  }
}

// the stem's packed 7x7 weights [Co][7][7][Cp] re-laid for the space-to-depth input:
// w2[co][i][j][(dy * 2 + dx) * 3 + c] = wp[co][2i + dy - 1][2j + dx - 1][c] (0 off the taps)
__global__ void stem_s2d_weights_kernel(const bf16* wp, bf16* w2, int Co, int Cp) {
  const int total = Co * 4 * 4 * 16;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int ch = i & 15, j = (i >> 4) & 3, ii = (i >> 6) & 3, co = i >> 8;
    float v = 0.f;
    if (ch < 12) {
      const int q = ch / 3, c = ch - 3 * q;
      const int kh = 2 * ii + (q >> 1) - 1, kw = 2 * j + (q & 1) - 1;
      if (kh >= 0 && kw >= 0 && kh < 7 && kw < 7) v = (float)wp[((co * 7 + kh) * 7 + kw) * Cp + c];
    }
    w2[i] = (bf16)v;
  }
}

// bf16 MaxPool2d(3, 2, 1) NHWC, C % 8 == 0: one thread per (output pixel, 8 channels), 16-byte
// loads of the 3x3 window and one 16-byte store
__global__ void maxpool8_kernel(const bf16* x, bf16* y, int N, int H, int W, int C, int OH,
                                int OW) {
  const int C8 = C / 8;
  const long total = (long)N * OH * OW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long pix = i / C8;
    const int ow = (int)(pix % OW);
    const long t = pix / OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = ow * 2 - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const bf16x8 v = *(const bf16x8*)(x + (((long)n * H + ih) * W + iw) * C + 8 * c8);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
    *(bf16x8*)(y + pix * C + 8 * c8) = o;
  }
}

// MaxPool2d(kernel 3, stride 2, padding 1) NHWC; padding acts as -inf.
template <typename T>
__global__ void maxpool_kernel(const T* x, T* y, int N, int H, int W, int C, int OH, int OW) {
  long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = i % C;
    long pix = i / C;
    int ow = pix % OW;
    long t = pix / OW;
    int oh = t % OH;
    int n = (int)(t / OH);
    float m = -INFINITY;
    for (int kh = 0; kh < 3; ++kh) {
      int ih = oh * 2 - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        int iw = ow * 2 - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        m = fmaxf(m, to_f(x[(((long)n * H + ih) * W + iw) * C + c]));
      }
    }
    y[i] = from_f<T>(m);
  }
}

// torch 'nearest' (legacy): src = min(floor(dst * (float)in/out), in-1)
__global__ void mask_nearest_kernel(const unsigned char* m, unsigned char* out, int N, int H,
                                    int W, int h, int w) {
  long total = (long)N * h * w;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= total) return;
  int x = i % w;
  long t = i / w;
  int y = t % h;
  int n = (int)(t / h);
  float sh = (float)H / (float)h, sw = (float)W / (float)w;
  int sy = min((int)floorf(y * sh), H - 1), sx = min((int)floorf(x * sw), W - 1);
  out[i] = m[((long)n * H + sy) * W + sx] ? 1 : 0;
}

template <typename TO>
__global__ void dropout_apply_kernel(const float* x, long ldx, TO* y, long ldy, int M, int N,
                                     DropoutParams dp) {
  // 8 consecutive columns per thread (N % 8 == 0 and 16-byte aligned rows: vector path)
  const int cpr = (N + 7) / 8;
  const long total = (long)M * cpr;
  const uint64_t seed = dp.thresh ? dp_seed(dp) : 0ull;
  const uint32_t th16 = drop_th16(dp.thresh);
  const bool vec = (N % 8 == 0) && (ldx % 4 == 0) && (ldy % 8 == 0);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / cpr), n = (int)(i - (long)m * cpr) * 8;
    const uint32_t km = dp.thresh ? drop_keep8(drop_row_key(seed, (uint32_t)m), (uint32_t)n, th16)
                                  : 0xffu;
    const float* xr = x + (long)m * ldx + n;
    TO* yr = y + (long)m * ldy + n;
    if (vec) {
      float v[8];
      const f32x4 a = *(const f32x4*)xr, b = *(const f32x4*)(xr + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = a[e], v[e + 4] = b[e];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = ((km >> e) & 1u) ? (dp.thresh ? v[e] * dp.scale : v[e]) : 0.f;
      if constexpr (sizeof(TO) == 2) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
        *(bf16x8*)yr = o;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) yr[e] = from_f<TO>(v[e]);
      }
    } else {
      for (int e = 0; e < 8 && n + e < N; ++e) {
        float v = xr[e];
        if (dp.thresh) v = ((km >> e) & 1u) ? v * dp.scale : 0.f;
        yr[e] = from_f<TO>(v);
      }
    }
  }
}

template <typename T>
__global__ void cast_kernel(const float* x, T* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = from_f<T>(x[i]);
}

template <typename T>
__global__ void pos_grad_kernel(const T* d, long ld, int M, int C, int period, float* dpos,
                                int acc) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)period * C) return;
  int c = i % C, p = (int)(i / C);
  float s = 0.f;
  for (int m = p; m < M; m += period) s += to_f(d[(long)m * ld + c]);
  float* o = dpos + (long)p * C + c;
  *o = (acc ? *o : 0.f) + s;
}

// 8 consecutive columns per thread with 16-byte loads, and the rows of one position loaded 8
// at a time before they are added (in row order, as pos_grad_kernel: bitwise the same sums) --
// the scalar loop kept one dependent 2-byte load per row in flight (7 us per call at cfg2)
template <typename T>
__global__ void pos_grad8_kernel(const T* d, long ld, int M, int C, int period, float* dpos,
                                 int acc) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c8 = C / 8;
  if (i >= (long)period * c8) return;
  const int c = (int)(i % c8) * 8, p = (int)(i / c8);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int m = p;
  for (; m + 7 * period < M; m += 8 * period) {
    float v[8][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) retr::load8<T>(d + (long)(m + u * period) * ld + c, v[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[u][e];
  }
  for (; m < M; m += period) {
    float v[8];
    retr::load8<T>(d + (long)m * ld + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += v[e];
  }
  float* o = dpos + (long)p * C + c;
  float cur[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // (0 + s: the zero-filled sums)
  if (acc) retr::load8<float>(o, cur);
#pragma unroll
  for (int e = 0; e < 8; ++e) cur[e] += s[e];
  retr::store8<float>(o, cur);
}

// Several position-gradient contributions into one buffer in one launch (the decoder's query
// positions: 12 blocks per step).  Thread (j, i) of a block forms item i's batch sum for chunk
// j exactly as pos_grad8_kernel does (same loop, same order), the sums meet in LDS, and chunk
// j's thread 0 adds them to dpos in item order: bitwise the sequence of per-item launches.
constexpr int kPosMulti = 16;                     // items per launch
struct PosItems {
  const void* d[kPosMulti];
  long ld[kPosMulti];
  int M[kPosMulti];
  int n;
};
template <typename T>
__global__ void __launch_bounds__(256) pos_grad_multi_kernel(PosItems it, int C, int period,
                                                             float* dpos, int acc) {
  __shared__ float sums[kPosMulti][16][8];
  const int j = threadIdx.x & 15, i = threadIdx.x >> 4;   // 16 chunks x 16 items per block
  const int c8 = C / 8;
  const long q = (long)blockIdx.x * 16 + j;
  const bool okq = q < (long)period * c8;
  const int c = okq ? (int)(q % c8) * 8 : 0, p = okq ? (int)(q / c8) : 0;
  if (okq && i < it.n) {
    const T* d = (const T*)it.d[i];
    const long ld = it.ld[i];
    const int M = it.M[i];
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int m = p;
    for (; m + 7 * period < M; m += 8 * period) {
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) retr::load8<T>(d + (long)(m + u * period) * ld + c, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += v[u][e];
    }
    for (; m < M; m += period) {
      float v[8];
      retr::load8<T>(d + (long)m * ld + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sums[i][j][e] = s[e];
  }
  __syncthreads();
  if (!okq || i != 0) return;
  float* o = dpos + (long)p * C + c;
  float cur[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (acc) retr::load8<float>(o, cur);
  for (int k = 0; k < it.n; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) cur[e] += sums[k][j][e];
  retr::store8<float>(o, cur);
}

int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

}  // namespace

extern "C" {

int retr_nchw_to_nhwc(int dtype, const float* x, void* y, int N, int C, int H, int W, int Cp,
                      void* stream) {
  long total = (long)N * H * W * Cp;
  if (total == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    if (Cp == 8) {
      const long pixels = (long)N * H * W;
      hipLaunchKernelGGL(nchw_to_nhwc8_kernel, dim3(grid_for(pixels)), dim3(256), 0, st, x, (bf16*)y, N, C, H, W);
    } else {
      hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, x, (bf16*)y, N, C, H, W, Cp);
    }
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x, (float*)y, N, C, H, W, Cp);
  return retr_check_launch("nchw_to_nhwc");
}

int retr_nchw_to_s2d16(const float* x, void* y, int N, int C, int H, int W, void* stream) {
  RETR_REQUIRE(C == 3 && H % 2 == 0 && W % 2 == 0, "nchw_to_s2d16: C=%d H=%d W=%d", C, H, W);
  const long pixels = (long)N * (H / 2) * (W / 2);
  if (pixels == 0) return 0;
  hipLaunchKernelGGL(nchw_to_s2d16_kernel, dim3(grid_for(pixels)), dim3(256), 0,
                     (hipStream_t)stream, x, (bf16*)y, N, H, W);
  return retr_check_launch("nchw_to_s2d16");
}

int retr_stem_s2d_weights(const void* wp, void* w2, int Co, int Cp, void* stream) {
  RETR_REQUIRE(Cp >= 3 && Co > 0, "stem_s2d_weights: Co=%d Cp=%d", Co, Cp);
  const int total = Co * 256;
  hipLaunchKernelGGL(stem_s2d_weights_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)wp, (bf16*)w2, Co, Cp);
  return retr_check_launch("stem_s2d_weights");
}

int retr_maxpool3x3s2(int dtype, const void* x, void* y, int N, int H, int W, int C, int OH,
                      int OW, void* stream) {
  long total = (long)N * OH * OW * C;
  if (total == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    if (C % 8 == 0)
      hipLaunchKernelGGL(maxpool8_kernel, dim3(grid_for(total / 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C, OH, OW);
    else
      hipLaunchKernelGGL(maxpool_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)y, N, H, W, C, OH, OW);
  return retr_check_launch("maxpool3x3s2");
}

int retr_mask_nearest(const unsigned char* m, unsigned char* out, int N, int H, int W, int h,
                      int w, void* stream) {
  long total = (long)N * h * w;
  if (total == 0) return 0;
  hipLaunchKernelGGL(mask_nearest_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, m, out, N, H, W, h, w);
  return retr_check_launch("mask_nearest");
}

int retr_dropout_apply(int dtype_out, const float* x, long ldx, void* y, long ldy, int M, int N,
                       float drop_p, unsigned long long seed, void* stream) {
  if ((long)M * N == 0) return 0;
  const long total = (long)M * ((N + 7) / 8);   // threads: 8 columns each
  hipStream_t st = (hipStream_t)stream;
  DropoutParams dp = make_dp(drop_p, seed);
  if (dtype_out == RETR_BF16)
    hipLaunchKernelGGL(dropout_apply_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, x, ldx, (bf16*)y, ldy, M, N, dp);
  else
    hipLaunchKernelGGL(dropout_apply_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x, ldx, (float*)y, ldy, M, N, dp);
  return retr_check_launch("dropout_apply");
}

int retr_cast(int dtype, const float* x, void* y, long n, void* stream) {
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, x, (bf16*)y, n);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, x, (float*)y, n);
  return retr_check_launch("cast");
}

static int pos_grad(int dtype, const void* d, long ld, int M, int C, int period, float* dpos,
                    int acc, void* stream) {
  long total = (long)period * C;
  if (total == 0 || M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int esz = dtype == RETR_BF16 ? 2 : 4;
  if (C % 8 == 0 && ld % 8 == 0 && ((uintptr_t)d % (8 * esz < 16 ? 8 * esz : 16)) == 0 &&
      ((uintptr_t)dpos & 15) == 0) {
    const unsigned blocks = (unsigned)((total / 8 + 255) / 256);
    if (dtype == RETR_BF16)
      hipLaunchKernelGGL(pos_grad8_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (const bf16*)d, ld, M, C, period, dpos, acc);
    else
      hipLaunchKernelGGL(pos_grad8_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)d, ld, M, C, period, dpos, acc);
    return retr_check_launch("pos_grad8");
  }
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(pos_grad_kernel<bf16>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const bf16*)d, ld, M, C, period, dpos, acc);
  else
    hipLaunchKernelGGL(pos_grad_kernel<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const float*)d, ld, M, C, period, dpos, acc);
  return retr_check_launch("pos_grad");
}

int retr_pos_grad(int dtype, const void* d, long ld, int M, int C, int period, float* dpos,
                  void* stream) {
  return pos_grad(dtype, d, ld, M, C, period, dpos, 1, stream);
}

int retr_pos_grad_set(int dtype, const void* d, long ld, int M, int C, int period, float* dpos,
                      void* stream) {
  return pos_grad(dtype, d, ld, M, C, period, dpos, 0, stream);
}

int retr_pos_grad_multi(int dtype, int n, const retr_pos_item* items, int C, int period,
                        float* dpos, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RETR_REQUIRE(n >= 0 && (n == 0 || items) && period > 0, "pos_grad_multi: n=%d period=%d", n,
               period);
  bool vec = C % 8 == 0 && ((uintptr_t)dpos & 15) == 0;
  for (int i = 0; i < n && vec; ++i)
    vec = items[i].ld % 8 == 0 && ((uintptr_t)items[i].d & 15) == 0;
  if (!vec) {         // the per-item launches (same results)
    for (int i = 0; i < n; ++i)
      if (int e = pos_grad(dtype, items[i].d, items[i].ld, items[i].M, C, period, dpos,
                           (accumulate || i > 0) ? 1 : 0, stream))
        return e;
    return 0;
  }
  for (int i0 = 0; i0 < n; i0 += kPosMulti) {
    PosItems it{};
    it.n = n - i0 < kPosMulti ? n - i0 : kPosMulti;
    for (int k = 0; k < it.n; ++k) {
      it.d[k] = items[i0 + k].d;
      it.ld[k] = items[i0 + k].ld;
      it.M[k] = items[i0 + k].M;
    }
    const long chunks = (long)period * (C / 8);
    const int acc = (accumulate || i0 > 0) ? 1 : 0;
    const dim3 grid((unsigned)((chunks + 15) / 16));
    if (dtype == RETR_BF16)
      hipLaunchKernelGGL(pos_grad_multi_kernel<bf16>, grid, dim3(256), 0, st, it, C, period, dpos, acc);
    else
      hipLaunchKernelGGL(pos_grad_multi_kernel<float>, grid, dim3(256), 0, st, it, C, period, dpos, acc);
    if (int e = retr_check_launch("pos_grad_multi")) return e;
  }
  return 0;
}

}  // extern "C"

// y[c][r] = x[r][c] through a 32x33 LDS tile (coalesced both ways); r in [R, R_pad) -> 0.
template <typename T>
__global__ void transpose_cast_kernel(const float* x, T* y, int R, int C, int R_pad) {
  __shared__ float tile[32][33];
  int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  for (int i = threadIdx.y; i < 32; i += 8) {
    int r = r0 + i, c = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (r < R && c < C) ? x[(long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    int c = c0 + i, r = r0 + threadIdx.x;
    if (c < C && r < R_pad) y[(long)c * R_pad + r] = from_f<T>(tile[threadIdx.x][i]);
  }
}

extern "C" int retr_transpose_cast(int dtype, const float* x, void* y, int R, int C, int R_pad,
                                   void* stream) {
  dim3 grid((C + 31) / 32, (R_pad + 31) / 32), block(32, 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(transpose_cast_kernel<bf16>, grid, block, 0, st, x, (bf16*)y, R, C, R_pad);
  else
    hipLaunchKernelGGL(transpose_cast_kernel<float>, grid, block, 0, st, x, (float*)y, R, C, R_pad);
  return retr_check_launch("transpose_cast");
}
