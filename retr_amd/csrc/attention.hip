// Multi-head attention core for the pre-norm DETR-style encoder/decoder
// (torch/nn/functional.py:6576-6606 need_weights path, used by
//  models/ConcatTransformer.py:160,204,210 through models/transformer_modules.py:38,66).
//
//   S = (q * hd^-1/2) k^T + mask      mask: key padding (-inf), causal (-inf above diagonal)
//   P = softmax(S);  O = dropout(P) v
//
// Forward: flash-style online softmax.  One block = (b, h, 64 query rows); 4 waves x 16 rows;
// K tiles of 64 keys staged in LDS (row-major for QK^T, V transposed for PV), MFMA 16x16
// (bf16 x32 or exact-f32 x4).  P goes through a per-wave LDS scratch to become the A operand.
// Backward: D = rowsum(dO*O); dQ kernel (per query tile, loop over keys) and dK/dV kernel (per
// key tile, loop over queries) recompute P from the saved log-sum-exp -> no atomics.
// Dropout: counter hash keep(seed, ((b*H+h)*Lq+i)*Lk+j) regenerated in backward.
// Fully masked rows produce NaN like torch's softmax of an all -inf row.
#include "gemm.hpp"
#include "../../include/retr_hip.h"

int retr_attention_fwd2(const void* q, long ldq, const void* k, long ldk, const void* v,
                        long ldv, void* o, long ldo, int B, int H, int Lq, int Lk, int hd,
                        const unsigned char* kpm, int causal, float p, unsigned long long seed,
                        float* lse, uint32_t* dmask, hipStream_t st);
int retr_attention_bwd2(const void* q, long ldq, const void* k, long ldk, const void* v,
                        long ldv, const void* o, long ldo, const void* dout, long lddo,
                        const float* lse, void* dq, long lddq, void* dk, long lddk, void* dv,
                        long lddv, int B, int H, int Lq, int Lk, int hd,
                        const unsigned char* kpm, int causal, float p, unsigned long long seed,
                        float* D, const uint32_t* dmask, hipStream_t st);

using namespace retr;

namespace {

constexpr int BQ = 64, BKV = 64;

template <typename T> struct AT {
  static constexpr int EPC = 16 / sizeof(T);
  static constexpr int PAD = EPC;  // one 16-byte chunk of row padding
};

// acc += A(16 x L) * B(16 x L)^T where lane (l&15) supplies row pointers of A and B; k split
// into chunk groups exactly as in the GEMM core (chunk (lane>>4) + 4*kb).
template <typename T, int L>
RETR_DEVICE void mma_row(f32x4& acc, const T* arow, const T* brow, int lane) {
  constexpr int EPC = AT<T>::EPC;
#pragma unroll
  for (int kb = 0; kb < L / (4 * EPC); ++kb) {
    int c = (lane >> 4) + 4 * kb;
    u32x4 a = *(const u32x4*)(arow + c * EPC);
    u32x4 b = *(const u32x4*)(brow + c * EPC);
    mfma_step<T>(acc, a, b);
  }
}

// reduce over the 16 lanes that share a row group (lane bits 0..3)
RETR_DEVICE float grp_max(float v) {
  v = fmaxf(v, xor_lane(v, 1));
  v = fmaxf(v, xor_lane(v, 2));
  v = fmaxf(v, xor_lane(v, 4));
  v = fmaxf(v, xor_lane(v, 8));
  return v;
}
RETR_DEVICE float grp_sum(float v) {
  v += xor_lane(v, 1);
  v += xor_lane(v, 2);
  v += xor_lane(v, 4);
  v += xor_lane(v, 8);
  return v;
}

// Load a 64-row x hd tile (row r at base + (r0+r)*ld) into LDS row-major [64][HDP+PAD], zero
// padded, optionally scaled; 16-byte global loads (hd and ld are multiples of EPC).
template <typename T, int HDP>
RETR_DEVICE void load_rows(T* dst, const T* base, long ld, int r0, int nrows, int hd,
                           float scale) {
  constexpr int EPC = AT<T>::EPC, S = HDP + AT<T>::PAD, CPR = HDP / EPC;
  for (int i = threadIdx.x; i < 64 * CPR; i += 256) {
    const int r = i / CPR, c = (i % CPR) * EPC;
    u32x4 v = zero16();
    if (r0 + r < nrows && c < hd) {
      v = *(const u32x4*)(base + (long)(r0 + r) * ld + c);
      if (scale != 1.f) {
        T* e = (T*)&v;
#pragma unroll
        for (int j = 0; j < EPC; ++j) e[j] = from_f<T>(to_f(e[j]) * scale);
      }
    }
    *(u32x4*)(dst + r * S + c) = v;
  }
}
// Transposed: dst[d][r] (row stride 64+PAD)
template <typename T, int HDP>
RETR_DEVICE void load_rows_t(T* dst, const T* base, long ld, int r0, int nrows, int hd,
                             float scale) {
  constexpr int EPC = AT<T>::EPC, S = 64 + AT<T>::PAD, CPR = HDP / EPC;
  for (int i = threadIdx.x; i < 64 * CPR; i += 256) {
    const int r = i % 64, c = (i / 64) * EPC;   // consecutive threads -> consecutive rows
    u32x4 v = zero16();
    if (r0 + r < nrows && c < hd) v = *(const u32x4*)(base + (long)(r0 + r) * ld + c);
    const T* e = (const T*)&v;
#pragma unroll
    for (int j = 0; j < EPC; ++j)
      dst[(c + j) * S + r] = scale != 1.f ? from_f<T>(to_f(e[j]) * scale) : e[j];
  }
}

// attention dropout keep decision of (query row, key): the fused kernels' RNG (common.hpp)
RETR_DEVICE bool attn_keep_at(const DropoutParams& dp, uint32_t row, int key) {
  const uint32_t bits = attn_pair_bits(attn_row_key(dp_seed(dp), row), (uint32_t)key);
  return attn_keep(bits, (uint32_t)key, (dp.thresh + 0x8000u) >> 16);
}

RETR_DEVICE bool masked(const unsigned char* kpm, int b, int Lk, int key, int qrow, int causal) {
  if (key >= Lk) return true;
  if (kpm && kpm[(long)b * Lk + key]) return true;
  if (causal && key > qrow) return true;
  return false;
}

template <typename T, int HDP>
__global__ void __launch_bounds__(256)
attn_fwd_kernel(const T* q, long ldq, const T* k, long ldk, const T* v, long ldv, T* o, long ldo,
                int H, int Lq, int Lk, int hd, const unsigned char* kpm, int causal, float scale,
                DropoutParams dp, float* lse, int kbr) {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Qs = (T*)smem;
  T* Ks = Qs + 64 * RS;
  T* Vt = Ks + 64 * RS;
  T* Ps = Vt + HDP * TS;
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * BQ;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const T* qb = q + (long)b * Lq * ldq + h * hd;
  const T* kb = k + (long)b * kbr * ldk + h * hd;  // kbr: key rows per batch in storage
  const T* vb = v + (long)b * kbr * ldv + h * hd;
  T* Pw = Ps + wave * 16 * TS;

  load_rows<T, HDP>(Qs, qb, ldq, q0, Lq, hd, scale);
  float m[4], l[4];
  f32x4 O[HDP / 16];
#pragma unroll
  for (int e = 0; e < 4; ++e) m[e] = -INFINITY, l[e] = 0.f;
#pragma unroll
  for (int j = 0; j < HDP / 16; ++j) O[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int kend = Lk;
  if (causal) kend = min(Lk, q0 + BQ);
  for (int k0 = 0; k0 < kend; k0 += BKV) {
    __syncthreads();
    load_rows<T, HDP>(Ks, kb, ldk, k0, Lk, hd, 1.f);
    load_rows_t<T, HDP>(Vt, vb, ldv, k0, Lk, hd, 1.f);
    __syncthreads();
    f32x4 S[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      S[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma_row<T, HDP>(S[j], Qs + (wave * 16 + c16) * RS, Ks + (16 * j + c16) * RS, lane);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int qrow = q0 + wave * 16 + 4 * g + e;
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int key = k0 + 16 * j + c16;
        if (masked(kpm, b, Lk, key, qrow, causal)) S[j][e] = -INFINITY;
        mx = fmaxf(mx, S[j][e]);
      }
      mx = grp_max(mx);
      const float mn = fmaxf(m[e], mx);
      const float alpha = (mn == -INFINITY) ? 1.f : __expf(m[e] - mn);
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float p = (mn == -INFINITY) ? 0.f : __expf(S[j][e] - mn);
        rs += p;
        if (dp.thresh) {
          const int key = k0 + 16 * j + c16;
          p = attn_keep_at(dp, ((uint32_t)b * H + h) * Lq + qrow, key) ? p * dp.scale : 0.f;
        }
        Pw[(4 * g + e) * TS + 16 * j + c16] = from_f<T>(p);
      }
      rs = grp_sum(rs);
      l[e] = l[e] * alpha + rs;
      m[e] = mn;
#pragma unroll
      for (int jd = 0; jd < HDP / 16; ++jd) O[jd][e] *= alpha;
    }
    __syncthreads();
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd)
      mma_row<T, 64>(O[jd], Pw + c16 * TS, Vt + (16 * jd + c16) * TS, lane);
  }

#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int qrow = q0 + wave * 16 + 4 * g + e;
    if (qrow >= Lq) continue;
    const float inv = 1.f / l[e];
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd) {
      int d = 16 * jd + c16;
      if (d < hd) o[((long)b * Lq + qrow) * ldo + h * hd + d] = from_f<T>(O[jd][e] * inv);
    }
    if (c16 == 0 && lse) lse[((long)b * H + h) * Lq + qrow] = m[e] + __logf(l[e]);
  }
}

// D[b,h,i] = sum_d dO[b,i,h,d] * O[b,i,h,d]
template <typename T>
__global__ void attn_bwd_dot_kernel(const T* o, long ldo, const T* dout, long lddo, int B, int H,
                                    int Lq, int hd, float* D) {
  long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)B * H * Lq) return;
  int i = idx % Lq;
  long bh = idx / Lq;
  int h = bh % H, b = (int)(bh / H);
  const T* orow = o + ((long)b * Lq + i) * ldo + h * hd;
  const T* drow = dout + ((long)b * Lq + i) * lddo + h * hd;
  float s = 0.f;
  for (int d = 0; d < hd; ++d) s += to_f(orow[d]) * to_f(drow[d]);
  D[idx] = s;
}

template <typename T, int HDP>
__global__ void __launch_bounds__(256)
attn_bwd_dq_kernel(const T* q, long ldq, const T* k, long ldk, const T* v, long ldv,
                   const T* dout, long lddo, const float* lse, const float* D, T* dq, long lddq,
                   int H, int Lq, int Lk, int hd, const unsigned char* kpm, int causal,
                   float scale, DropoutParams dp) {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Qs = (T*)smem;
  T* dOs = Qs + 64 * RS;
  T* Ks = dOs + 64 * RS;
  T* Vs = Ks + 64 * RS;
  T* Kt = Vs + 64 * RS;
  T* Ps = Kt + HDP * TS;
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * BQ;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const T* qb = q + (long)b * Lq * ldq + h * hd;
  const T* kb = k + (long)b * Lk * ldk + h * hd;
  const T* vb = v + (long)b * Lk * ldv + h * hd;
  const T* db = dout + (long)b * Lq * lddo + h * hd;
  T* Pw = Ps + wave * 16 * TS;
  load_rows<T, HDP>(Qs, qb, ldq, q0, Lq, hd, scale);
  load_rows<T, HDP>(dOs, db, lddo, q0, Lq, hd, 1.f);
  float L_[4], D_[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int qrow = q0 + wave * 16 + 4 * g + e;
    long ri = ((long)b * H + h) * Lq + min(qrow, Lq - 1);
    L_[e] = lse[ri];
    D_[e] = D[ri];
  }
  f32x4 dQ[HDP / 16];
#pragma unroll
  for (int j = 0; j < HDP / 16; ++j) dQ[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int kend = causal ? min(Lk, q0 + BQ) : Lk;
  for (int k0 = 0; k0 < kend; k0 += BKV) {
    __syncthreads();
    load_rows<T, HDP>(Ks, kb, ldk, k0, Lk, hd, 1.f);
    load_rows<T, HDP>(Vs, vb, ldv, k0, Lk, hd, 1.f);
    load_rows_t<T, HDP>(Kt, kb, ldk, k0, Lk, hd, 1.f);
    __syncthreads();
    f32x4 S[4], dP[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      S[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dP[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma_row<T, HDP>(S[j], Qs + (wave * 16 + c16) * RS, Ks + (16 * j + c16) * RS, lane);
      mma_row<T, HDP>(dP[j], dOs + (wave * 16 + c16) * RS, Vs + (16 * j + c16) * RS, lane);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int qrow = q0 + wave * 16 + 4 * g + e;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int key = k0 + 16 * j + c16;
        float ds = 0.f;
        if (!masked(kpm, b, Lk, key, qrow, causal) && qrow < Lq) {
          float p = __expf(S[j][e] - L_[e]);
          float dpv = dP[j][e];
          if (dp.thresh)
            dpv = attn_keep_at(dp, ((uint32_t)b * H + h) * Lq + qrow, key) ? dpv * dp.scale : 0.f;
          ds = p * (dpv - D_[e]);
        }
        Pw[(4 * g + e) * TS + 16 * j + c16] = from_f<T>(ds);
      }
    }
    __syncthreads();
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd)
      mma_row<T, 64>(dQ[jd], Pw + c16 * TS, Kt + (16 * jd + c16) * TS, lane);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int qrow = q0 + wave * 16 + 4 * g + e;
    if (qrow >= Lq) continue;
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd) {
      int d = 16 * jd + c16;
      if (d < hd) dq[((long)b * Lq + qrow) * lddq + h * hd + d] = from_f<T>(dQ[jd][e] * scale);
    }
  }
}

template <typename T, int HDP>
__global__ void __launch_bounds__(256)
attn_bwd_dkdv_kernel(const T* q, long ldq, const T* k, long ldk, const T* v, long ldv,
                     const T* dout, long lddo, const float* lse, const float* D, T* dk,
                     long lddk, T* dv, long lddv, int H, int Lq, int Lk, int hd,
                     const unsigned char* kpm, int causal, float scale, DropoutParams dp) {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = (T*)smem;
  T* Vs = Ks + 64 * RS;
  T* Qs = Vs + 64 * RS;
  T* dOs = Qs + 64 * RS;
  T* Qt = dOs + 64 * RS;
  T* dOt = Qt + HDP * TS;
  T* Ps = dOt + HDP * TS;
  float* Ls = (float*)(Ps + 4 * 16 * TS);
  float* Ds = Ls + 64;
  const int b = blockIdx.z, h = blockIdx.y, k0 = blockIdx.x * BKV;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const T* qb = q + (long)b * Lq * ldq + h * hd;
  const T* kb = k + (long)b * Lk * ldk + h * hd;
  const T* vb = v + (long)b * Lk * ldv + h * hd;
  const T* db = dout + (long)b * Lq * lddo + h * hd;
  T* Pw = Ps + wave * 16 * TS;
  load_rows<T, HDP>(Ks, kb, ldk, k0, Lk, hd, 1.f);
  load_rows<T, HDP>(Vs, vb, ldv, k0, Lk, hd, 1.f);
  f32x4 dK[HDP / 16], dV[HDP / 16];
#pragma unroll
  for (int j = 0; j < HDP / 16; ++j) dK[j] = dV[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qstart = causal ? (k0 / BQ) * BQ : 0;
  for (int q0 = qstart; q0 < Lq; q0 += BQ) {
    __syncthreads();
    load_rows<T, HDP>(Qs, qb, ldq, q0, Lq, hd, scale);
    load_rows_t<T, HDP>(Qt, qb, ldq, q0, Lq, hd, scale);
    load_rows<T, HDP>(dOs, db, lddo, q0, Lq, hd, 1.f);
    load_rows_t<T, HDP>(dOt, db, lddo, q0, Lq, hd, 1.f);
    if (threadIdx.x < 64) {
      int qr = q0 + threadIdx.x;
      long ri = ((long)b * H + h) * Lq + min(qr, Lq - 1);
      Ls[threadIdx.x] = lse[ri];
      Ds[threadIdx.x] = D[ri];
    }
    __syncthreads();
    // S^T[key][q] = K Q^T ; dP^T = V dO^T
    f32x4 S[4], dP[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      S[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dP[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma_row<T, HDP>(S[j], Ks + (wave * 16 + c16) * RS, Qs + (16 * j + c16) * RS, lane);
      mma_row<T, HDP>(dP[j], Vs + (wave * 16 + c16) * RS, dOs + (16 * j + c16) * RS, lane);
    }
    float P[4][4];
    bool keep[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int key = k0 + wave * 16 + 4 * g + e;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qi = 16 * j + c16, qrow = q0 + qi;
        bool valid = qrow < Lq && !masked(kpm, b, Lk, key, qrow, causal);
        float p = valid ? __expf(S[j][e] - Ls[qi]) : 0.f;
        bool kp = true;
        if (dp.thresh && valid) kp = attn_keep_at(dp, ((uint32_t)b * H + h) * Lq + qrow, key);
        P[e][j] = p;
        keep[e][j] = kp;
        float pd = dp.thresh ? (kp ? p * dp.scale : 0.f) : p;
        Pw[(4 * g + e) * TS + qi] = from_f<T>(pd);
      }
    }
    __syncthreads();
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd)
      mma_row<T, 64>(dV[jd], Pw + c16 * TS, dOt + (16 * jd + c16) * TS, lane);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qi = 16 * j + c16;
        float dpv = dP[j][e];
        if (dp.thresh) dpv = keep[e][j] ? dpv * dp.scale : 0.f;
        float ds = P[e][j] * (dpv - Ds[qi]);
        Pw[(4 * g + e) * TS + qi] = from_f<T>(ds);
      }
    }
    __syncthreads();
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd)
      mma_row<T, 64>(dK[jd], Pw + c16 * TS, Qt + (16 * jd + c16) * TS, lane);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int key = k0 + wave * 16 + 4 * g + e;
    if (key >= Lk) continue;
#pragma unroll
    for (int jd = 0; jd < HDP / 16; ++jd) {
      int d = 16 * jd + c16;
      if (d < hd) {
        dk[((long)b * Lk + key) * lddk + h * hd + d] = from_f<T>(dK[jd][e]);
        dv[((long)b * Lk + key) * lddv + h * hd + d] = from_f<T>(dV[jd][e]);
      }
    }
  }
}

// Head-averaged probabilities (return_attention path only; eval, no dropout).
template <typename T>
__global__ void attn_probs_kernel(const T* q, long ldq, const T* k, long ldk, int H, int Lq,
                                  int Lk, int hd, const unsigned char* kpm, int causal,
                                  float scale, const float* lse, float* probs) {
  long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  int b = blockIdx.y;
  if (idx >= (long)Lq * Lk) return;
  int i = idx / Lk, j = idx % Lk;
  float acc = 0.f;
  for (int h = 0; h < H; ++h) {
    float p = 0.f;
    if (!masked(kpm, b, Lk, j, i, causal)) {
      const T* qr = q + ((long)b * Lq + i) * ldq + h * hd;
      const T* kr = k + ((long)b * Lk + j) * ldk + h * hd;
      float s = 0.f;
      for (int d = 0; d < hd; ++d) s += from_f<T>(to_f(qr[d]) * scale) * to_f(kr[d]);
      p = __expf(s - lse[((long)b * H + h) * Lq + i]);
    } else if (lse[((long)b * H + h) * Lq + i] == -INFINITY) {
      p = NAN;
    }
    acc += p;
  }
  probs[((long)b * Lq + i) * Lk + j] = acc / H;
}


template <typename T>
__global__ void __launch_bounds__(256)
attn_decode_kernel(const T* q, long ldq, const T* k, long ldk, const T* v, long ldv, T* o, long ldo,
                   int H, int Lk, int Lmax, int hd, const unsigned char* kpm, float scale,
                   int kv_group, const int* anc) {
  extern __shared__ float sm[];
  float* sc = sm;            // [Lk] scores -> probabilities
  float* qs = sc + Lk;       // [64] scaled query (rounded to T like the tiled kernel)
  float* red = qs + 64;      // [256] reduction scratch
  const int tid = threadIdx.x, b = blockIdx.x / H, h = blockIdx.x % H;
  constexpr int EPC = 16 / sizeof(T);
  for (int d = tid; d < hd; d += 256) qs[d] = to_f(from_f<T>(to_f(q[(long)b * ldq + h * hd + d]) * scale));
  __syncthreads();
  // key/value row of key j: the query's kv batch (b / kv_group) or, for beam search, the cache
  // row named by the ancestry table (beam rows are reordered without moving the cache)
  const int kvb = b / kv_group;
  const int* ar = anc ? anc + (long)b * Lmax : nullptr;
  auto kvrow = [&](int j) -> long { return (ar ? (long)ar[j] : (long)kvb) * Lmax + j; };
  const T* kb = k + h * hd;
  const T* vb = v + h * hd;
  float mx = -INFINITY;
  for (int j = tid; j < Lk; j += 256) {
    float s = -INFINITY;
    if (!(kpm && kpm[(long)kvb * Lk + j])) {
      s = 0.f;
      const T* kr = kb + kvrow(j) * ldk;
      for (int d0 = 0; d0 < hd; d0 += EPC) {
        u32x4 raw = *(const u32x4*)(kr + d0);
        const T* e = (const T*)&raw;
#pragma unroll
        for (int t = 0; t < EPC; ++t) s += qs[d0 + t] * to_f(e[t]);
      }
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j < Lk; j += 256) {
    float p = mx == -INFINITY ? 0.f : __expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  __syncthreads();
  const int nc = 256 / hd, d = tid % hd, c = tid / hd;
  float acc = 0.f;
  if (c < nc) {
    // (unrolled: the value loads of a stripe are independent, the sum stays in key order)
#pragma unroll 8
    for (int j = c; j < Lk; j += nc) acc += sc[j] * to_f(vb[kvrow(j) * ldv + d]);
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < hd) {
    float s = 0.f;
    for (int cc = 0; cc < nc; ++cc) s += red[cc * hd + tid];
    o[(long)b * ldo + h * hd + tid] = from_f<T>(s * inv);
  }
}

template <typename T, int HDP> size_t fwd_lds() {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  return sizeof(T) * (2 * 64 * RS + HDP * TS + 4 * 16 * TS);
}
template <typename T, int HDP> size_t dq_lds() {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  return sizeof(T) * (4 * 64 * RS + HDP * TS + 4 * 16 * TS);
}
template <typename T, int HDP> size_t dkdv_lds() {
  constexpr int RS = HDP + AT<T>::PAD, TS = 64 + AT<T>::PAD;
  return sizeof(T) * (4 * 64 * RS + 2 * HDP * TS + 4 * 16 * TS) + 2 * 64 * sizeof(float);
}

template <typename K>
void allow_lds(K kern, size_t bytes) {
  // once per kernel instantiation (host-side attribute, not a stream operation)
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    done = true;
  }
}

template <typename T>
int launch_probs(const void* q, long ldq, const void* k, long ldk, int B, int H, int Lq, int Lk,
                 int hd, const unsigned char* kpm, int causal, const float* lse, float* probs,
                 hipStream_t st) {
  const float scale = 1.0f / sqrtf((float)hd);
  dim3 g2(cdiv((long)Lq * Lk, 256), B);
  hipLaunchKernelGGL((attn_probs_kernel<T>), g2, dim3(256), 0, st, (const T*)q, ldq,
                     (const T*)k, ldk, H, Lq, Lk, hd, kpm, causal, scale, lse, probs);
  return retr_check_launch("attention_probs");
}

template <typename T, int HDP>
int fwd_t(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, void* o,
          long ldo, int B, int H, int Lq, int Lk, int hd, const unsigned char* kpm, int causal,
          float p, unsigned long long seed, float* lse, float* probs, hipStream_t st,
          int kbr = 0) {
  float scale = 1.0f / sqrtf((float)hd);
  size_t lds = fwd_lds<T, HDP>();
  allow_lds(attn_fwd_kernel<T, HDP>, lds);
  dim3 grid(cdiv(Lq, BQ), H, B);
  hipLaunchKernelGGL((attn_fwd_kernel<T, HDP>), grid, dim3(256), lds, st, (const T*)q, ldq,
                     (const T*)k, ldk, (const T*)v, ldv, (T*)o, ldo, H, Lq, Lk, hd, kpm, causal,
                     scale, make_dp(p, seed), lse, kbr > 0 ? kbr : Lk);
  if (retr_check_launch("attention_fwd")) return 1;
  if (probs) return launch_probs<T>(q, ldq, k, ldk, B, H, Lq, Lk, hd, kpm, causal, lse, probs, st);
  return 0;
}

template <typename T, int HDP>
int bwd_t(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, const void* o,
          long ldo, const void* dout, long lddo, const float* lse, void* dq, long lddq, void* dk,
          long lddk, void* dv, long lddv, int B, int H, int Lq, int Lk, int hd,
          const unsigned char* kpm, int causal, float p, unsigned long long seed, float* D,
          hipStream_t st) {
  float scale = 1.0f / sqrtf((float)hd);
  DropoutParams dp = make_dp(p, seed);
  long rows = (long)B * H * Lq;
  hipLaunchKernelGGL((attn_bwd_dot_kernel<T>), dim3(cdiv(rows, 256)), dim3(256), 0, st,
                     (const T*)o, ldo, (const T*)dout, lddo, B, H, Lq, hd, D);
  if (retr_check_launch("attention_bwd_dot")) return 1;
  size_t l1 = dq_lds<T, HDP>();
  allow_lds(attn_bwd_dq_kernel<T, HDP>, l1);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, HDP>), dim3(cdiv(Lq, BQ), H, B), dim3(256), l1, st,
                     (const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, (const T*)dout, lddo,
                     lse, D, (T*)dq, lddq, H, Lq, Lk, hd, kpm, causal, scale, dp);
  if (retr_check_launch("attention_bwd_dq")) return 1;
  size_t l2 = dkdv_lds<T, HDP>();
  allow_lds(attn_bwd_dkdv_kernel<T, HDP>, l2);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, HDP>), dim3(cdiv(Lk, BKV), H, B), dim3(256), l2,
                     st, (const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, (const T*)dout,
                     lddo, lse, D, (T*)dk, lddk, (T*)dv, lddv, H, Lq, Lk, hd, kpm, causal, scale,
                     dp);
  return retr_check_launch("attention_bwd_dkdv");
}

}  // namespace

extern "C" {

int retr_attention_fwd(int dtype, const void* q, long ldq, const void* k, long ldk,
                       const void* v, long ldv, void* o, long ldo, int B, int H, int Lq, int Lk,
                       int hd, const unsigned char* kpm, int causal, float drop_p,
                       unsigned long long seed, float* lse, float* probs, void* stream) {
  return retr_attention_fwd_dm(dtype, q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm,
                               causal, drop_p, seed, lse, probs, nullptr, stream);
}

size_t retr_attention_dropout_mask_bytes(int B, int H, int Lq, int Lk) {
  return sizeof(uint32_t) * (size_t)B * H * (size_t)((Lk + 31) / 32) * (size_t)Lq;
}

int retr_attention_fwd_dm(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, void* o, long ldo, int B, int H, int Lq,
                          int Lk, int hd, const unsigned char* kpm, int causal, float drop_p,
                          unsigned long long seed, float* lse, float* probs, void* dmask,
                          void* stream) {
  RETR_REQUIRE(hd >= 8 && hd <= 64 && hd % 8 == 0, "attention: head dim %d unsupported", hd);
  RETR_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0, "attention: row strides %%8");
  if (B == 0 || Lq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16 && (hd == 32 || hd == 64) && ldo % 4 == 0) {
    if (int e = retr_attention_fwd2(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm,
                                    causal, drop_p, seed, lse, (uint32_t*)dmask, st))
      return e;
    return probs ? launch_probs<bf16>(q, ldq, k, ldk, B, H, Lq, Lk, hd, kpm, causal, lse, probs, st)
                 : 0;
  }
  if (dtype == RETR_BF16) {
    if (hd <= 32) return fwd_t<bf16, 32>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, lse, probs, st);
    return fwd_t<bf16, 64>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, lse, probs, st);
  }
  if (hd <= 32) return fwd_t<float, 32>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, lse, probs, st);
  return fwd_t<float, 64>(q, ldq, k, ldk, v, ldv, o, ldo, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, lse, probs, st);
}

// Decode step: one query row per (batch, head) against the first Lk rows of a key/value cache
// whose batch stride is Lmax rows (KV-cache incremental greedy decode, decode.py:68-79).
// One 256-thread block per (b, h): scores in LDS (16-byte K loads), block max/sum, then
// P.V with threads split over (head dim, key stripe) and an LDS reduction.
int retr_attention_decode(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, void* o, long ldo, int B, int H, int Lk,
                          int Lmax, int hd, const unsigned char* kpm, int kv_group,
                          const int* anc, void* stream) {
  RETR_REQUIRE(hd >= 8 && hd <= 64 && hd % 8 == 0, "attention: head dim %d unsupported", hd);
  RETR_REQUIRE(kpm == nullptr || Lmax == Lk, "attention_decode: kpm needs Lmax == Lk");
  RETR_REQUIRE(kv_group >= 1, "attention_decode: kv_group must be >= 1");
  RETR_REQUIRE(Lk >= 1 && Lk <= 4096, "attention_decode: Lk=%d out of range", Lk);
  RETR_REQUIRE(ldk % 8 == 0 && ldv % 8 == 0, "attention_decode: row strides %%8");
  hipStream_t st = (hipStream_t)stream;
  const float scale = 1.0f / sqrtf((float)hd);
  const size_t lds = sizeof(float) * (Lk + 64 + 256 + 8);
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(attn_decode_kernel<bf16>, dim3(B * H), dim3(256), lds, st, (const bf16*)q, ldq,
                       (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, H, Lk, Lmax, hd, kpm,
                       scale, kv_group, anc);
  else
    hipLaunchKernelGGL(attn_decode_kernel<float>, dim3(B * H), dim3(256), lds, st, (const float*)q,
                       ldq, (const float*)k, ldk, (const float*)v, ldv, (float*)o, ldo, H, Lk, Lmax,
                       hd, kpm, scale, kv_group, anc);
  return retr_check_launch("attention_decode");
}

size_t retr_attention_bwd_workspace(int B, int H, int Lq) { return sizeof(float) * (size_t)B * H * Lq; }

int retr_attention_bwd(int dtype, const void* q, long ldq, const void* k, long ldk,
                       const void* v, long ldv, const void* o, long ldo, const void* dout,
                       long lddo, const float* lse, void* dq, long lddq, void* dk, long lddk,
                       void* dv, long lddv, int B, int H, int Lq, int Lk, int hd,
                       const unsigned char* kpm, int causal, float drop_p,
                       unsigned long long seed, float* workspace, void* stream) {
  return retr_attention_bwd_dm(dtype, q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq,
                               dk, lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed,
                               workspace, nullptr, stream);
}

int retr_attention_bwd_dm(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, const void* o, long ldo, const void* dout,
                          long lddo, const float* lse, void* dq, long lddq, void* dk, long lddk,
                          void* dv, long lddv, int B, int H, int Lq, int Lk, int hd,
                          const unsigned char* kpm, int causal, float drop_p,
                          unsigned long long seed, float* workspace, const void* dmask,
                          void* stream) {
  RETR_REQUIRE(hd >= 8 && hd <= 64 && hd % 8 == 0, "attention: head dim %d unsupported", hd);
  RETR_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && lddo % 8 == 0,
               "attention: row strides %%8");
  if (B == 0 || Lq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16 && (hd == 32 || hd == 64) && lddq % 4 == 0 && lddk % 4 == 0 &&
      lddv % 4 == 0)
    return retr_attention_bwd2(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk,
                               lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed,
                               workspace, (const uint32_t*)dmask, st);
  if (dtype == RETR_BF16) {
    if (hd <= 32) return bwd_t<bf16, 32>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, workspace, st);
    return bwd_t<bf16, 64>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, workspace, st);
  }
  if (hd <= 32) return bwd_t<float, 32>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, workspace, st);
  return bwd_t<float, 64>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, workspace, st);
}

}  // extern "C"
