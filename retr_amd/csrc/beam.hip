// Beam-search decode step kernels (new capability: the reference has only greedy decoding,
// eval_utils/decode.py:53-81).  Semantics (retr_amd/eval_utils/decode.py,
// IncrementalBeam): K beams per image, score = sum of log-softmax(logits) of the chosen tokens;
// a finished beam (EOS emitted) keeps its score and is continued by its argmax token (the
// greedy contract's post-EOS writes), every other beam offers its K best tokens; the K best of
// all candidates (ties: lower parent beam, then better-ranked token) survive.  With K = 1 the
// chosen token is exactly the first-index argmax of the logits, so beam=1 == greedy.
//
// KV caches are never copied when beams are reordered: anc[r][t] names the cache row that holds
// position t of beam row r (the row whose beam computed it at step t), and the decode attention
// kernel reads keys / values through it (retr_attention_decode's `anc`).
#include "common.hpp"
#include "../../include/retr_hip.h"

namespace {

constexpr int kMaxK = 8;
constexpr int kThreads = 256;

// lexicographic "better": larger value, then smaller index (first-index argmax semantics)
RETR_DEVICE bool better(float v, int i, float w, int j) { return v > w || (v == w && i < j); }

template <typename T>
RETR_DEVICE void load8f(const T* p, float (&v)[8]);
template <> RETR_DEVICE void load8f<bf16>(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
}
template <> RETR_DEVICE void load8f<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  v[0] = a[0], v[1] = a[1], v[2] = a[2], v[3] = a[3];
  v[4] = b[0], v[5] = b[1], v[6] = b[2], v[7] = b[3];
}

// One block per logits row: log-sum-exp and the K best (value, index), first index on ties.
// Each thread keeps a sorted private list over its 8-wide chunks, then K rounds of a block-wide
// (value desc, index asc) reduction pop the global best.
template <typename T>
__global__ void __launch_bounds__(kThreads)
topk_kernel(const T* x, long ld, int V, int K, int* idx_out, float* lp_out) {
  __shared__ float rv[kThreads / 64];
  __shared__ int ri[kThreads / 64], rt[kThreads / 64];
  __shared__ float red[2 * kThreads / 64];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* xr = x + (long)row * ld;
  float tv[kMaxK];
  int ti[kMaxK];
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) tv[k] = -INFINITY, ti[k] = 0x7fffffff;
  float mx = -INFINITY, sum = 0.f;   // online log-sum-exp
  auto offer = [&](float v, int i) {
    if (v > mx) {
      sum = sum * __expf(mx - v) + 1.f;
      mx = v;
    } else {
      sum += __expf(v - mx);
    }
    // insertion into the sorted private list (static indices only: registers, no scratch)
    float cv = v;
    int ci = i;
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
      if (k < K && better(cv, ci, tv[k], ti[k])) {
        const float tvk = tv[k];
        const int tik = ti[k];
        tv[k] = cv;
        ti[k] = ci;
        cv = tvk;
        ci = tik;
      }
    }
  };
  const int V8 = V / 8;
  for (int c = tid; c < V8; c += kThreads) {
    float v[8];
    load8f<T>(xr + 8 * c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) offer(v[e], 8 * c + e);
  }
  for (int i = 8 * V8 + tid; i < V; i += kThreads) offer(to_f(xr[i]), i);
  // block log-sum-exp
  float gm = wave_max(mx);
  float s = (mx == -INFINITY) ? 0.f : sum * __expf(mx - gm);
  s = wave_sum(s);
  if (lane == 0) red[wave] = gm, red[4 + wave] = s;
  __syncthreads();
  float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float bs = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) bs += red[4 + w] * __expf(red[w] - bm);
  const float lse = bm + __logf(bs);
  // K rounds of block argmax over the private list heads
  for (int k = 0; k < K; ++k) {
    float v = tv[0];
    int i = ti[0];
    int who = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float v2 = __shfl_xor(v, o, 64);
      int i2 = __shfl_xor(i, o, 64), w2 = __shfl_xor(who, o, 64);
      if (better(v2, i2, v, i)) v = v2, i = i2, who = w2;
    }
    __syncthreads();
    if (lane == 0) rv[wave] = v, ri[wave] = i, rt[wave] = who;
    __syncthreads();
    float bv = rv[0];
    int bi = ri[0], bw = rt[0];
    for (int w = 1; w < kThreads / 64; ++w)
      if (better(rv[w], ri[w], bv, bi)) bv = rv[w], bi = ri[w], bw = rt[w];
    if (tid == bw) {
      // pop: shift the private list (static indexing keeps it in registers)
#pragma unroll
      for (int q = 0; q < kMaxK - 1; ++q) {
        tv[q] = tv[q + 1];
        ti[q] = ti[q + 1];
      }
      tv[kMaxK - 1] = -INFINITY;
      ti[kMaxK - 1] = 0x7fffffff;
    }
    if (tid == 0) {
      idx_out[(long)row * K + k] = bi;
      if (lp_out) lp_out[(long)row * K + k] = bv - lse;
    }
  }
}

// One block per image b: select the K surviving beams from the candidates, then reorder the
// token history and the cache-ancestry rows in LDS and append step i's token.
__global__ void __launch_bounds__(64)
beam_select_kernel(const int* cand_tok, const float* cand_lp, int B, int K, int i, int T,
                   long long eos, float* scores, unsigned char* finished, long long* hist,
                   int* anc, long long* tok, unsigned char* item_done, const int* done) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // all LDS in one region
  int* par = (int*)smem;                            // [kMaxK]
  int* ntok = par + kMaxK;                          // [kMaxK]
  float* nsc = (float*)(ntok + kMaxK);              // [kMaxK]
  int* nfin = (int*)(nsc + kMaxK);                  // [kMaxK]
  long long* h_old = (long long*)(nfin + kMaxK);    // [K][T]  (offset 128 B)
  int* a_old = (int*)(h_old + (long)K * T);         // [K][T]
  const int b = blockIdx.x, tid = threadIdx.x;
  if (*done >= 0) return;      // the decode already ended (reference contract: no more writes)
  const int r0 = b * K;
  if (tid == 0) {
    // candidates in (beam, rank) order; a stable selection of the K best by score
    float cs[kMaxK * kMaxK];
    int cp[kMaxK * kMaxK], ct[kMaxK * kMaxK], n = 0;
    for (int k = 0; k < K; ++k) {
      if (i == 0 && k > 0) break;                 // all beams start identical: expand one
      const bool fin = i > 0 && finished[r0 + k];
      const float base = i > 0 ? scores[r0 + k] : 0.f;
      const int m = fin ? 1 : K;
      for (int j = 0; j < m; ++j) {
        cs[n] = fin ? base : base + cand_lp[(long)(r0 + k) * K + j];
        cp[n] = k;
        ct[n] = cand_tok[(long)(r0 + k) * K + j];
        ++n;
      }
    }
    bool used[kMaxK * kMaxK];
    for (int c = 0; c < n; ++c) used[c] = false;
    for (int s = 0; s < K; ++s) {
      int best = -1;
      for (int c = 0; c < n; ++c)
        if (!used[c] && (best < 0 || cs[c] > cs[best])) best = c;   // first index on ties
      used[best] = true;
      par[s] = cp[best];
      ntok[s] = ct[best];
      nsc[s] = cs[best];
      const bool pf = i > 0 && finished[r0 + cp[best]];
      nfin[s] = (pf || ct[best] == eos) ? 1 : 0;
    }
  }
  // stage old rows
  for (int e = tid; e < K * T; e += blockDim.x) {
    h_old[e] = hist[(long)r0 * T + e];
    a_old[e] = anc[(long)r0 * T + e];
  }
  __syncthreads();
  for (int e = tid; e < K * T; e += blockDim.x) {
    const int s = e / T, t = e % T, p = par[s];
    long long hv = h_old[p * T + t];
    int av = a_old[p * T + t];
    if (t == i + 1) hv = ntok[s];
    if (t == i) av = r0 + p;                       // position i was computed in row r0+p
    if (t > i) av = r0 + s;                        // future positions: written by this row
    hist[(long)r0 * T + e] = hv;
    anc[(long)r0 * T + e] = av;
  }
  if (tid < K) {
    scores[r0 + tid] = nsc[tid];
    finished[r0 + tid] = nfin[tid];
    tok[r0 + tid] = ntok[tid];
  }
  if (tid == 0) {
    unsigned char all = 1;
    for (int s = 0; s < K; ++s) all &= nfin[s];
    item_done[b] = all;
  }
}

// done = i once every image's K beams are finished (column i+1 then does not count).
__global__ void beam_done_kernel(const unsigned char* item_done, int B, int i, int* done) {
  __shared__ int all;
  if (threadIdx.x == 0) all = 1;
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x)
    if (!item_done[b]) atomicAnd(&all, 0);
  __syncthreads();
  if (threadIdx.x == 0 && *done < 0 && all) *done = i;
}

}  // namespace

extern "C" {

int retr_topk_rows(int dtype, const void* x, long ld, int M, int V, int K, int* idx,
                   float* logprob, void* stream) {
  RETR_REQUIRE(K >= 1 && K <= kMaxK, "topk_rows: K=%d must be in [1, %d]", K, kMaxK);
  RETR_REQUIRE(ld % 8 == 0 && V >= K, "topk_rows: row stride %%8 and V >= K");
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RETR_BF16)
    hipLaunchKernelGGL(topk_kernel<bf16>, dim3(M), dim3(kThreads), 0, st, (const bf16*)x, ld, V,
                       K, idx, logprob);
  else
    hipLaunchKernelGGL(topk_kernel<float>, dim3(M), dim3(kThreads), 0, st, (const float*)x, ld,
                       V, K, idx, logprob);
  return retr_check_launch("topk_rows");
}

int retr_beam_select(const int* cand_tok, const float* cand_lp, int B, int K, int i, int T,
                     long long eos, float* scores, unsigned char* finished, long long* hist,
                     int* anc, long long* tok, unsigned char* item_done, int* done,
                     void* stream) {
  RETR_REQUIRE(K >= 1 && K <= kMaxK && i >= 0 && i + 1 < T, "beam_select: bad K/i/T");
  size_t lds = 128 + (size_t)K * T * (sizeof(long long) + sizeof(int));
  RETR_REQUIRE(lds <= 65536, "beam_select: K*T too large");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(beam_select_kernel, dim3(B), dim3(64), lds, st, cand_tok, cand_lp, B, K, i,
                     T, eos, scores, finished, hist, anc, tok, item_done, done);
  if (int e = retr_check_launch("beam_select")) return e;
  hipLaunchKernelGGL(beam_done_kernel, dim3(1), dim3(256), 0, st, item_done, B, i, done);
  return retr_check_launch("beam_done");
}

}  // extern "C"
