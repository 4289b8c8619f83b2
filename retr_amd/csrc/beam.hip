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
template <typename T, int K>
__global__ void __launch_bounds__(kThreads)
topk_kernel(const T* x, long ld, int V, int* idx_out, float* lp_out) {
  __shared__ float rv[kThreads / 64];
  __shared__ int ri[kThreads / 64], rt[kThreads / 64];
  __shared__ float red[2 * kThreads / 64];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* xr = x + (long)row * ld;
  float tv[K];
  int ti[K];
#pragma unroll
  for (int k = 0; k < K; ++k) tv[k] = -INFINITY, ti[k] = 0x7fffffff;
  float mx = -INFINITY, sum = 0.f;   // online log-sum-exp
  // sorted private list insertion (K is a compile-time constant: static indices, registers)
  auto insert = [&](float v, int i) {
    if (!better(v, i, tv[K - 1], ti[K - 1])) return;
    float cv = v;
    int ci = i;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (better(cv, ci, tv[k], ti[k])) {
        const float tvk = tv[k];
        const int tik = ti[k];
        tv[k] = cv;
        ti[k] = ci;
        cv = tvk;
        ci = tik;
      }
    }
  };
  auto offer = [&](float v, int i) {
    if (v > mx) {
      sum = sum * __expf(mx - v) + 1.f;
      mx = v;
    } else {
      sum += __expf(v - mx);
    }
    insert(v, i);
  };
  // 8-element chunks: one running-max rescale per chunk (no per-element divergent branch), and
  // the insertion only for chunks whose max reaches the current K-th best (after the first few
  // chunks almost none do) -- the per-element compare-and-shift chain made this kernel
  // VALU-bound at ~40 us for 320 rows of 30522 words
  auto offer8 = [&](const float (&v)[8], int base) {
    float cm = v[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) cm = fmaxf(cm, v[e]);
    if (cm > mx) {
      sum = mx == -INFINITY ? 0.f : sum * __expf(mx - cm);
      mx = cm;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += __expf(v[e] - mx);
    if (cm >= tv[K - 1]) {
#pragma unroll
      for (int e = 0; e < 8; ++e) insert(v[e], base + e);
    }
  };
  // 8 chunks per thread in flight before any is offered
  const int V8 = V / 8;
  constexpr int U = 8;
  for (int c0 = tid; c0 < V8; c0 += U * kThreads) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * kThreads;
      if (c < V8) load8f<T>(xr + 8 * c, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * kThreads;
      if (c < V8) offer8(v[u], 8 * c);
    }
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
      float v2 = xor_lane(v, o);
      int i2 = xor_lane(i, o), w2 = xor_lane(who, o);
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
      for (int q = 0; q < K - 1; ++q) {
        tv[q] = tv[q + 1];
        ti[q] = ti[q + 1];
      }
      tv[K - 1] = -INFINITY;
      ti[K - 1] = 0x7fffffff;
    }
    if (tid == 0) {
      idx_out[(long)row * K + k] = bi;
      if (lp_out) lp_out[(long)row * K + k] = bv - lse;
    }
  }
}

// Register-resident variant for rows of up to 512 x 8 x 8 = 32768 words (the 30522-word
// vocabulary): 512 threads, each holds its 8 chunks of 8 in registers.  Pass 1 gives the row's
// log-sum-exp and every wave's maximum; the K-th largest wave maximum tau is a lower bound of the
// K-th best word (K distinct waves each hold a word >= tau), so pass 2 offers only words >= tau to
// the private lists -- a handful per row instead of a compare-and-shift chain per chunk, which
// left topk_kernel VALU-bound at ~37 us for 320 rows.  Same (value desc, index asc) result.
constexpr int kT2 = 512, kT2W = kT2 / 64, kT2C = 8;
template <typename T, int K>
__global__ void __launch_bounds__(kT2)
topk_reg_kernel(const T* x, long ld, int V, int* idx_out, float* lp_out) {
  static_assert(K <= kT2W, "tau needs K distinct waves");
  __shared__ float wmax[kT2W], wsum[kT2W];
  __shared__ float rv[kT2W];
  __shared__ int ri[kT2W], rt[kT2W];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* xr = x + (long)row * ld;
  const int V8 = V / 8;
  float v[kT2C][8];
#pragma unroll
  for (int u = 0; u < kT2C; ++u) {
    const int c = tid + u * kT2;
    if (c < V8) {
      load8f<T>(xr + 8 * c, v[u]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = 8 * c + e;
        v[u][e] = (c == V8 && i < V) ? to_f(xr[i]) : -INFINITY;
      }
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < kT2C; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) mx = fmaxf(mx, v[u][e]);
  float sum = 0.f;
  if (mx != -INFINITY) {
#pragma unroll
    for (int u = 0; u < kT2C; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += __expf(v[u][e] - mx);
  }
  const float gm = wave_max(mx);
  float s = (mx == -INFINITY) ? 0.f : sum * __expf(mx - gm);
  s = wave_sum(s);
  if (lane == 0) wmax[wave] = gm, wsum[wave] = s;
  __syncthreads();
  float bm = wmax[0];
#pragma unroll
  for (int w = 1; w < kT2W; ++w) bm = fmaxf(bm, wmax[w]);
  float bs = 0.f;
#pragma unroll
  for (int w = 0; w < kT2W; ++w) bs += wmax[w] == -INFINITY ? 0.f : wsum[w] * __expf(wmax[w] - bm);
  const float lse = bm + __logf(bs);
  // tau = K-th largest wave maximum (counting equal maxima of distinct waves)
  float tau = -INFINITY;
#pragma unroll
  for (int w = 0; w < kT2W; ++w) {
    int above = 0;
#pragma unroll
    for (int q = 0; q < kT2W; ++q) above += (wmax[q] > wmax[w] || (wmax[q] == wmax[w] && q < w));
    if (above == K - 1) tau = wmax[w];
  }
  float tv[K];
  int ti[K];
#pragma unroll
  for (int k = 0; k < K; ++k) tv[k] = -INFINITY, ti[k] = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < kT2C; ++u) {
    float cm = v[u][0];
#pragma unroll
    for (int e = 1; e < 8; ++e) cm = fmaxf(cm, v[u][e]);
    if (cm >= tau) {
      const int base = 8 * (tid + u * kT2);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float cv0 = v[u][e];
        if (base + e >= V || cv0 < tau || !better(cv0, base + e, tv[K - 1], ti[K - 1])) continue;
        float cv = cv0;
        int ci = base + e;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (better(cv, ci, tv[k], ti[k])) {
            const float tvk = tv[k];
            const int tik = ti[k];
            tv[k] = cv;
            ti[k] = ci;
            cv = tvk;
            ci = tik;
          }
        }
      }
    }
  }
  // the candidates (at least K, usually few): gathered into LDS and ranked by one wave --
  // instead of K rounds of a block-wide argmax (two barriers each); more than 64 (ties at the
  // threshold) take the rounds below
  __shared__ float cvs[64];
  __shared__ int cis[64];
  __shared__ int ncand;
  if (tid == 0) ncand = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (ti[k] != 0x7fffffff) {
      const int slot = atomicAdd(&ncand, 1);
      if (slot < 64) cvs[slot] = tv[k], cis[slot] = ti[k];
    }
  __syncthreads();
  const int nc = ncand;
  if (nc <= 64) {
    if (wave == 0 && lane < nc) {
      const float mv = cvs[lane];
      const int mi = cis[lane];
      int rank = 0;
      for (int q = 0; q < nc; ++q) rank += better(cvs[q], cis[q], mv, mi) ? 1 : 0;
      if (rank < K) {
        idx_out[(long)row * K + rank] = mi;
        if (lp_out) lp_out[(long)row * K + rank] = mv - lse;
      }
    }
    return;
  }
  for (int k = 0; k < K; ++k) {
    float bv = tv[0];
    int bi = ti[0];
    int who = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float v2 = xor_lane(bv, o);
      const int i2 = xor_lane(bi, o), w2 = xor_lane(who, o);
      if (better(v2, i2, bv, bi)) bv = v2, bi = i2, who = w2;
    }
    __syncthreads();
    if (lane == 0) rv[wave] = bv, ri[wave] = bi, rt[wave] = who;
    __syncthreads();
    float cv = rv[0];
    int ci = ri[0], cw = rt[0];
#pragma unroll
    for (int w = 1; w < kT2W; ++w)
      if (better(rv[w], ri[w], cv, ci)) cv = rv[w], ci = ri[w], cw = rt[w];
    if (tid == cw) {
#pragma unroll
      for (int q = 0; q < K - 1; ++q) {
        tv[q] = tv[q + 1];
        ti[q] = ti[q + 1];
      }
      tv[K - 1] = -INFINITY;
      ti[K - 1] = 0x7fffffff;
    }
    if (tid == 0) {
      idx_out[(long)row * K + k] = ci;
      if (lp_out) lp_out[(long)row * K + k] = cv - lse;
    }
  }
}

// One block per image b: select the K surviving beams from the candidates (the first wave),
// then reorder the token history and the cache-ancestry rows in LDS and append step i's token
// (all four waves: the K x T row copies in a quarter of the dependent passes of one wave).
__global__ void __launch_bounds__(256)
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
  // candidate c = (beam k, rank j) on thread c = k K + j (K <= 8: <= 64 candidates, one wave);
  // its place in the stable order (score desc, then (k, j)) is the number of candidates ahead
  // of it, so the K survivors are the candidates of rank < K -- the serial "pick the first best
  // unused candidate K times" selection, without a single-thread loop over scratch arrays
  {
    __shared__ float cs_s[kMaxK * kMaxK];
    __shared__ int ok_s[kMaxK * kMaxK];
    const int k = tid / K, j = tid - k * K;
    bool ok = tid < K * K && !(i == 0 && k > 0);
    const bool fin = ok && i > 0 && finished[r0 + k];
    if (fin && j > 0) ok = false;                  // a finished beam offers one continuation
    float sc = -INFINITY;
    int tk = 0;
    if (ok) {
      const float base = i > 0 ? scores[r0 + k] : 0.f;
      sc = fin ? base : base + cand_lp[(long)(r0 + k) * K + j];
      tk = cand_tok[(long)(r0 + k) * K + j];
    }
    if (tid < kMaxK * kMaxK) {
      cs_s[tid] = sc;
      ok_s[tid] = ok;
    }
    __syncthreads();
    if (ok) {
      int rank = 0;
      for (int c = 0; c < K * K; ++c)
        if (ok_s[c] && (cs_s[c] > sc || (cs_s[c] == sc && c < tid))) ++rank;
      if (rank < K) {
        par[rank] = k;
        ntok[rank] = tk;
        nsc[rank] = sc;
        nfin[rank] = (fin || (long long)tk == eos) ? 1 : 0;
      }
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
  const bool reg = V <= kT2 * kT2C * 8;
#define TOPK(KK)                                                                                 \
  if (reg && dtype == RETR_BF16)                                                                 \
    hipLaunchKernelGGL((topk_reg_kernel<bf16, KK>), dim3(M), dim3(kT2), 0, st, (const bf16*)x,   \
                       ld, V, idx, logprob);                                                     \
  else if (reg)                                                                                  \
    hipLaunchKernelGGL((topk_reg_kernel<float, KK>), dim3(M), dim3(kT2), 0, st, (const float*)x, \
                       ld, V, idx, logprob);                                                     \
  else if (dtype == RETR_BF16)                                                                   \
    hipLaunchKernelGGL((topk_kernel<bf16, KK>), dim3(M), dim3(kThreads), 0, st, (const bf16*)x,  \
                       ld, V, idx, logprob);                                                     \
  else                                                                                           \
    hipLaunchKernelGGL((topk_kernel<float, KK>), dim3(M), dim3(kThreads), 0, st,                 \
                       (const float*)x, ld, V, idx, logprob);
  switch (K) {
    case 1: TOPK(1) break;
    case 2: TOPK(2) break;
    case 3: TOPK(3) break;
    case 4: TOPK(4) break;
    case 5: TOPK(5) break;
    case 6: TOPK(6) break;
    case 7: TOPK(7) break;
    default: TOPK(8) break;
  }
#undef TOPK
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
  hipLaunchKernelGGL(beam_select_kernel, dim3(B), dim3(256), lds, st, cand_tok, cand_lp, B, K, i,
                     T, eos, scores, finished, hist, anc, tok, item_done, done);
  if (int e = retr_check_launch("beam_select")) return e;
  hipLaunchKernelGGL(beam_done_kernel, dim3(1), dim3(256), 0, st, item_done, B, i, done);
  return retr_check_launch("beam_done");
}

}  // extern "C"
