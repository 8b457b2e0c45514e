// Token sampling for gfx950, reproducing transformers' sampling order
// (temperature -> top-k -> top-p -> softmax -> multinomial; reference call
// model.generate(max_new_tokens=150, temperature=0.7, top_p=0.9) at
// /root/reference/llm/rag.py:172 with the GenerationConfig default top_k=50).
//
// Two stages so tensor-parallel vocab shards compose exactly (top-k precedes top-p):
//   1. topk_candidates: per row, radix-select the K largest logits of a (possibly
//      vocab-sharded) row -> K (value, global index) pairs sorted descending.
//   2. sample_candidates: merge R candidate lists (R = TP ranks, all-gathered),
//      keep the global top-K, apply temperature, top-p, and draw with a
//      counter-based RNG (seed, step) -- deterministic across TP ranks.
#include "common.h"
using namespace ragk;

namespace {

constexpr int TK_THREADS = 1024;
constexpr int MAXK = 256;

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(unsigned k) {
  const unsigned u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// ascending-by-"rank" bitonic sort in LDS: sorts (key desc, idx asc). n power of two.
__device__ void bitonic_desc(float* v, int* ix, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;  // "up" segments end up descending
          const float a = v[i], b = v[p];
          const int ia = ix[i], ib = ix[p];
          // a should precede b if a > b (or equal and ia < ib)
          const bool a_first = (a > b) || (a == b && (unsigned)ia < (unsigned)ib);
          if (a_first != up) {
            v[i] = b; v[p] = a; ix[i] = ib; ix[p] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Block (row b, vocab chunk c): top-K of logits[b, c*Vc : min((c+1)*Vc, V)] -> candidates
// [b][c*K + i]; chunking spreads one row over `chunks` workgroups (128k vocab: 16 x 8k).
__global__ __launch_bounds__(TK_THREADS) void topk_candidates_kernel(const float* __restrict__ logits, int ld, int Vtot,
                                                                     int K, int vocab_offset, int chunks,
                                                                     float* cand_v, int* cand_i) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_krem, s_cnt_gt, s_cnt_eq;
  __shared__ float sv[MAXK];
  __shared__ int si[MAXK];
  const int b = blockIdx.x / chunks, chunk = blockIdx.x % chunks;
  const int Vc = ((Vtot + chunks - 1) / chunks + 7) & ~7;
  const int c0 = min(chunk * Vc, Vtot);
  const int V = min(Vtot - c0, Vc);
  const float* row = logits + (size_t)b * ld + c0;
  vocab_offset += c0;
  unsigned prefix = 0, mask = 0, krem = (unsigned)min(K, max(V, 1));
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += TK_THREADS) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += TK_THREADS) {
      const unsigned k = fkey(row[i]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned above = 0;
      int d = 255;
      for (; d >= 0; --d) {
        if (above + hist[d] >= krem) break;
        above += hist[d];
      }
      if (d < 0) d = 0;
      s_prefix = prefix | ((unsigned)d << shift);
      s_krem = krem - above;
    }
    __syncthreads();
    prefix = s_prefix;
    krem = s_krem;
    mask |= 255u << shift;
  }
  // prefix = key of the K-th largest; take all keys > prefix plus `krem` of those == prefix
  if (threadIdx.x == 0) { s_cnt_gt = 0; s_cnt_eq = 0; }
  for (int i = threadIdx.x; i < MAXK; i += TK_THREADS) { sv[i] = -INFINITY; si[i] = 0x7fffffff; }
  __syncthreads();
  const int kk = max(0, min(K, V));
  const unsigned n_gt = (unsigned)kk - min(krem, (unsigned)kk);
  for (int i = threadIdx.x; i < V; i += TK_THREADS) {
    const float x = row[i];
    const unsigned k = fkey(x);
    if (k > prefix) {
      const unsigned slot = atomicAdd(&s_cnt_gt, 1u);
      if (slot < (unsigned)MAXK) { sv[slot] = x; si[slot] = i + vocab_offset; }
    } else if (k == prefix) {
      const unsigned e = atomicAdd(&s_cnt_eq, 1u);
      if (e < krem) {
        const unsigned slot = n_gt + e;
        if (slot < (unsigned)MAXK) { sv[slot] = x; si[slot] = i + vocab_offset; }
      }
    }
  }
  __syncthreads();
  int n = 1;
  while (n < kk) n <<= 1;
  bitonic_desc(sv, si, n);
  const size_t obase = ((size_t)b * chunks + chunk) * K;  // row b, slots [chunk*K, chunk*K + K)
  for (int i = threadIdx.x; i < K; i += TK_THREADS) {
    cand_v[obase + i] = i < kk ? sv[i] : -INFINITY;
    cand_i[obase + i] = i < kk ? si[i] : -1;
  }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

constexpr int SC_THREADS = 256;
constexpr int SC_MAX = 2048;  // R * K candidates

// cand_v/cand_i: [B][R*K] (R lists of K, each sorted descending). Output token per row.
__global__ __launch_bounds__(SC_THREADS) void sample_candidates_kernel(
    const float* __restrict__ cand_v, const int* __restrict__ cand_i, int n_cand, const float* __restrict__ temps,
    const int* __restrict__ top_ks, const float* __restrict__ top_ps, const unsigned long long* __restrict__ seeds,
    const int* __restrict__ steps, int* out_tok, float* out_logprob) {
  __shared__ float sv[SC_MAX];
  __shared__ int si[SC_MAX];
  const int b = blockIdx.x;
  int n = 1;
  while (n < n_cand) n <<= 1;
  for (int i = threadIdx.x; i < n; i += SC_THREADS) {
    sv[i] = i < n_cand ? cand_v[(size_t)b * n_cand + i] : -INFINITY;
    si[i] = i < n_cand ? cand_i[(size_t)b * n_cand + i] : 0x7fffffff;
  }
  __syncthreads();
  bitonic_desc(sv, si, n);
  if (threadIdx.x != 0) return;
  const float T = temps[b];
  int K = top_ks[b];
  if (K <= 0 || K > n_cand) K = n_cand;
  // drop -inf / invalid tail
  int valid = 0;
  while (valid < K && sv[valid] > -INFINITY && si[valid] >= 0) ++valid;
  if (valid == 0) { out_tok[b] = 0; if (out_logprob) out_logprob[b] = -INFINITY; return; }
  if (!(T > 0.f)) {  // greedy
    out_tok[b] = si[0];
    if (out_logprob) out_logprob[b] = 0.f;
    return;
  }
  const float inv_t = 1.f / T;
  const float m = sv[0] * inv_t;
  float Z = 0.f;
  for (int i = 0; i < valid; ++i) Z += __expf(sv[i] * inv_t - m);
  // top-p: keep token i iff the probability mass ranked strictly above it is < top_p
  const float top_p = top_ps[b];
  int keep = valid;
  if (top_p < 1.f) {
    float cum = 0.f;
    for (int i = 0; i < valid; ++i) {
      if (i > 0 && cum >= top_p) { keep = i; break; }
      cum += __expf(sv[i] * inv_t - m) / Z;
    }
  }
  float Zk = 0.f;
  for (int i = 0; i < keep; ++i) Zk += __expf(sv[i] * inv_t - m);
  const unsigned long long r = splitmix64(seeds[b] ^ splitmix64((unsigned long long)steps[b] + 0x51ED270Bull));
  const float u = (float)((r >> 40) * (1.0 / 16777216.0)) * Zk;
  float c = 0.f;
  int pick = keep - 1;
  for (int i = 0; i < keep; ++i) {
    c += __expf(sv[i] * inv_t - m);
    if (u < c) { pick = i; break; }
  }
  out_tok[b] = si[pick];
  if (out_logprob) out_logprob[b] = (sv[pick] * inv_t - m) - __logf(Zk);
}

}  // namespace

// cand_v / cand_i: [B][chunks*K]
RAGK_API int ragk_topk_candidates(const float* logits, int ld, int B, int V, int K, int vocab_offset, int chunks,
                                  float* cand_v, int* cand_i, hipStream_t st) {
  if (B <= 0) return 0;
  if (K < 1 || K > MAXK || chunks < 1 || chunks > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_candidates_kernel, dim3(B * chunks), dim3(TK_THREADS), 0, st, logits, ld, V, K, vocab_offset,
                     chunks, cand_v, cand_i);
  return (int)hipGetLastError();
}

RAGK_API int ragk_sample_candidates(const float* cand_v, const int* cand_i, int B, int n_cand, const float* temps,
                                    const int* top_ks, const float* top_ps, const unsigned long long* seeds,
                                    const int* steps, int* out_tok, float* out_logprob, hipStream_t st) {
  if (B <= 0) return 0;
  if (n_cand < 1 || n_cand > SC_MAX) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_candidates_kernel, dim3(B), dim3(SC_THREADS), 0, st, cand_v, cand_i, n_cand, temps, top_ks,
                     top_ps, seeds, steps, out_tok, out_logprob);
  return (int)hipGetLastError();
}
