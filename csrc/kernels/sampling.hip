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
#include <float.h>
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

// LDS-resident variant (chunks of up to TK_VMAX entries, i.e. every chunk of a 128k vocab split 7
// ways): the chunk's keys are read from HBM once into LDS, the four 8-bit radix passes count into 16
// per-wave histograms (no single hot LDS counter for the common exponent byte), and wave 0 finds the
// bin with a shuffle scan instead of a serial 256-step walk by one thread. Ties at the K-th value take
// the lowest vocabulary ids (deterministic).
constexpr int TK_VMAX = 24576;
constexpr int TK_WAVES = TK_THREADS / 64;

__global__ __launch_bounds__(TK_THREADS) void topk_lds_kernel(const float* __restrict__ logits, int ld, int Vtot,
                                                              int K, int vocab_offset, int chunks,
                                                              float* cand_v, int* cand_i) {
  extern __shared__ __attribute__((aligned(16))) unsigned tk_smem[];
  unsigned* whist = tk_smem;                   // [TK_WAVES][256]
  unsigned* skey = tk_smem + TK_WAVES * 256;   // [Vc] order-preserving keys
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_krem, s_eqtot, s_cnt_gt, s_cnt_eq;
  __shared__ float sv[MAXK];
  __shared__ int si[MAXK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x / chunks, chunk = blockIdx.x % chunks;
  const int Vc = ((Vtot + chunks - 1) / chunks + 7) & ~7;
  const int c0 = min(chunk * Vc, Vtot);
  const int V = min(Vtot - c0, Vc);
  const size_t obase = ((size_t)b * chunks + chunk) * K;
  if (V <= 0) {  // block-uniform: an empty chunk of a short row
    for (int i = tid; i < K; i += TK_THREADS) {
      cand_v[obase + i] = -INFINITY;
      cand_i[obase + i] = -1;
    }
    return;
  }
  const float* row = logits + (size_t)b * ld + c0;
  for (int i = tid; i < V; i += TK_THREADS) skey[i] = fkey(row[i]);
  unsigned prefix = 0, mask = 0, krem = (unsigned)min(K, V);
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < TK_WAVES * 256; i += TK_THREADS) whist[i] = 0;
    __syncthreads();
    for (int i = tid; i < V; i += TK_THREADS) {
      const unsigned k = skey[i];
      if ((k & mask) == prefix) atomicAdd(&whist[wid * 256 + ((k >> shift) & 255)], 1u);
    }
    __syncthreads();
    if (tid < 256) {
      unsigned h = 0;
#pragma unroll
      for (int w = 0; w < TK_WAVES; ++w) h += whist[w * 256 + tid];
      hist[tid] = h;
    }
    __syncthreads();
    if (wid == 0) {  // lane l owns bins 255-4l .. 252-4l; scan from the top
      unsigned c[4], tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * lane - j];
        tot += c[j];
      }
      unsigned incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      const unsigned excl = incl - tot;
      if (excl < krem && krem <= incl) {  // exactly one lane
        unsigned above = excl;
        int d = 255 - 4 * lane - 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (above + c[j] >= krem) {
            d = 255 - 4 * lane - j;
            break;
          }
          above += c[j];
        }
        s_prefix = prefix | ((unsigned)d << shift);
        s_krem = krem - above;
        s_eqtot = hist[d];
      }
    }
    __syncthreads();
    prefix = s_prefix;
    krem = s_krem;
    mask |= 255u << shift;
  }
  // prefix = key of the K-th largest: every key > prefix, plus the krem lowest-id keys == prefix
  const int kk = min(K, V);
  const unsigned n_gt = (unsigned)kk - krem;
  if (tid == 0) { s_cnt_gt = 0; s_cnt_eq = 0; }
  for (int i = tid; i < MAXK; i += TK_THREADS) { sv[i] = -INFINITY; si[i] = 0x7fffffff; }
  __syncthreads();
  const bool all_eq = s_eqtot == krem;
  for (int i = tid; i < V; i += TK_THREADS) {
    const unsigned k = skey[i];
    if (k > prefix) {
      const unsigned slot = atomicAdd(&s_cnt_gt, 1u);
      if (slot < (unsigned)MAXK) { sv[slot] = unkey(k); si[slot] = i + vocab_offset + c0; }
    } else if (k == prefix && all_eq) {
      const unsigned slot = n_gt + atomicAdd(&s_cnt_eq, 1u);
      if (slot < (unsigned)MAXK) { sv[slot] = unkey(k); si[slot] = i + vocab_offset + c0; }
    }
  }
  if (!all_eq && tid == 0) {  // ties beyond the K-th value (rare): the lowest ids, in order
    unsigned e = 0;
    for (int i = 0; i < V && e < krem; ++i)
      if (skey[i] == prefix) {
        const unsigned slot = n_gt + e++;
        if (slot < (unsigned)MAXK) { sv[slot] = unkey(prefix); si[slot] = i + vocab_offset + c0; }
      }
  }
  __syncthreads();
  int n = 1;
  while (n < kk) n <<= 1;
  bitonic_desc(sv, si, n);
  for (int i = tid; i < K; i += TK_THREADS) {
    cand_v[obase + i] = i < kk ? sv[i] : -INFINITY;
    cand_i[obase + i] = i < kk ? si[i] : -1;
  }
}

// Small-batch top-K (decode batch <= 4): many short chunks (~4k logits) so one row's selection spreads
// over ~32 CUs, each chunk selected without radix passes. Keys = -logit (ascending = best first), ties
// -> lower vocab id. Per wave (its ~1k logits, all in registers):
//   1. every lane's best element; the 64 lane bests sorted by one network -> a valid top-64 list L;
//   2. T = L[K-1]: at least K elements precede or equal it, so only elements strictly before T (other
//      than the lane bests already in L) can still enter the top K -- on logits ~9 % of them;
//   3. those survivors are compacted through LDS (wave prefix count) and offered 64 at a time.
// Offering every 64-logit tile instead cost a full 27-step network on nearly every tile (each tile of
// a not-yet-warm list improves it): ~16 networks per wave, ~20 us per row at batch 1. The block then
// merges its 4 lists. Output as topk_lds: K candidates per chunk, value descending, ids ascending
// within equal values.
constexpr int TW_THREADS = 256;
constexpr int TW_VMAX = 6144;  // chunk sizes this kernel takes (larger chunks: topk_lds)
constexpr int TW_NT = TW_VMAX / 256;  // logits per lane

__global__ __launch_bounds__(TW_THREADS) void topk_wave_kernel(const float* __restrict__ logits, int ld, int Vtot,
                                                               int K, int vocab_offset, int chunks, float* cand_v,
                                                               int* cand_i) {
  __shared__ float mv[4][64];
  __shared__ int mi[4][64];
  __shared__ float sk[4][TW_NT * 64];  // per-wave survivor keys / ids (worst case: every logit)
  __shared__ int sid[4][TW_NT * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x / chunks, chunk = blockIdx.x % chunks;
  const int Vc = ((Vtot + chunks - 1) / chunks + 7) & ~7;
  const int c0 = min(chunk * Vc, Vtot);
  const int V = min(Vtot - c0, Vc);
  const float* row = logits + (size_t)b * ld + c0;
  const int id0 = vocab_offset + c0;
  // element t of this lane: chunk index w*64 + lane + 256 t (loads unconditional, index clamped)
  float key[TW_NT];
#pragma unroll
  for (int t = 0; t < TW_NT; ++t) key[t] = -row[min(w * 64 + lane + 256 * t, V - 1)];  // (V = 0: row[-1], in the row)
  auto elem_id = [&](int t) { return w * 64 + lane + 256 * t; };
  // 1. lane best (padding sorts after real -inf logits: key +inf, id -1 = 0xffffffff unsigned)
  float bv = INFINITY;
  int bi = -1, bt = -1;
#pragma unroll
  for (int t = 0; t < TW_NT; ++t) {
    const int e = elem_id(t);
    const bool ok = e < V;
    const float kv = ok ? key[t] : INFINITY;
    const int id = ok ? id0 + e : -1;
    const bool take = cand_lt(kv, id, bv, bi);
    bv = take ? kv : bv;
    bi = take ? id : bi;
    bt = take ? t : bt;
  }
  // 2. sorted list of the lane bests; threshold = its K-th entry
  wave_sort64(bv, bi, lane);
  const float tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv), K - 1));
  const int ti = __builtin_amdgcn_readlane(bi, K - 1);
  // 3. survivors (strictly before the threshold, not this lane's best) -> LDS, compacted
  int cnt = 0;
#pragma unroll
  for (int t = 0; t < TW_NT; ++t) {
    const int e = elem_id(t);
    cnt += (e < V && t != bt && cand_lt(key[t], id0 + e, tv, ti)) ? 1 : 0;
  }
  int incl = cnt;  // inclusive prefix over lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  const int total = __shfl(incl, 63, 64);
  if (total > 0) {
    int pos = incl - cnt;
#pragma unroll
    for (int t = 0; t < TW_NT; ++t) {
      const int e = elem_id(t);
      if (e < V && t != bt && cand_lt(key[t], id0 + e, tv, ti)) {
        sk[w][pos] = key[t];
        sid[w][pos] = id0 + e;
        ++pos;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's survivor writes landed
    __builtin_amdgcn_wave_barrier();
    for (int base = 0; base < total; base += 64) {
      const bool ok = base + lane < total;
      wave_offer(bv, bi, ok ? sk[w][base + lane] : INFINITY, ok ? sid[w][base + lane] : -1, K, lane);
    }
  }
  mv[w][lane] = bv;
  mi[w][lane] = bi;
  __syncthreads();
  if (w == 0) {
    for (int g = 1; g < 4; ++g) wave_merge64(bv, bi, mv[g][lane], mi[g][lane], lane);
    if (lane < K) {
      const size_t o = ((size_t)b * chunks + chunk) * K + lane;
      cand_v[o] = bi >= 0 ? -bv : -INFINITY;
      cand_i[o] = bi;
    }
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
    const int* __restrict__ steps, int* out_tok, float* out_logprob, int list_len) {
  __shared__ float sv[SC_MAX];
  __shared__ int si[SC_MAX];
  __shared__ float mv[64];
  __shared__ int mi[64];
  const int b = blockIdx.x;
  int K = top_ks[b];
  if (K <= 0 || K > n_cand) K = n_cand;
  if (K <= 64 && list_len > 0 && list_len <= 64 && n_cand / list_len > 8) {
    // Many lists (small-batch chunked top-k, x TP ranks): merged by the lane network -- wave w folds
    // lists w, w + 4, ... into its running sorted top-64 (keys = -value), then wave 0 folds the four.
    const int R = n_cand / list_len;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float bv = INFINITY;
    int bi = -1;
    for (int r = w; r < R; r += SC_THREADS / 64) {
      const size_t o = (size_t)b * n_cand + (size_t)r * list_len + lane;
      const int id = lane < list_len ? cand_i[o] : -1;
      const float v = lane < list_len ? cand_v[o] : -INFINITY;
      wave_merge64(bv, bi, id >= 0 ? -v : INFINITY, id, lane);
    }
    sv[w * 64 + lane] = bv;
    si[w * 64 + lane] = bi;
    __syncthreads();
    if (w == 0) {
      for (int g = 1; g < SC_THREADS / 64; ++g) wave_merge64(bv, bi, sv[g * 64 + lane], si[g * 64 + lane], lane);
      mv[lane] = bi >= 0 ? -bv : -INFINITY;
      mi[lane] = bi;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      sv[threadIdx.x] = mv[threadIdx.x];
      si[threadIdx.x] = mi[threadIdx.x];
    }
    __syncthreads();
  } else if (K <= 64 && list_len > 0) {
    // The candidate lists (R = n_cand / list_len of them) are each sorted in the total order
    // (value desc, vocabulary id asc as unsigned, position asc): the global top-64 is found by
    // ranking every candidate -- its position in its own list plus a binary search per other list --
    // and scattering the ones ranked < 64 (one barrier instead of a 512-entry bitonic sort's 45).
    for (int i = threadIdx.x; i < n_cand; i += SC_THREADS) {
      sv[i] = cand_v[(size_t)b * n_cand + i];
      si[i] = cand_i[(size_t)b * n_cand + i];
    }
    if (threadIdx.x < 64) {
      mv[threadIdx.x] = -INFINITY;
      mi[threadIdx.x] = -1;
    }
    __syncthreads();
    const int R = n_cand / list_len;
    for (int c = threadIdx.x; c < n_cand; c += SC_THREADS) {
      const float v = sv[c];
      const unsigned ix = (unsigned)si[c];
      const int own = c / list_len;
      int rank = c - own * list_len;
      for (int j = 0; j < R; ++j) {
        if (j == own) continue;
        // count of list j's entries that precede c: (v' > v) or (v' == v and (ix' < ix or (ix' == ix and j < own)))
        int lo = 0, hi = list_len;
        const int base = j * list_len;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const float w = sv[base + mid];
          const unsigned iw = (unsigned)si[base + mid];
          const bool before = w > v || (w == v && (iw < ix || (iw == ix && j < own)));
          if (before) lo = mid + 1; else hi = mid;
        }
        rank += lo;
        if (rank >= 64) break;
      }
      if (rank < 64) {
        mv[rank] = v;
        mi[rank] = (int)ix;
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      sv[threadIdx.x] = mv[threadIdx.x];
      si[threadIdx.x] = mi[threadIdx.x];
    }
    __syncthreads();
  } else {
    int n = 1;
    while (n < n_cand) n <<= 1;
    for (int i = threadIdx.x; i < n; i += SC_THREADS) {
      sv[i] = i < n_cand ? cand_v[(size_t)b * n_cand + i] : -INFINITY;
      si[i] = i < n_cand ? cand_i[(size_t)b * n_cand + i] : 0x7fffffff;
    }
    __syncthreads();
    bitonic_desc(sv, si, n);
  }
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const float T = temps[b];
  const unsigned long long r = splitmix64(seeds[b] ^ splitmix64((unsigned long long)steps[b] + 0x51ED270Bull));
  const float top_p = top_ps[b];
  if (K > 64) {  // wide top-k (or top_k disabled): the serial tail
    if (lane != 0) return;
    int valid = 0;
    while (valid < K && sv[valid] > -INFINITY && si[valid] >= 0) ++valid;
    if (valid == 0) { out_tok[b] = 0; if (out_logprob) out_logprob[b] = -INFINITY; return; }
    if (!(T > 0.f)) { out_tok[b] = si[0]; if (out_logprob) out_logprob[b] = 0.f; return; }
    const float inv_t = 1.f / T;
    const float m = sv[0] * inv_t;
    float Z = 0.f;
    for (int i = 0; i < valid; ++i) Z += __expf(sv[i] * inv_t - m);
    // top-p: keep token i iff the probability mass ranked strictly above it is < top_p
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
    const float u = (float)((r >> 40) * (1.0 / 16777216.0)) * Zk;
    float c = 0.f;
    int pick = keep - 1;
    for (int i = 0; i < keep; ++i) {
      c += __expf(sv[i] * inv_t - m);
      if (u < c) { pick = i; break; }
    }
    out_tok[b] = si[pick];
    if (out_logprob) out_logprob[b] = (sv[pick] * inv_t - m) - __logf(Zk);
    return;
  }
  // K <= 64: one candidate per lane of wave 0, reductions and scans by shuffles
  const float v = lane < K ? sv[lane] : -INFINITY;
  const int ix = lane < K ? si[lane] : -1;
  const bool ok = lane < K && v > -INFINITY && ix >= 0;  // sorted: the valid ones lead
  const unsigned long long okm = __ballot(ok);
  const int valid = okm == ~0ull ? 64 : __builtin_ctzll(~okm);
  if (valid == 0) {
    if (lane == 0) { out_tok[b] = 0; if (out_logprob) out_logprob[b] = -INFINITY; }
    return;
  }
  if (!(T > 0.f)) {  // greedy
    if (lane == 0) { out_tok[b] = ix; if (out_logprob) out_logprob[b] = 0.f; }
    return;
  }
  const float inv_t = 1.f / T;
  const float m = __shfl(v, 0, 64) * inv_t;
  const float e = lane < valid ? __expf(v * inv_t - m) : 0.f;
  const float Z = wave_sum(e);
  float incl = e;  // inclusive prefix of e over lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  // top-p: keep token i iff the probability mass ranked strictly above it is < top_p
  const bool kept = lane < valid && (top_p >= 1.f || lane == 0 || (incl - e) / Z < top_p);
  const float ek = kept ? e : 0.f;
  const float Zk = wave_sum(ek);
  const float u = (float)((r >> 40) * (1.0 / 16777216.0)) * Zk;
  float ck = ek;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(ck, o, 64);
    if (lane >= o) ck += t;
  }
  const unsigned long long hit = __ballot(kept && u < ck);
  const unsigned long long keptm = __ballot(kept);
  const int pick = hit ? __builtin_ctzll(hit) : 63 - __builtin_clzll(keptm);
  const float pv = __shfl(v, pick, 64);
  const int pix = __shfl(ix, pick, 64);
  if (lane == 0) {
    out_tok[b] = pix;
    if (out_logprob) out_logprob[b] = (pv * inv_t - m) - __logf(Zk);
  }
}

}  // namespace

// cand_v / cand_i: [B][chunks*K]
RAGK_API int ragk_topk_candidates(const float* logits, int ld, int B, int V, int K, int vocab_offset, int chunks,
                                  float* cand_v, int* cand_i, hipStream_t st) {
  if (B <= 0) return 0;
  if (K < 1 || K > MAXK || chunks < 1 || chunks > 64) return (int)hipErrorInvalidValue;
  const int Vc = ((V + chunks - 1) / chunks + 7) & ~7;
  if (K <= 64 && Vc <= TW_VMAX && chunks >= 8) {  // small batch, many short chunks
    hipLaunchKernelGGL(topk_wave_kernel, dim3(B * chunks), dim3(TW_THREADS), 0, st, logits, ld, V, K, vocab_offset,
                       chunks, cand_v, cand_i);
    return (int)hipGetLastError();
  }
  if (Vc <= TK_VMAX) {
    static bool attr = false;  // > 64 KiB of dynamic LDS needs the opt-in
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)topk_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (TK_WAVES * 256 + TK_VMAX) * 4);
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    hipLaunchKernelGGL(topk_lds_kernel, dim3(B * chunks), dim3(TK_THREADS), (TK_WAVES * 256 + Vc) * 4, st, logits, ld,
                       V, K, vocab_offset, chunks, cand_v, cand_i);
    return (int)hipGetLastError();
  }
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
                     top_ps, seeds, steps, out_tok, out_logprob, 0);
  return (int)hipGetLastError();
}

// As ragk_sample_candidates for candidates that arrive as n_cand / list_len lists of list_len, each
// sorted (topk_candidates output, all-gathered per TP rank): rows with top_k <= 64 rank-merge the
// lists instead of sorting all candidates.
RAGK_API int ragk_sample_candidates_lists(const float* cand_v, const int* cand_i, int B, int n_cand, int list_len,
                                          const float* temps, const int* top_ks, const float* top_ps,
                                          const unsigned long long* seeds, const int* steps, int* out_tok,
                                          float* out_logprob, hipStream_t st) {
  if (B <= 0) return 0;
  if (n_cand < 1 || n_cand > SC_MAX || list_len < 1 || n_cand % list_len) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_candidates_kernel, dim3(B), dim3(SC_THREADS), 0, st, cand_v, cand_i, n_cand, temps, top_ks,
                     top_ps, seeds, steps, out_tok, out_logprob, list_len);
  return (int)hipGetLastError();
}
