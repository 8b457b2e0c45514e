// Exact squared-L2 k-nearest-neighbour search for gfx950 (faiss IndexFlatL2
// semantics: squared distances, ascending, ties -> lower id, missing results = (-1, FLT_MAX)).
// Reference: faiss index.search at /root/reference/llm/rag.py:116.
//
// The database stays resident in HBM in a COLUMN-major layout xt[d][cap] (cap = row
// capacity): lane l of a wave reads row r0 + l of one dimension per load, 256 contiguous
// bytes per wave instruction, no LDS for the data. Queries are staged in LDS in 256-dim
// chunks and read as broadcasts. Distances are sum((x - q)^2) in fp32 (faiss' exact path).
//
// Top-k without sorting the scanned rows: every wave keeps a RUNNING sorted top-64 list per
// query in its lanes (lane j = j-th best). A tile of 64 fresh distances (one per lane) is
// skipped outright when none beats the current k-th best (after the first few tiles almost
// all of them); otherwise it is bitonic-sorted across the lanes (21 shuffle steps) and merged
// into the running list (min against the reversed list + 6 bitonic-merge steps).
//   l2_scan:   grid (row-tile groups, query groups); each block loops over its row tiles and
//              emits one sorted top-k per query -> partial lists [nq][G][k]
//   ivf_scan:  the same per (query, probe): the probed inverted list's row range
//   topk_lists_merge: one block per query merges the G sorted lists with the same wave
//              machinery (64 candidates per step, skip test first).
// Small indexes split each row tile's dimensions over S waves (S = 4 below 64k rows) so that
// a 10k-row index still spreads over ~160 blocks; the partial sums are added in slice order.
#include "common.h"
#include <float.h>
using namespace ragk;

namespace {

constexpr int ST = 256;   // threads per block (4 waves)
constexpr int DCH = 256;  // query dims staged per LDS chunk
constexpr int UNR = 16;   // dims (independent loads) in flight per lane

// wave_offer for QB queries at once (the same 64 rows, one candidate per lane and query): the QB
// bitonic networks run interleaved step by step, so the cross-lane permutes of one query's
// dependent chain hide behind the others' (one query at a time left a 16-query block
// latency-bound on ~28 dependent permute round trips per query). Skipped outright when no query's
// candidates beat its current k-th best.
template <int QB>
__device__ __forceinline__ void wave_offer_q(float (&bv)[QB], int (&bi)[QB], float (&v)[QB], int id, int nqb, int k,
                                             int lane) {
  bool any = false;
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    if (q < nqb) {
      const float tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv[q]), k - 1));
      const int ti = __builtin_amdgcn_readlane(bi[q], k - 1);
      any |= __any(cand_lt(v[q], id, tv, ti));
    }
  }
  if (!any) return;  // wave-uniform
  int ix[QB];
#pragma unroll
  for (int q = 0; q < QB; ++q) ix[q] = id;
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int q = 0; q < QB; ++q) cx(v[q], ix[q], lane, j, (lane & kk) == 0);
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const float rv = rev_lane(v[q], lane);
    const int ri = rev_lane(ix[q], lane);
    if (cand_lt(rv, ri, bv[q], bi[q])) {
      bv[q] = rv;
      bi[q] = ri;
    }
  }
#pragma unroll
  for (int j = 32; j > 0; j >>= 1)
#pragma unroll
    for (int q = 0; q < QB; ++q) cx(bv[q], bi[q], lane, j, true);
}

// As wave_offer_q with a separate candidate id per query (lists of different queries).
template <int NQ>
__device__ __forceinline__ void wave_offer_multi(float (&bv)[NQ], int (&bi)[NQ], float (&v)[NQ], int (&ix)[NQ], int k,
                                                 int lane) {
  bool any = false;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv[q]), k - 1));
    const int ti = __builtin_amdgcn_readlane(bi[q], k - 1);
    any |= __any(cand_lt(v[q], ix[q], tv, ti));
  }
  if (!any) return;
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int q = 0; q < NQ; ++q) cx(v[q], ix[q], lane, j, (lane & kk) == 0);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float rv = rev_lane(v[q], lane);
    const int ri = rev_lane(ix[q], lane);
    if (cand_lt(rv, ri, bv[q], bi[q])) {
      bv[q] = rv;
      bi[q] = ri;
    }
  }
#pragma unroll
  for (int j = 32; j > 0; j >>= 1)
#pragma unroll
    for (int q = 0; q < NQ; ++q) cx(bv[q], bi[q], lane, j, true);
}

// Distances of rows [rbase, rbase + 64) (one per lane; rows clamped into [0, cap)) over dims
// [t0, t1) of the staged chunk starting at dim dc, for QB queries.
template <int QB, int U = (QB <= 2 ? 32 : UNR)>
__device__ __forceinline__ void scan_dims(const float* __restrict__ xt, size_t cap, int rc, int dc, int t0, int t1,
                                          const float* qs, float* acc) {
  const float* col = xt + (size_t)(dc + t0) * cap + rc;
  int t = t0;
  for (; t + U <= t1; t += U, col += U * cap) {
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = col[(size_t)u * cap];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const float df = x[u] - qs[j * DCH + t + u];
        acc[j] = fmaf(df, df, acc[j]);
      }
  }
  for (; t < t1; ++t, col += cap) {
    const float x = *col;
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      const float df = x - qs[j * DCH + t];
      acc[j] = fmaf(df, df, acc[j]);
    }
  }
}

// Flat scan. Row tile = 64 * (4 / S) rows: wave w scans rows 64 * (w / S) .. +63 of the tile over
// dim slice w % S of every 256-dim chunk. Block bx handles tiles bx, bx + gridDim.x, ...; its
// queries are q0 = blockIdx.y * QB .. + QB. Output: per query one sorted list of k at [q][bx].
template <int QB, int S>
__global__ __launch_bounds__(ST) void l2_scan_kernel(const float* __restrict__ xt, int cap, int d, int row_begin,
                                                     int row_end, int ntiles, const float* __restrict__ q, int nq,
                                                     int k, float* __restrict__ out_d, int* __restrict__ out_i,
                                                     const int* __restrict__ ids_map) {
  constexpr int RG = 4 / S;
  constexpr int RB = 64 * RG;
  extern __shared__ __attribute__((aligned(16))) float sc_smem[];
  float* qs = sc_smem;              // [QB][DCH]
  float* red = sc_smem + QB * DCH;  // [S - 1][RG][QB][64]
  __shared__ float mv[4][64];
  __shared__ int mi[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = w / S, s = w % S;
  const int q0 = blockIdx.y * QB;
  const int nqb = min(QB, nq - q0);
  float bv[QB];
  int bi[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    bv[j] = FLT_MAX;
    bi[j] = -1;
  }
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row = row_begin + tile * RB + 64 * g + lane;
    const int rc = min(row, cap - 1);  // rows in [row_end, cap) are valid memory; masked below
    float acc[QB];
#pragma unroll
    for (int j = 0; j < QB; ++j) acc[j] = 0.f;
    for (int dc = 0; dc < d; dc += DCH) {
      const int dn = min(DCH, d - dc);
      __syncthreads();  // previous chunk (and the previous tile's slice reduction) consumed
      for (int e = threadIdx.x; e < QB * DCH; e += ST) {
        const int j = e / DCH, t = e % DCH;
        qs[e] = (j < nqb && t < dn) ? q[(size_t)(q0 + j) * d + dc + t] : 0.f;
      }
      __syncthreads();
      const int per = (dn + S - 1) / S;
      const int t0 = min(dn, s * per), t1 = min(dn, t0 + per);
      scan_dims<QB>(xt, (size_t)cap, rc, dc, t0, t1, qs, acc);
    }
    if (S > 1) {
      if (s > 0) {
#pragma unroll
        for (int j = 0; j < QB; ++j) red[(((s - 1) * RG + g) * QB + j) * 64 + lane] = acc[j];
      }
      __syncthreads();
      if (s == 0) {
#pragma unroll
        for (int ss = 1; ss < S; ++ss)
#pragma unroll
          for (int j = 0; j < QB; ++j) acc[j] += red[(((ss - 1) * RG + g) * QB + j) * 64 + lane];
      }
    }
    if (s == 0) {  // wave-uniform
      const bool ok = row < row_end;
      const int id = ok ? (ids_map ? ids_map[row] : row) : -1;
#pragma unroll
      for (int j = 0; j < QB; ++j) acc[j] = (ok && j < nqb) ? acc[j] : FLT_MAX;
      wave_offer_q<QB>(bv, bi, acc, ok ? id : -1, nqb, k, lane);
    }
  }
  // block merge: the RG list-holding waves (s == 0) -> wave 0 -> k outputs per query
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    if (j >= nqb) continue;  // block-uniform
    if (RG > 1) {
      __syncthreads();
      if (s == 0 && g > 0) {
        mv[g][lane] = bv[j];
        mi[g][lane] = bi[j];
      }
      __syncthreads();
      if (w == 0)
        for (int gg = 1; gg < RG; ++gg) wave_merge64(bv[j], bi[j], mv[gg][lane], mi[gg][lane], lane);
    }
    if (w == 0 && lane < k) {
      const size_t o = ((size_t)(q0 + j) * gridDim.x + blockIdx.x) * k + lane;
      out_d[o] = bv[j];
      out_i[o] = bi[j];
    }
  }
}

// Batched queries (nq >= 16: the BLAS path of faiss' IndexFlatL2): ||x||^2 + ||q||^2 - 2 x.q with the
// dot products on the exact fp32-input MFMA (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain), 16 rows x
// 16 queries per instruction. Block = 4 waves x 64 rows per iteration, QT query tiles of 16 (all of a
// <= 32-query batch in one block: the index is streamed from HBM once). Lane l of a wave loads
// x[row0 + 16 rt + (l & 15)][k0 + (l >> 4)] (A fragment) and reads q^T[k0 + (l >> 4)][16 qt + (l & 15)]
// from LDS (B fragment); its accumulators hold rows 16 rt + 4 (l >> 4) + r of query 16 qt + (l & 15).
// Selection: every lane keeps a sorted list of the MK best (distance, id) of its query among the rows
// it sees (MK >= k; a quarter of the rows of its query per wave), and the block merges the 16 lists of
// each query (4 lanes x 4 waves) -> one sorted list of k per query. Distances clamp at 0 like faiss.
constexpr int MQ_MK = 8;   // k <= 8 on this path
constexpr int MQ_KU = 8;   // k-steps (of 4 dims) per unrolled group
constexpr int MQ_DMAX = 1024;

constexpr int MQ_DCH = 256;  // query dims staged per LDS chunk (4 blocks per CU fit)
// LDS floats of region 0: a q^T chunk during the scan, the candidate lists at the merge (aliased)
__host__ __device__ inline int mq_region0(int d, int QT) {
  return max(min(d, MQ_DCH) * 16 * QT, 2 * 16 * QT * 128);
}

template <int QT, int RT>
__global__ __launch_bounds__(ST) void l2_mfma_kernel(const float* __restrict__ xt, int cap, int d, int row_begin,
                                                     int row_end, int ntiles, const float* __restrict__ q, int nq,
                                                     int k, float* __restrict__ out_d, int* __restrict__ out_i,
                                                     const int* __restrict__ ids_map) {
  extern __shared__ __attribute__((aligned(16))) float mq_smem[];
  float* qsT = mq_smem;                              // [MQ_DCH][16 * QT]: q transposed, one dim chunk
  float* cd = mq_smem;                               // [16 * QT][128] candidates (merge, aliases qsT)
  int* ci = reinterpret_cast<int*>(mq_smem + 16 * QT * 128);
  float* qn = mq_smem + mq_region0(d, QT);           // [16 * QT] ||q||^2
  float* xnl = qn + 16 * QT;                         // [4 waves][16 * RT] ||x||^2 of the wave's rows
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q0 = blockIdx.y * 16 * QT;
  const int nqb = min(16 * QT, nq - q0);
  {
    // ||q||^2 by the whole block: query j = tid / QP, part p = tid % QP sums dims p, p + QP, ...
    // (consecutive threads read consecutive floats, 8 loads in flight), parts summed in order by
    // shuffles. One thread per query walking all d dims with a dependent load each was ~60 us of a
    // 10k-row search.
    constexpr int QP = ST / (16 * QT);  // parts per query: 8 (QT 2) or 16 (QT 1)
    const int j = threadIdx.x / QP, p = threadIdx.x % QP;
    float sq = 0.f;
    if (j < nqb) {
      const float* qr = q + (size_t)(q0 + j) * d;
      int t = p;
      for (; t + 7 * QP < d; t += 8 * QP) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = qr[t + u * QP];
#pragma unroll
        for (int u = 0; u < 8; ++u) sq = fmaf(v[u], v[u], sq);
      }
      for (; t < d; t += QP) sq = fmaf(qr[t], qr[t], sq);
    }
#pragma unroll
    for (int o = 1; o < QP; o <<= 1) sq += __shfl_xor(sq, o, 64);
    if (p == 0) qn[j] = sq;
  }
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  // per-lane sorted lists, one per query tile
  float lv[QT][MQ_MK];
  int lix[QT][MQ_MK];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int m = 0; m < MQ_MK; ++m) {
      lv[qt][m] = FLT_MAX;
      lix[qt][m] = -1;
    }
  float qnv[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) qnv[qt] = qn[16 * qt + fr];
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int rbase = row_begin + tile * (64 * RT) + 16 * RT * w;
    int rc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) rc[rt] = min(rbase + 16 * rt + fr, cap - 1);
    f32x4 acc[RT][QT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) acc[rt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float xs[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) xs[rt] = 0.f;
    for (int dc = 0; dc < d; dc += MQ_DCH) {
    const int dn = min(MQ_DCH, d - dc);  // host guarantees d % (4 * MQ_KU) == 0
    __syncthreads();  // every wave is done with the previous chunk
    // q^T chunk: consecutive threads read consecutive dims of one query (coalesced; the transposed LDS
    // writes are the cheap side)
    // (8 loads per thread in flight: a one-at-a-time loop paid a full L2 latency per element)
    const int tot = dn * 16 * QT;
    for (int e0 = threadIdx.x; e0 < tot; e0 += 16 * ST) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = min(e0 + u * ST, tot - 1);
        const int j = e / dn, t = e % dn;
        v[u] = q[(size_t)(q0 + min(j, nqb - 1)) * d + dc + t];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = e0 + u * ST;
        if (e < tot) {
          const int j = e / dn, t = e % dn;
          qsT[t * 16 * QT + j] = j < nqb ? v[u] : 0.f;
        }
      }
    }
    __syncthreads();
    // index columns of the next group of MQ_KU k-steps are requested before the current group's
    // MFMAs (two register buffers, loop unrolled by two): one group at a time left every group
    // waiting a full memory latency (12 round trips per 384-dim tile)
    const int nk = dn / 4;  // multiple of MQ_KU
    auto load_grp = [&](int k0, float (&a)[MQ_KU][RT]) {
#pragma unroll
      for (int u = 0; u < MQ_KU; ++u) {
        const float* col = xt + (size_t)(dc + 4 * (k0 + u) + fg) * cap;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) a[u][rt] = col[rc[rt]];
      }
    };
    auto mma_grp = [&](int k0, const float (&a)[MQ_KU][RT]) {
#pragma unroll
      for (int u = 0; u < MQ_KU; ++u) {
        float b[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) b[qt] = qsT[(4 * (k0 + u) + fg) * 16 * QT + 16 * qt + fr];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          xs[rt] = fmaf(a[u][rt], a[u][rt], xs[rt]);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt)
            acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][rt], b[qt], acc[rt][qt], 0, 0, 0);
        }
      }
    };
    // three register buffers, two groups in flight ahead of the MFMAs (a group's 8 k-steps of MFMA
    // are far shorter than one memory latency)
    float a0[MQ_KU][RT], a1[MQ_KU][RT], a2[MQ_KU][RT];
    load_grp(0, a0);
    if (MQ_KU < nk) load_grp(MQ_KU, a1);
    for (int k0 = 0; k0 < nk; k0 += 3 * MQ_KU) {
      if (k0 + 2 * MQ_KU < nk) load_grp(k0 + 2 * MQ_KU, a2);
      mma_grp(k0, a0);
      if (k0 + MQ_KU >= nk) break;
      if (k0 + 3 * MQ_KU < nk) load_grp(k0 + 3 * MQ_KU, a0);
      mma_grp(k0 + MQ_KU, a1);
      if (k0 + 2 * MQ_KU >= nk) break;
      if (k0 + 4 * MQ_KU < nk) load_grp(k0 + 4 * MQ_KU, a1);
      mma_grp(k0 + 2 * MQ_KU, a2);
    }
    }  // dim chunk
    // ||x||^2 of row 16 rt + fr: the 4 dim phases (lanes fr, fr+16, fr+32, fr+48) summed in order
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float t = xs[rt];
      t += __int_as_float(xor_lane(__float_as_int(t), 16, lane));
      t += __int_as_float(xor_lane(__float_as_int(t), 32, lane));
      if (fg == 0) xnl[w * 16 * RT + 16 * rt + fr] = t;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's xnl writes landed (wave-local rows)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = 16 * rt + 4 * fg + r;
        const int row = rbase + rl;
        const bool ok = row < row_end;
        const int id = ok ? (ids_map ? ids_map[row] : row) : -1;
        const float xn = xnl[w * 16 * RT + rl];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const float dv = ok ? fmaxf(xn + qnv[qt] - 2.f * acc[rt][qt][r], 0.f) : FLT_MAX;
          if (cand_lt(dv, id, lv[qt][MQ_MK - 1], lix[qt][MQ_MK - 1])) {  // insert (rare once warm)
            float cv = dv;
            int cidx = id;
#pragma unroll
            for (int m = 0; m < MQ_MK; ++m) {
              if (cand_lt(cv, cidx, lv[qt][m], lix[qt][m])) {
                const float tv = lv[qt][m];
                const int ti = lix[qt][m];
                lv[qt][m] = cv;
                lix[qt][m] = cidx;
                cv = tv;
                cidx = ti;
              }
            }
          }
        }
      }
    __builtin_amdgcn_wave_barrier();
  }
  // merge: query j's lists live in lanes with fr == j % 16 of every wave: 4 waves x 4 lane groups x MQ_MK
  __syncthreads();  // every wave is done reading q^T: the candidate lists reuse its LDS
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int m = 0; m < MQ_MK; ++m) {
      const int j = 16 * qt + fr;
      const int slot = (w * 4 + fg) * MQ_MK + m;  // 0 .. 127
      cd[(size_t)j * 128 + slot] = lv[qt][m];
      ci[(size_t)j * 128 + slot] = lix[qt][m];
    }
  __syncthreads();
  // wave w merges queries w, w + 4, ... (4 * QT of them). A query's 128 candidates are 16 sorted
  // lists of MQ_MK: lane l holds entries 2 (l >> 4) and 2 (l >> 4) + 1 of list l & 15 (a sorted pair),
  // and k rounds of a wave-wide argmin over the lanes' first entries emit the top k in order (the
  // winner shifts its pair). Two full 64-lane bitonic offers per query cost ~3x the steps for k <= 8.
  {
    constexpr int NQW = 4 * QT;
    float v0[NQW], v1[NQW];
    int i0[NQW], i1[NQW];
    const int slot = (lane & 15) * MQ_MK + 2 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < NQW; ++t) {
      const int j = w + 4 * t;
      v0[t] = cd[(size_t)j * 128 + slot];
      i0[t] = ci[(size_t)j * 128 + slot];
      v1[t] = cd[(size_t)j * 128 + slot + 1];
      i1[t] = ci[(size_t)j * 128 + slot + 1];
    }
    for (int r = 0; r < k; ++r) {
      float mv[NQW];
      int mi[NQW];
#pragma unroll
      for (int t = 0; t < NQW; ++t) {
        mv[t] = v0[t];
        mi[t] = i0[t];
      }
#pragma unroll
      for (int jx = 1; jx < 64; jx <<= 1)
#pragma unroll
        for (int t = 0; t < NQW; ++t) {
          const float ov = __int_as_float(xor_lane(__float_as_int(mv[t]), jx, lane));
          const int oi = xor_lane(mi[t], jx, lane);
          const bool take = cand_lt(ov, oi, mv[t], mi[t]);
          mv[t] = take ? ov : mv[t];
          mi[t] = take ? oi : mi[t];
        }
#pragma unroll
      for (int t = 0; t < NQW; ++t) {
        const bool won = (v0[t] == mv[t]) & (i0[t] == mi[t]);
        v0[t] = won ? v1[t] : v0[t];
        i0[t] = won ? i1[t] : i0[t];
        v1[t] = won ? FLT_MAX : v1[t];
        i1[t] = won ? -1 : i1[t];
        const int j = w + 4 * t;
        if (j < nqb && lane == 0) {
          const size_t o = ((size_t)(q0 + j) * gridDim.x + blockIdx.x) * k + r;
          out_d[o] = mv[t];
          out_i[o] = mi[t];
        }
      }
    }
  }
}

// IVF-Flat scan: block (probe p, query qi) scans the whole inverted list probes[qi][p] (store rows
// [offsets[list], ends[list]); packed lists when ends == nullptr: end = offsets[list + 1]) in
// 256-row tiles (one wave per 64 rows) -> one sorted list of k at [qi][p].
constexpr int IVF_DMAX = 2048;
__global__ __launch_bounds__(ST) void ivf_scan_kernel(const float* __restrict__ xt, int cap, int d,
                                                      const float* __restrict__ q, const int* __restrict__ probes,
                                                      int nprobe, const int* __restrict__ offsets,
                                                      const int* __restrict__ ends, const int* __restrict__ ids_map,
                                                      int k, float* __restrict__ out_d, int* __restrict__ out_i) {
  __shared__ float qs[IVF_DMAX];
  __shared__ float mv[4][64];
  __shared__ int mi[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = blockIdx.y, p = blockIdx.x;
  const int list = probes[(size_t)qi * nprobe + p];
  const int lbeg = list >= 0 ? offsets[list] : 0;
  const int lend = list < 0 ? 0 : (ends ? ends[list] : offsets[list + 1]);
  for (int t = threadIdx.x; t < d; t += ST) qs[t] = q[(size_t)qi * d + t];
  __syncthreads();
  float bv = FLT_MAX;
  int bi = -1;
  for (int r0 = lbeg; r0 < lend; r0 += 4 * 64) {
    const int row = r0 + 64 * w + lane;
    const int rc = min(row, cap - 1);
    float acc = 0.f;
    const float* col = xt + rc;
    int t = 0;
    for (; t + UNR <= d; t += UNR, col += (size_t)UNR * cap) {
      float x[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) x[u] = col[(size_t)u * cap];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float df = x[u] - qs[t + u];
        acc = fmaf(df, df, acc);
      }
    }
    for (; t < d; ++t, col += cap) {
      const float df = *col - qs[t];
      acc = fmaf(df, df, acc);
    }
    const bool ok = row < lend;
    wave_offer(bv, bi, ok ? acc : FLT_MAX, ok ? ids_map[row] : -1, k, lane);
  }
  if (w > 0) {
    mv[w][lane] = bv;
    mi[w][lane] = bi;
  }
  __syncthreads();
  if (w == 0) {
    for (int gg = 1; gg < 4; ++gg) wave_merge64(bv, bi, mv[gg][lane], mi[gg][lane], lane);
    if (lane < k) {
      const size_t o = ((size_t)qi * gridDim.x + p) * k + lane;
      out_d[o] = bv;
      out_i[o] = bi;
    }
  }
}

// in: [nq][G][k] sorted lists -> out: [nq][k] (distances fp32, ids int64). One block of MW waves per query; each wave takes 64
// candidates at a time (64 / k whole lists per step) and offers them to its running top list; the
// waves' lists are merged last.
constexpr int MW = 16;
__global__ __launch_bounds__(MW * 64) void topk_lists_merge_kernel(const float* __restrict__ in_d,
                                                                   const int* __restrict__ in_i, int G, int k,
                                                                   float* __restrict__ out_d,
                                                                   long long* __restrict__ out_i) {
  __shared__ float mv[MW][64];
  __shared__ int mi[MW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = blockIdx.x;
  const int lpw = 64 / k;  // whole lists per 64-lane step
  const int li = lane / k, e = lane % k;
  const size_t base = (size_t)qi * G * k;
  float bv = FLT_MAX;
  int bi = -1;
  // software-pipelined: the next step's candidates are loaded before this step's network runs (its
  // data-dependent branch otherwise keeps hipcc from hoisting them: one memory latency per step)
  int l0 = w * lpw;
  bool ok = li < lpw && l0 + li < G;
  float v = ok ? in_d[base + (size_t)(l0 + li) * k + e] : FLT_MAX;
  int id = ok ? in_i[base + (size_t)(l0 + li) * k + e] : -1;
  for (; l0 < G; l0 += MW * lpw) {
    const int ln = l0 + MW * lpw + li;
    const bool okn = li < lpw && ln < G;
    const float vn = okn ? in_d[base + (size_t)ln * k + e] : FLT_MAX;
    const int idn = okn ? in_i[base + (size_t)ln * k + e] : -1;
    wave_offer(bv, bi, v, id, k, lane);
    v = vn;
    id = idn;
  }
  mv[w][lane] = bv;
  mi[w][lane] = bi;
  __syncthreads();
  if (w == 0) {
    for (int gg = 1; gg < MW; ++gg) wave_merge64(bv, bi, mv[gg][lane], mi[gg][lane], lane);
    if (lane < k) {
      out_d[(size_t)qi * k + lane] = bv;
      out_i[(size_t)qi * k + lane] = bi;  // int64 ids: the caller's final type, no widening launch
    }
  }
}

// fill columns [n0, n0+n) of the column-major store from row-major rows x[n][d]
__global__ void l2_append_kernel(float* xt, int cap, int d, int n0, const float* __restrict__ x, int n) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  const int dim = blockIdx.y;
  if (row < n) xt[(size_t)dim * cap + n0 + row] = x[(size_t)row * d + dim];
}

// scatter row-major rows x[j] into column-major store slots pos[j] (IVF list appends)
__global__ void l2_scatter_kernel(float* xt, int cap, int d, const int* __restrict__ pos, const float* __restrict__ x,
                                  int n) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int dim = blockIdx.y;
  if (j < n) xt[(size_t)dim * cap + pos[j]] = x[(size_t)j * d + dim];
}

// gather rows (by index) out of the column-major store -> row-major [n][d]
__global__ void l2_gather_kernel(const float* __restrict__ xt, int cap, int d, const int* __restrict__ idx, int n,
                                 float* out) {
  const int i = blockIdx.x;
  const int row = idx[i];
  for (int t = threadIdx.x; t < d; t += blockDim.x) out[(size_t)i * d + t] = row >= 0 ? xt[(size_t)t * cap + row] : 0.f;
}

// ---------------------------------------------------------------------------------------------
// k-means assignment as an MFMA distance GEMM with a fused argmin (index/ivf.py training, IVF
// list assignment). ||x - c||^2 = ||x||^2 + (||c||^2 - 2 x.c): the x.c products run on the exact
// fp32-input MFMA (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain, 1/16 of the bf16 rate but
// exact like faiss' sgemm path), the argmin over centroids is kept per lane in registers.
// Block = 32 rows of X resident in LDS (pitch d + 4 floats: 16 distinct 16-B slots for the 16 rows
// a ds_read_b128 lane group touches) x every centroid, streamed in [64 centroids][64 dims] chunks.
// Wave w: rows 16*(w >> 1) .. +15 against centroids 32*(w & 1) .. +31 of each 64-centroid tile (two
// 16x16 accumulator tiles). MFMA k-slot mapping: lane l feeds dims 4*(l >> 4) + s of a 16-dim step
// in MFMA s = 0..3, so A and B fragments are single ds_read_b128s.
constexpr int KA_ROWS = 32, KA_CT = 64, KA_DC = 64, KA_DMAX = 1024;

__device__ __forceinline__ void ka_better(float v, int i, float& bv, int& bi) {
  if (v < bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

// DUMP: also write every (row, centroid) score -(||c||^2 - 2 x.c) to scores[row][k] -- the IVF
// coarse search takes its top-nprobe from these (topk_lds, ties -> lower id), so probing and list
// assignment rank centroids by the SAME numbers (a vector is always found by a query at its own
// position with nprobe = 1).
template <bool DUMP>
__global__ __launch_bounds__(256) void kmeans_assign_kernel(const float* __restrict__ X, int n, int d,
                                                            const float* __restrict__ C,
                                                            const float* __restrict__ cnorm, int k,
                                                            int* __restrict__ assign, float* __restrict__ dist,
                                                            float* __restrict__ scores) {
  extern __shared__ __attribute__((aligned(16))) float ka_smem[];
  const int xp = d + 4;
  float* xs = ka_smem;                          // [KA_ROWS][xp]
  float* cs = ka_smem + KA_ROWS * xp;           // [KA_CT][KA_DC + 4]
  __shared__ float s_bv[2][KA_ROWS];
  __shared__ int s_bi[2][KA_ROWS];
  __shared__ float s_xn[KA_ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row0 = blockIdx.x * KA_ROWS;
  // X tile -> LDS (rows past n are zero)
  const int d4 = d / 4;
  for (int e = tid; e < KA_ROWS * d4; e += 256) {
    const int r = e / d4, c4 = e % d4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row0 + r < n) v = *reinterpret_cast<const f32x4*>(X + (size_t)(row0 + r) * d + 4 * c4);
    *reinterpret_cast<f32x4*>(xs + r * xp + 4 * c4) = v;
  }
  __syncthreads();
  if (tid < KA_ROWS) {
    float sq = 0.f;
    for (int t = 0; t < d; ++t) sq = fmaf(xs[tid * xp + t], xs[tid * xp + t], sq);
    s_xn[tid] = sq;
  }
  const int rg = wid >> 1, ch = wid & 1;  // row group, centroid half
  const int fr = lane & 15, fg = lane >> 4;
  const float* xrow = xs + (16 * rg + fr) * xp + 4 * fg;
  float bv[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
  int bi[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
  for (int c0 = 0; c0 < k; c0 += KA_CT) {
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int d0 = 0; d0 < d; d0 += KA_DC) {
      __syncthreads();  // previous chunk fully consumed
      for (int e = tid; e < KA_CT * (KA_DC / 4); e += 256) {
        const int r = e / (KA_DC / 4), c4 = e % (KA_DC / 4);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (c0 + r < k) v = *reinterpret_cast<const f32x4*>(C + (size_t)(c0 + r) * d + d0 + 4 * c4);
        *reinterpret_cast<f32x4*>(cs + r * (KA_DC + 4) + 4 * c4) = v;
      }
      __syncthreads();
      const float* c0row = cs + (32 * ch + fr) * (KA_DC + 4) + 4 * fg;
      const float* c1row = c0row + 16 * (KA_DC + 4);
#pragma unroll
      for (int kk = 0; kk < KA_DC; kk += 16) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(xrow + d0 + kk);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(c0row + kk);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(c1row + kk);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b0[s], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b1[s], acc1, 0, 0, 0);
        }
      }
    }
    // lane holds rows 4*fg + r (of this wave's 16), centroids c0 + 32*ch + fr (acc0) / + 16 (acc1)
    const int ca = c0 + 32 * ch + fr, cb = ca + 16;
    const float na = ca < k ? cnorm[ca] : 0.f, nb = cb < k ? cnorm[cb] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float va = na - 2.f * acc0[r], vb = nb - 2.f * acc1[r];
      if (ca < k) ka_better(va, ca, bv[r], bi[r]);
      if (cb < k) ka_better(vb, cb, bv[r], bi[r]);
      if (DUMP) {
        const int row = row0 + 16 * rg + 4 * fg + r;
        if (row < n) {
          if (ca < k) scores[(size_t)row * k + ca] = -va;
          if (cb < k) scores[(size_t)row * k + cb] = -vb;
        }
      }
    }
  }
  // argmin across the 16 lanes of a row group (same fg), then across the two centroid halves
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float ov = __shfl_xor(bv[r], o, 64);
      const int oi = __shfl_xor(bi[r], o, 64);
      ka_better(ov, oi, bv[r], bi[r]);
    }
  }
  if (fr == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s_bv[ch][16 * rg + 4 * fg + r] = bv[r];
      s_bi[ch][16 * rg + 4 * fg + r] = bi[r];
    }
  }
  __syncthreads();
  if (tid < KA_ROWS && row0 + tid < n) {
    float v = s_bv[0][tid];
    int i = s_bi[0][tid];
    ka_better(s_bv[1][tid], s_bi[1][tid], v, i);
    if (assign) assign[row0 + tid] = i;
    if (dist) dist[row0 + tid] = fmaxf(s_xn[tid] + v, 0.f);
  }
}

}  // namespace

// dims split over S waves per row tile: more blocks for small indexes (the summation order,
// and so the last bits of a distance, depend on S -- i.e. on the index size only)
static int scan_slices(int n) { return n < 65536 ? 4 : (n < 262144 ? 2 : 1); }

template <int QB, int S>
static void launch_scan(dim3 grid, size_t lds, hipStream_t st, const float* xt, int cap, int d, int rb, int re,
                        int ntiles, const float* q, int nq, int k, float* od, int* oi, const int* ids) {
  hipLaunchKernelGGL((l2_scan_kernel<QB, S>), grid, dim3(ST), lds, st, xt, cap, d, rb, re, ntiles, q, nq, k, od, oi,
                     ids);
}

template <int QB>
static void launch_scan_s(int S, dim3 grid, hipStream_t st, const float* xt, int cap, int d, int rb, int re,
                          int ntiles, const float* q, int nq, int k, float* od, int* oi, const int* ids) {
  const size_t lds = (size_t)QB * DCH * 4 + (size_t)(S - 1) * (4 / S) * QB * 64 * 4;
  if (S == 4) launch_scan<QB, 4>(grid, lds, st, xt, cap, d, rb, re, ntiles, q, nq, k, od, oi, ids);
  else if (S == 2) launch_scan<QB, 2>(grid, lds, st, xt, cap, d, rb, re, ntiles, q, nq, k, od, oi, ids);
  else launch_scan<QB, 1>(grid, lds, st, xt, cap, d, rb, re, ntiles, q, nq, k, od, oi, ids);
}

// the MFMA path (batched queries, k <= 8, d % 32 == 0) for nq >= this
static int g_mfma_min_nq = 16;
RAGK_API int ragk_l2_search_set_mfma_min_nq(int n) {
  g_mfma_min_nq = n > 0 ? n : 16;
  return 0;
}
static bool use_mfma(int nq, int k, int d) {
  return nq >= g_mfma_min_nq && k <= MQ_MK && d % (4 * MQ_KU) == 0 && d <= MQ_DMAX;
}
static size_t mfma_lds(int d, int QT) { return ((size_t)mq_region0(d, QT) + 16 * QT + 4 * 64) * 4; }
static int mfma_rt(int n) { return n < 262144 ? 1 : 4; }  // 16 or 64 rows per wave and tile

// Number of partial lists per query the scan of rows [row_begin, row_end) emits (size the
// partial buffers [nq][G][k] with it).
RAGK_API int ragk_l2_scan_groups(int row_begin, int row_end, int nq) {
  const int n = max(0, row_end - row_begin);
  const int S = scan_slices(n);
  const int ntiles = (n + 64 * (4 / S) - 1) / (64 * (4 / S));  // (the MFMA path's 256-row tiles: <= this)
  const int qgroups = (max(nq, 1) + 15) / 16;
  const int target = max(1, 2048 / qgroups);  // bounded list count: the merge stays short
  return max(1, min(ntiles, target));
}

// As ragk_l2_scan_groups, for the kernel ragk_l2_search actually launches for (nq, k, d).
RAGK_API int ragk_l2_search_groups(int row_begin, int row_end, int nq, int k, int d) {
  if (!use_mfma(nq, k, d)) return ragk_l2_scan_groups(row_begin, row_end, nq);
  const int n = max(0, row_end - row_begin);
  const int ntiles = (n + 64 * mfma_rt(n) - 1) / (64 * mfma_rt(n));
  const int qgroups = (nq + 31) / 32;
  return max(1, min(ntiles, max(1, 2048 / qgroups)));
}

// Exact top-k (k <= 64) over rows [row_begin, row_end) of xt[d][cap]; part_d / part_i hold
// nq * ragk_l2_scan_groups(...) * k entries; results -> out_d / out_i [nq][k].
RAGK_API int ragk_l2_search(const float* xt, int cap, int d, int row_begin, int row_end, const float* q, int nq,
                            int k, const int* ids_map, float* part_d, int* part_i, float* out_d,
                            long long* out_i, hipStream_t st) {
  if (nq <= 0) return 0;
  if (k < 1 || k > 64 || d < 1 || cap < 1 || row_end > cap) return (int)hipErrorInvalidValue;
  if (use_mfma(nq, k, d)) {
    static bool attr = false;
    if (!attr) {
      hipError_t e = hipSuccess;
      const void* fns[4] = {(const void*)l2_mfma_kernel<1, 1>, (const void*)l2_mfma_kernel<1, 4>,
                            (const void*)l2_mfma_kernel<2, 1>, (const void*)l2_mfma_kernel<2, 4>};
      for (int i = 0; i < 4 && e == hipSuccess; ++i)
        e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)mfma_lds(MQ_DMAX, 1 + i / 2));
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    const int n = max(0, row_end - row_begin);
    const int RT = mfma_rt(n);
    const int ntiles = (n + 64 * RT - 1) / (64 * RT);
    const int G = ragk_l2_search_groups(row_begin, row_end, nq, k, d);
    const int QT = nq >= 32 ? 2 : 1;
    const dim3 grid(G, (nq + 16 * QT - 1) / (16 * QT));
    const size_t lds = mfma_lds(d, QT);
#define RAGK_MQ(Q, R) hipLaunchKernelGGL((l2_mfma_kernel<Q, R>), grid, dim3(ST), lds, st, xt, cap, d, row_begin, row_end, \
                                         ntiles, q, nq, k, part_d, part_i, ids_map)
    if (QT == 2) {
      if (RT == 4) RAGK_MQ(2, 4); else RAGK_MQ(2, 1);
    } else {
      if (RT == 4) RAGK_MQ(1, 4); else RAGK_MQ(1, 1);
    }
#undef RAGK_MQ
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(topk_lists_merge_kernel, dim3(nq), dim3(MW * 64), 0, st, part_d, part_i, G, k, out_d, out_i);
    return (int)hipGetLastError();
  }
  const int n = max(0, row_end - row_begin);
  const int S = scan_slices(n);
  const int ntiles = (n + 64 * (4 / S) - 1) / (64 * (4 / S));
  const int G = ragk_l2_search_groups(row_begin, row_end, nq, k, d);
  // queries per block: up to 16 (32 accumulators + the x[] ring would leave one wave per SIMD);
  // the last group of the y-dimension may be partial (handled in-kernel)
  const int QB = nq >= 16 ? 16 : (nq >= 8 ? 8 : (nq >= 4 ? 4 : (nq >= 2 ? 2 : 1)));
  const dim3 grid(G, (nq + QB - 1) / QB);
  if (QB == 16) launch_scan_s<16>(S, grid, st, xt, cap, d, row_begin, row_end, ntiles, q, nq, k, part_d, part_i, ids_map);
  else if (QB == 8) launch_scan_s<8>(S, grid, st, xt, cap, d, row_begin, row_end, ntiles, q, nq, k, part_d, part_i, ids_map);
  else if (QB == 4) launch_scan_s<4>(S, grid, st, xt, cap, d, row_begin, row_end, ntiles, q, nq, k, part_d, part_i, ids_map);
  else if (QB == 2) launch_scan_s<2>(S, grid, st, xt, cap, d, row_begin, row_end, ntiles, q, nq, k, part_d, part_i, ids_map);
  else launch_scan_s<1>(S, grid, st, xt, cap, d, row_begin, row_end, ntiles, q, nq, k, part_d, part_i, ids_map);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(topk_lists_merge_kernel, dim3(nq), dim3(MW * 64), 0, st, part_d, part_i, G, k, out_d, out_i);
  return (int)hipGetLastError();
}

// IVF: part buffers hold nq * nprobe * k entries; results -> out [nq][k]
RAGK_API int ragk_ivf_search(const float* xt, int cap, int d, const float* q, int nq, const int* probes, int nprobe,
                             const int* offsets, const int* ends, const int* ids_map, int k, float* part_d,
                             int* part_i, float* out_d, long long* out_i, hipStream_t st) {
  if (nq <= 0) return 0;
  if (d > IVF_DMAX || k < 1 || k > 64 || nprobe < 1 || cap < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ivf_scan_kernel, dim3(nprobe, nq), dim3(ST), 0, st, xt, cap, d, q, probes, nprobe, offsets, ends,
                     ids_map, k, part_d, part_i);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(topk_lists_merge_kernel, dim3(nq), dim3(MW * 64), 0, st, part_d, part_i, nprobe, k, out_d,
                     out_i);
  return (int)hipGetLastError();
}

// k-means / IVF assignment: a[i] = argmin_c ||x_i - c||^2 over the k centroids (ties -> lower c),
// dist[i] = that squared distance. X [n][d], C [k][d] fp32 row-major, cnorm[c] = ||c||^2.
// scores (optional, nullptr = none): [n][k] floats, see kmeans_assign_kernel<true>
RAGK_API int ragk_kmeans_assign(const float* X, int n, int d, const float* C, const float* cnorm, int k, int* assign,
                                float* dist, float* scores, hipStream_t st) {
  if (n <= 0) return 0;
  if (d % KA_DC || d > KA_DMAX || k <= 0 || ((uintptr_t)X & 15) || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)KA_ROWS * (d + 4) * 4 + (size_t)KA_CT * (KA_DC + 4) * 4;
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in (d up to 1024: ~149 KiB)
  if (!attr_set) {
    const int mx = KA_ROWS * (KA_DMAX + 4) * 4 + KA_CT * (KA_DC + 4) * 4;
    hipError_t e = hipFuncSetAttribute((const void*)kmeans_assign_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)kmeans_assign_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  if (scores)
    hipLaunchKernelGGL(kmeans_assign_kernel<true>, dim3((n + KA_ROWS - 1) / KA_ROWS), dim3(256), lds, st, X, n, d, C,
                       cnorm, k, assign, dist, scores);
  else
    hipLaunchKernelGGL(kmeans_assign_kernel<false>, dim3((n + KA_ROWS - 1) / KA_ROWS), dim3(256), lds, st, X, n, d, C,
                       cnorm, k, assign, dist, scores);
  return (int)hipGetLastError();
}

RAGK_API int ragk_l2_append(float* xt, int cap, int d, int n0, const float* x, int n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n0 + n > cap) return (int)hipErrorInvalidValue;
  dim3 grid((n + 255) / 256, d);
  hipLaunchKernelGGL(l2_append_kernel, grid, dim3(256), 0, st, xt, cap, d, n0, x, n);
  return (int)hipGetLastError();
}

// x [n][d] row-major -> store slots pos[j] (every pos < cap; the launcher's caller checks)
RAGK_API int ragk_l2_scatter(float* xt, int cap, int d, const int* pos, const float* x, int n, hipStream_t st) {
  if (n <= 0) return 0;
  dim3 grid((n + 255) / 256, d);
  hipLaunchKernelGGL(l2_scatter_kernel, grid, dim3(256), 0, st, xt, cap, d, pos, x, n);
  return (int)hipGetLastError();
}

RAGK_API int ragk_l2_gather(const float* xt, int cap, int d, const int* idx, int n, float* out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(l2_gather_kernel, dim3(n), dim3(256), 0, st, xt, cap, d, idx, n, out);
  return (int)hipGetLastError();
}
