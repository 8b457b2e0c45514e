// Exact squared-L2 k-nearest-neighbour search for gfx950 (faiss IndexFlatL2
// semantics: squared distances, ascending, missing results = (-1, FLT_MAX)).
// Reference: faiss index.search at /root/reference/llm/rag.py:116.
//
// The database stays resident in HBM in a COLUMN-major layout xt[d][cap]
// (cap = row capacity), so a block's 256 threads read 256 consecutive rows of one
// dimension per load: fully coalesced, no LDS for the data. Queries are staged in
// LDS and broadcast. Distances are computed directly as sum((x - q)^2) in fp32
// (faiss' exact path for small query batches), then:
//   1. l2_block_topk: per (row block, query group) -> top-k per query (bitonic in LDS)
//   2. topk_merge:    repeatedly merges 64 partial lists per query until one remains.
// IVF-Flat scans reuse the same kernels over an inverted-list ordered layout
// (list rows are contiguous) with per-(query, probe) row ranges.
#include "common.h"
#include <float.h>
using namespace ragk;

namespace {

constexpr int ST = 256;      // threads
constexpr int RPT = 4;       // rows per thread
constexpr int RPB = ST * RPT;  // rows per block (1024)
constexpr int QC = 8;        // queries per block
constexpr int DCH = 256;     // query dims staged per LDS chunk

// sort `n` (power of 2) pairs ascending by (dist, idx) in LDS
__device__ void bitonic_asc(float* v, int* ix, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const float a = v[i], b = v[p];
          const int ia = ix[i], ib = ix[p];
          const bool a_first = (a < b) || (a == b && (unsigned)ia < (unsigned)ib);
          if (a_first != up) { v[i] = b; v[p] = a; ix[i] = ib; ix[p] = ia; }
        }
      }
      __syncthreads();
    }
  }
}

// xt: [d][cap] fp32 column-major database; rows [row_begin, row_end) are searched.
// For IVF each blockIdx.z selects a (query, probe) row range via `ranges` (nullptr = flat).
__global__ __launch_bounds__(ST) void l2_block_topk_kernel(const float* __restrict__ xt, int cap, int d,
                                                           int row_begin, int row_end, const float* __restrict__ q,
                                                           int nq, int k, float* out_d, int* out_i,
                                                           const int* __restrict__ ids_map) {
  __shared__ float qs[QC][DCH];
  __shared__ float sd[RPB];
  __shared__ int sidx[RPB];
  const int q0 = blockIdx.y * QC;
  const int r0 = row_begin + blockIdx.x * RPB;
  float acc[RPT][QC];
#pragma unroll
  for (int r = 0; r < RPT; ++r)
#pragma unroll
    for (int j = 0; j < QC; ++j) acc[r][j] = 0.f;

  for (int dc = 0; dc < d; dc += DCH) {
    const int dn = min(DCH, d - dc);
    __syncthreads();
    for (int e = threadIdx.x; e < QC * DCH; e += ST) {
      const int j = e / DCH, t = e % DCH;
      qs[j][t] = (q0 + j < nq && t < dn) ? q[(size_t)(q0 + j) * d + dc + t] : 0.f;
    }
    __syncthreads();
    for (int t = 0; t < dn; ++t) {
      const float* col = xt + (size_t)(dc + t) * cap;
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int row = r0 + r * ST + threadIdx.x;
        const float x = row < row_end ? col[row] : 0.f;
#pragma unroll
        for (int j = 0; j < QC; ++j) {
          const float df = x - qs[j][t];
          acc[r][j] = fmaf(df, df, acc[r][j]);
        }
      }
    }
  }
  const int nblk_out = gridDim.x;
  for (int j = 0; j < QC && q0 + j < nq; ++j) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int slot = r * ST + threadIdx.x;
      const int row = r0 + slot;
      const bool ok = row < row_end;
      sd[slot] = ok ? acc[r][j] : FLT_MAX;
      sidx[slot] = ok ? (ids_map ? ids_map[row] : row) : -1;
    }
    __syncthreads();
    bitonic_asc(sd, sidx, RPB);
    for (int i = threadIdx.x; i < k; i += ST) {
      const size_t o = ((size_t)(q0 + j) * nblk_out + blockIdx.x) * k + i;
      out_d[o] = sd[i];
      out_i[o] = sidx[i];
    }
  }
}

// IVF-Flat scan: block (probe p, chunk c) x query q scans rows [start, end) of list
// probes[q][p] in the list-ordered column-major store -> partial top-k at [q][p*chunks+c].
constexpr int IVF_DMAX = 2048;
__global__ __launch_bounds__(ST) void ivf_scan_kernel(const float* __restrict__ xt, int cap, int d,
                                                      const float* __restrict__ q, const int* __restrict__ probes,
                                                      int nprobe, int chunks, const int* __restrict__ offsets,
                                                      const int* __restrict__ ids_map, int k, float* out_d,
                                                      int* out_i) {
  __shared__ float qs[IVF_DMAX];
  __shared__ float sd[RPB];
  __shared__ int sidx[RPB];
  const int qi = blockIdx.y;
  const int p = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int list = probes[(size_t)qi * nprobe + p];
  const int lend = offsets[list + 1];
  const int r0 = offsets[list] + c * RPB;
  const int r1 = min(lend, r0 + RPB);
  for (int t = threadIdx.x; t < d; t += ST) qs[t] = q[(size_t)qi * d + t];
  __syncthreads();
  float acc[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) acc[r] = 0.f;
  if (r0 < r1) {
    for (int t = 0; t < d; ++t) {
      const float* col = xt + (size_t)t * cap;
      const float qv = qs[t];
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int row = r0 + r * ST + threadIdx.x;
        const float x = row < r1 ? col[row] : 0.f;
        const float df = x - qv;
        acc[r] = fmaf(df, df, acc[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int slot = r * ST + threadIdx.x;
    const int row = r0 + slot;
    const bool ok = row < r1;
    sd[slot] = ok ? acc[r] : FLT_MAX;
    sidx[slot] = ok ? ids_map[row] : -1;
  }
  __syncthreads();
  bitonic_asc(sd, sidx, RPB);
  const int G = gridDim.x;
  for (int i = threadIdx.x; i < k; i += ST) {
    const size_t o = ((size_t)qi * G + blockIdx.x) * k + i;
    out_d[o] = sd[i];
    out_i[o] = sidx[i];
  }
}

// in: [nq][G][k] -> out: [nq][ceil(G/64)][k]
constexpr int MG = 64;
__global__ __launch_bounds__(ST) void topk_merge_kernel(const float* __restrict__ in_d, const int* __restrict__ in_i,
                                                        int G, int k, int n_pow2, float* out_d, int* out_i) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sd = reinterpret_cast<float*>(smem);
  int* si = reinterpret_cast<int*>(smem + n_pow2 * sizeof(float));
  const int qi = blockIdx.y, g0 = blockIdx.x * MG;
  const int ng = min(MG, G - g0);
  const int n = ng * k;
  for (int e = threadIdx.x; e < n_pow2; e += ST) {
    if (e < n) {
      const size_t o = ((size_t)qi * G + g0) * k + e;
      sd[e] = in_d[o];
      si[e] = in_i[o];
    } else {
      sd[e] = FLT_MAX;
      si[e] = -1;
    }
  }
  __syncthreads();
  bitonic_asc(sd, si, n_pow2);
  const int Gout = gridDim.x;
  for (int i = threadIdx.x; i < k; i += ST) {
    const size_t o = ((size_t)qi * Gout + blockIdx.x) * k + i;
    out_d[o] = sd[i];
    out_i[o] = si[i];
  }
}

// fill columns [n0, n0+n) of the column-major store from row-major rows x[n][d]
__global__ void l2_append_kernel(float* xt, int cap, int d, int n0, const float* __restrict__ x, int n) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  const int dim = blockIdx.y;
  if (row < n) xt[(size_t)dim * cap + n0 + row] = x[(size_t)row * d + dim];
}

// gather rows (by index) out of the column-major store -> row-major [n][d]
__global__ void l2_gather_kernel(const float* __restrict__ xt, int cap, int d, const int* __restrict__ idx, int n,
                                 float* out) {
  const int i = blockIdx.x;
  const int row = idx[i];
  for (int t = threadIdx.x; t < d; t += blockDim.x) out[(size_t)i * d + t] = row >= 0 ? xt[(size_t)t * cap + row] : 0.f;
}

}  // namespace

// Partial pass. out buffers must hold nq * ceil((row_end-row_begin)/1024) * k entries.
// Returns the number of row blocks G through *out_groups.
RAGK_API int ragk_l2_partial(const float* xt, int cap, int d, int row_begin, int row_end, const float* q, int nq,
                             int k, float* out_d, int* out_i, const int* ids_map, int* out_groups, hipStream_t st) {
  const int n = row_end - row_begin;
  if (nq <= 0 || k <= 0) return 0;
  if (k > RPB) return (int)hipErrorInvalidValue;
  const int G = n > 0 ? (n + RPB - 1) / RPB : 1;
  if (out_groups) *out_groups = G;
  dim3 grid(G, (nq + QC - 1) / QC);
  hipLaunchKernelGGL(l2_block_topk_kernel, grid, dim3(ST), 0, st, xt, cap, d, row_begin, n > 0 ? row_end : row_begin,
                     q, nq, k, out_d, out_i, ids_map);
  return (int)hipGetLastError();
}

// out buffers: nq * nprobe * chunks * k entries; chunks = ceil(max_list_len / 1024)
RAGK_API int ragk_ivf_scan(const float* xt, int cap, int d, const float* q, int nq, const int* probes, int nprobe,
                           int chunks, const int* offsets, const int* ids_map, int k, float* out_d, int* out_i,
                           hipStream_t st) {
  if (nq <= 0) return 0;
  if (d > IVF_DMAX || k > RPB || chunks < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ivf_scan_kernel, dim3(nprobe * chunks, nq), dim3(ST), 0, st, xt, cap, d, q, probes, nprobe,
                     chunks, offsets, ids_map, k, out_d, out_i);
  return (int)hipGetLastError();
}

RAGK_API int ragk_topk_merge(const float* in_d, const int* in_i, int nq, int G, int k, float* out_d, int* out_i,
                             hipStream_t st) {
  if (nq <= 0) return 0;
  if (k > 64) return (int)hipErrorInvalidValue;
  int n_pow2 = 1;
  while (n_pow2 < MG * k) n_pow2 <<= 1;
  const int gout = (G + MG - 1) / MG;
  hipLaunchKernelGGL(topk_merge_kernel, dim3(gout, nq), dim3(ST), n_pow2 * 8, st, in_d, in_i, G, k, n_pow2, out_d,
                     out_i);
  return (int)hipGetLastError();
}

RAGK_API int ragk_l2_append(float* xt, int cap, int d, int n0, const float* x, int n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n0 + n > cap) return (int)hipErrorInvalidValue;
  dim3 grid((n + 255) / 256, d);
  hipLaunchKernelGGL(l2_append_kernel, grid, dim3(256), 0, st, xt, cap, d, n0, x, n);
  return (int)hipGetLastError();
}

RAGK_API int ragk_l2_gather(const float* xt, int cap, int d, const int* idx, int n, float* out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(l2_gather_kernel, dim3(n), dim3(256), 0, st, xt, cap, d, idx, n, out);
  return (int)hipGetLastError();
}
