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
                                                      const int* __restrict__ ends,
                                                      const int* __restrict__ ids_map, int k, float* out_d,
                                                      int* out_i) {
  __shared__ float qs[IVF_DMAX];
  __shared__ float sd[RPB];
  __shared__ int sidx[RPB];
  const int qi = blockIdx.y;
  const int p = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int list = probes[(size_t)qi * nprobe + p];
  // list rows [offsets[list], ends[list]) -- lists may carry spare capacity after their rows
  // (incremental appends); without `ends` the lists are packed: end = offsets[list + 1]
  const int lend = ends ? ends[list] : offsets[list + 1];
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

__global__ __launch_bounds__(256) void kmeans_assign_kernel(const float* __restrict__ X, int n, int d,
                                                            const float* __restrict__ C,
                                                            const float* __restrict__ cnorm, int k,
                                                            int* __restrict__ assign, float* __restrict__ dist) {
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
      if (ca < k) ka_better(na - 2.f * acc0[r], ca, bv[r], bi[r]);
      if (cb < k) ka_better(nb - 2.f * acc1[r], cb, bv[r], bi[r]);
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
    assign[row0 + tid] = i;
    if (dist) dist[row0 + tid] = fmaxf(s_xn[tid] + v, 0.f);
  }
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
                           int chunks, const int* offsets, const int* ends, const int* ids_map, int k, float* out_d,
                           int* out_i, hipStream_t st) {
  if (nq <= 0) return 0;
  if (d > IVF_DMAX || k > RPB || chunks < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ivf_scan_kernel, dim3(nprobe * chunks, nq), dim3(ST), 0, st, xt, cap, d, q, probes, nprobe,
                     chunks, offsets, ends, ids_map, k, out_d, out_i);
  return (int)hipGetLastError();
}

// k-means / IVF assignment: a[i] = argmin_c ||x_i - c||^2 over the k centroids (ties -> lower c),
// dist[i] = that squared distance. X [n][d], C [k][d] fp32 row-major, cnorm[c] = ||c||^2.
RAGK_API int ragk_kmeans_assign(const float* X, int n, int d, const float* C, const float* cnorm, int k, int* assign,
                                float* dist, hipStream_t st) {
  if (n <= 0) return 0;
  if (d % KA_DC || d > KA_DMAX || k <= 0 || ((uintptr_t)X & 15) || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)KA_ROWS * (d + 4) * 4 + (size_t)KA_CT * (KA_DC + 4) * 4;
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in (d up to 1024: ~149 KiB)
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kmeans_assign_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       KA_ROWS * (KA_DMAX + 4) * 4 + KA_CT * (KA_DC + 4) * 4);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kmeans_assign_kernel, dim3((n + KA_ROWS - 1) / KA_ROWS), dim3(256), lds, st, X, n, d, C, cnorm, k,
                     assign, dist);
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
