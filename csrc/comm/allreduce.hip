// Single-node all-reduce over xGMI peer mappings (gfx950 / MI355X).
//
// The reference has no collectives at all; this is the latency path for
// tensor-parallel decode, where each layer all-reduces a [B, 4096] bf16 residual
// (8 KB x B). RCCL's ring is per-link bound on the point-to-point xGMI mesh (7 links per
// GPU) and pays launch + protocol latency per call; here every rank maps every peer's
// staging buffer once (hipIpc handles exchanged over the gloo control group) and one
// kernel does the whole collective with direct xGMI loads:
//
//   one-shot  (small messages): every rank copies its input into its staging buffer,
//             signals all peers, waits for all peers, then reads ALL ranks' copies of its
//             output slice and sums them in rank order (bit-identical on every rank).
//   two-shot  (medium messages): reduce-scatter (rank r reduces sub-slice r from all
//             peers into its result buffer) -> signal -> all-gather (read every peer's
//             reduced sub-slice).  Each byte crosses xGMI ~2x instead of world x.
//
// Synchronisation is per workgroup: block b of every rank owns the same element range, so
// block b only waits for block b of its peers (no grid-wide barrier). Flags are
// monotonically increasing epochs kept on the device (graph-capturable: no host-side
// counter). Staging/result buffers are double-buffered by epoch parity. The grid size is
// fixed per communicator, so every block takes part in every call and all blocks share
// the epoch = call index: when block b passes the start barrier of call e, every peer has
// finished call e-1 (stream order), so no peer still reads the half of call e-2 that the
// next call overwrites, whatever element range any block owns.
//
// Fused row-parallel reduction for tensor-parallel decode (ar_add_rmsnorm): the consumer of the
// split-K o_proj / down GEMMs does the cross-rank reduction itself. Block `row` of every rank sums
// its fp32 partial slabs of that row, publishes the row in its staging area, waits for block `row`
// of every peer, then (one-shot) sums all ranks' rows in rank order, or (two-shot) reduces its
// 1/world column slice in rank order, publishes it as bf16, waits again and gathers the row -- and
// finishes with the residual add + RMSNorm. Same value on every rank, bit for bit; no standalone
// all-reduce launch per layer. The row barriers have their own flags / epochs (one per row slot),
// so a call with M rows advances exactly the epochs of rows 0..M-1, identically on every rank.
//
// The whole region is allocated uncached (hipDeviceMallocUncached): payload stores and
// peer loads bypass the per-XCD L2s; flag stores/polls are system-scope atomics and the
// reader issues a system-scope acquire after its poll. Every spin is bounded (wall-clock, via
// s_memrealtime): a peer that never arrives sets an error word -- on the device (ragk_ar_error) and
// in pinned host memory (polled by the engine after each step) -- and the block reads no peer data.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../kernels/common.h"
using namespace ragk;

namespace {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 80;
constexpr int AR_THREADS = 512;
// Default bound of one peer wait: 5 s of s_memrealtime (constant 100 MHz clock), then give up.
// Ranks step in lockstep, so a healthy wait is microseconds; the bound only has to cover host-side
// skew between ranks (a Python pause) and must stay far below the engine watchdog.
constexpr unsigned AR_TIMEOUT_TICKS = 500000000u;

struct ArFlags {
  unsigned start[AR_MAX_BLOCKS][AR_MAX_RANKS];  // written by peers: "rank p reached epoch e (phase 1)"
  unsigned mid[AR_MAX_BLOCKS][AR_MAX_RANKS];    // two-shot phase 2
  unsigned epoch[AR_MAX_BLOCKS];                // local per-block epoch counter
  unsigned error;                               // set when a bounded spin gives up
};

constexpr size_t FLAG_BYTES = (sizeof(ArFlags) + 4095) & ~size_t(4095);

constexpr int AR_MAX_ROWS = 256;
struct ArRowFlags {
  unsigned start[AR_MAX_ROWS][AR_MAX_RANKS];
  unsigned mid[AR_MAX_ROWS][AR_MAX_RANKS];
  unsigned epoch[AR_MAX_ROWS];
};
constexpr size_t ROW_FLAG_BYTES = (sizeof(ArRowFlags) + 4095) & ~size_t(4095);

struct ArPeers {
  char* base[AR_MAX_RANKS];  // every rank's region (own one included), mapped in this process
  int fences;                // 1: system-scope release/acquire fences around every flag (A/B, RAGK_AR_FENCES=1)
  size_t rows_off;           // fused row area: [ArRowFlags | fp32 stage x2 | bf16 result x2] (0 = none)
  size_t row_stage_bytes;    // one fp32 staging half: max_rows * max_h * 4
  size_t row_result_bytes;   // one bf16 result half: max_rows * max_h * 2
  unsigned* host_err;        // host-mapped pinned word: the engine polls it after every step, no sync
  unsigned long long spin_limit;  // bound of one peer wait, in s_memrealtime ticks (100 MHz; 64-bit: > 43 s)
};

// Which wait gave up: the error record names the collective (call site), the peer that never arrived,
// the block / row slot and the low bits of the epoch (the call index of that slot), so a timeout says
// WHICH collective of WHICH step stalled on WHICH peer (tests/test_tp_gpu.py, parallel/comm.py).
enum ArSite : unsigned { AR_SITE_AR_START = 1, AR_SITE_AR_MID = 2, AR_SITE_GATHER = 3, AR_SITE_ROW_START = 4,
                         AR_SITE_ROW_MID = 5 };
// record = 1 | site << 1 (3 bits) | peer << 4 (3 bits) | slot << 7 (8 bits) | (epoch & 0xffff) << 15 (bit 31 clear)
__device__ __forceinline__ unsigned ar_record(unsigned site, int peer, int slot, unsigned ep) {
  return 1u | (site & 7u) << 1 | ((unsigned)peer & 7u) << 4 | ((unsigned)slot & 255u) << 7 | (ep & 0xffffu) << 15;
}

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block-level barrier with the same block of every peer: release my writes, publish `ep` into
// slot [b][rank] of every peer's `which` array, wait until all peers published `ep` into mine.
// Returns false (block-uniform) if a peer did not arrive within the bounded spin: the caller then
// reads no peer data (the result is garbage either way and the host raises CommError).
__device__ bool peer_barrier(const ArPeers& P, int rank, int world, int which, unsigned ep, unsigned site) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = 1;
  __syncthreads();
  const int b = blockIdx.x;
  if (threadIdx.x < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: payload visible before the flag
    ArFlags* pf = reinterpret_cast<ArFlags*>(P.base[threadIdx.x]);
    st_sys(which ? &pf->mid[b][rank] : &pf->start[b][rank], ep);
    ArFlags* mf = reinterpret_cast<ArFlags*>(P.base[rank]);
    const unsigned* slot = which ? &mf->mid[b][threadIdx.x] : &mf->start[b][threadIdx.x];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_sys(slot) < ep) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > P.spin_limit) {  // a peer never arrived: report, never hang
        const unsigned rec = ar_record(site, threadIdx.x, b, ep);
        st_sys(&mf->error, rec);
        if (P.host_err) st_sys(P.host_err, rec);
        s_ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return s_ok != 0;
}

__device__ __forceinline__ u32x4 ld16(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// n8 = elements / 8 (16-byte vectors). data_bytes = capacity of one staging half.
template <bool TWO_SHOT>
__global__ __launch_bounds__(AR_THREADS) void allreduce_kernel(ArPeers P, int rank, int world, const bf16_t* in,
                                                               bf16_t* out, long n8, size_t data_bytes) {
  const int b = blockIdx.x;
  ArFlags* mine = reinterpret_cast<ArFlags*>(P.base[rank]);
  __shared__ unsigned s_ep;
  if (threadIdx.x == 0) s_ep = mine->epoch[b] + 1;
  __syncthreads();
  const unsigned ep = s_ep;
  // staging half h (input copies), result half h (two-shot reduced slices)
  const size_t stage_off = FLAG_BYTES + (size_t)(ep & 1) * data_bytes;
  const size_t result_off = FLAG_BYTES + 2 * data_bytes + (size_t)(ep & 1) * data_bytes;
  const long per = (n8 + gridDim.x - 1) / gridDim.x;
  const long v0 = min((long)b * per, n8), v1 = min(v0 + per, n8);

  // 1. copy my slice of the input into my staging buffer
  u32x4* my_stage = reinterpret_cast<u32x4*>(P.base[rank] + stage_off);
  const u32x4* in4 = reinterpret_cast<const u32x4*>(in);
  for (long v = v0 + threadIdx.x; v < v1; v += AR_THREADS) my_stage[v] = in4[v];
  const bool ok = peer_barrier(P, rank, world, 0, ep, AR_SITE_AR_START);

  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  if (!ok) {
    // no peer reads after a failed wait
  } else if (!TWO_SHOT) {
    for (long v = v0 + threadIdx.x; v < v1; v += AR_THREADS) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < world; ++p) {
        float f[8];
        unpack8(ld16(P.base[p] + stage_off + v * 16), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += f[i];
      }
      out4[v] = pack8(acc);
    }
  } else {
    // sub-slice r of this block's range is reduced by rank r
    const long sub = (v1 - v0 + world - 1) / world;
    const long s0 = min(v0 + rank * sub, v1), s1 = min(s0 + sub, v1);
    u32x4* my_res = reinterpret_cast<u32x4*>(P.base[rank] + result_off);
    for (long v = s0 + threadIdx.x; v < s1; v += AR_THREADS) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < world; ++p) {
        float f[8];
        unpack8(ld16(P.base[p] + stage_off + v * 16), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += f[i];
      }
      my_res[v] = pack8(acc);
    }
    if (peer_barrier(P, rank, world, 1, ep, AR_SITE_AR_MID))
    for (int p = 0; p < world; ++p) {
      const long t0 = min(v0 + p * sub, v1), t1 = min(t0 + sub, v1);
      for (long v = t0 + threadIdx.x; v < t1; v += AR_THREADS) out4[v] = ld16(P.base[p] + result_off + v * 16);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) mine->epoch[b] = ep;
}

// Barrier of block `row` with block `row` of every peer over the fused-row flags.
// One shared flag per barrier of a kernel (`which`): the two-shot kernel calls this twice, and a wave
// still reading the first barrier's result must never see the second call's reset.
__device__ bool row_barrier(const ArPeers& P, int rank, int world, int which, int row, unsigned ep) {
  __shared__ int s_oks[2];
  int& s_ok = s_oks[which & 1];
  if (threadIdx.x == 0) s_ok = 1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its payload stores are complete
  __syncthreads();
  // The whole region is uncached (hipDeviceMallocUncached): payload stores are write-through and no
  // cache level holds a copy of a peer's bytes. With every peer on THIS device that is enough: every
  // storing wave drains its stores (vmcnt(0)) before the barrier above, then one lane per peer stores
  // the flag (system-scope atomic). Peers on other GPUs read over xGMI, where that ordering is not
  // established by one memory controller, so the host turns the system-scope release / acquire fences
  // on whenever any peer region lives on another device (ragk_ar_set_fences; parallel/ipc_allreduce.py
  // decides from the ranks' device ids). Measured cost on one GPU: +0.6 % of a TP=8-shard decode step.
  if (threadIdx.x < world) {
    if (P.fences) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    ArRowFlags* pf = reinterpret_cast<ArRowFlags*>(P.base[threadIdx.x] + P.rows_off);
    st_sys(which ? &pf->mid[row][rank] : &pf->start[row][rank], ep);
    ArRowFlags* mf = reinterpret_cast<ArRowFlags*>(P.base[rank] + P.rows_off);
    const unsigned* slot = which ? &mf->mid[row][threadIdx.x] : &mf->start[row][threadIdx.x];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_sys(slot) < ep) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > P.spin_limit) {
        ArFlags* ef = reinterpret_cast<ArFlags*>(P.base[rank]);
        const unsigned rec = ar_record(which ? AR_SITE_ROW_MID : AR_SITE_ROW_START, threadIdx.x, row, ep);
        st_sys(&ef->error, rec);
        if (P.host_err) st_sys(P.host_err, rec);
        s_ok = 0;
        break;
      }
    }
    if (P.fences) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: no load moves above the poll
  }
  __syncthreads();
  return s_ok != 0;
}

__device__ __forceinline__ void ld8f(const char* p, float* f) {
  const u32x4 a = ld16(p), b = ld16(p + 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = __uint_as_float(a[i]);
    f[4 + i] = __uint_as_float(b[i]);
  }
}

constexpr int FR_THREADS = 512;
constexpr int FR_MAXV = 2;  // 2 x 8 x 512 = 8192 columns in registers

// h[row] = bf16(h[row] + bf16(sum over ranks of sum_s P[s][row])); out[row] = rmsnorm(h[row]) * w
// (add_partials_rmsnorm_kernel's math with the cross-rank sum inside). grid = M rows.
template <bool TWO_SHOT>
__global__ __launch_bounds__(FR_THREADS) void ar_add_rmsnorm_kernel(ArPeers P, int rank, int world,
                                                                    const float* __restrict__ Pp, int S, int M,
                                                                    bf16_t* h, int ldh, const bf16_t* __restrict__ w,
                                                                    bf16_t* out, int ldo, int H, float eps) {
  __shared__ float red[FR_THREADS / 64];
  const int row = blockIdx.x;
  ArRowFlags* mine = reinterpret_cast<ArRowFlags*>(P.base[rank] + P.rows_off);
  const int nvec = H >> 3;
  // 0. every load that does not wait on a peer is issued together, one memory round trip instead of
  // four serial ones (at batch 1 this kernel is a single block: its latency is the sum of its round
  // trips): this row's epoch (uncached flag region; every wave reads the same word), this rank's
  // split-K slabs, the residual row and the norm weights.
  const unsigned ep_ld = mine->epoch[row];
  const size_t slab = (size_t)M * H;
  f32x4 pv[FR_MAXV][PSU][2];
  u32x4 hv[FR_MAXV], gv[FR_MAXV];
#pragma unroll
  for (int i = 0; i < FR_MAXV; ++i) {
    const int vi = min((int)threadIdx.x + i * FR_THREADS, nvec - 1);
    if (i * FR_THREADS < nvec) {  // block-uniform
      load_slabs8(Pp + (size_t)row * H + vi * 8, S, slab, pv[i]);
      hv[i] = *reinterpret_cast<const u32x4*>(h + (size_t)row * ldh + vi * 8);
      gv[i] = *reinterpret_cast<const u32x4*>(w + vi * 8);
    }
  }
  float a[FR_MAXV][8];
#pragma unroll
  for (int i = 0; i < FR_MAXV; ++i) {
    const int vi = min((int)threadIdx.x + i * FR_THREADS, nvec - 1);
    if (i * FR_THREADS < nvec) add_slabs8(pv[i], Pp + (size_t)row * H + vi * 8, S, slab, a[i]);
  }
  const unsigned ep = __builtin_amdgcn_readfirstlane(ep_ld) + 1;
  const size_t stage_off = P.rows_off + ROW_FLAG_BYTES + (size_t)(ep & 1) * P.row_stage_bytes + (size_t)row * H * 4;
  const size_t res_off = P.rows_off + ROW_FLAG_BYTES + 2 * P.row_stage_bytes + (size_t)(ep & 1) * P.row_result_bytes +
                         (size_t)row * H * 2;
  // 1. this rank's partial row (its split-K slabs summed) -> staging
#pragma unroll
  for (int i = 0; i < FR_MAXV; ++i) {
    const int vi = threadIdx.x + i * FR_THREADS;
    if (vi < nvec) {
      f32x4* dst = reinterpret_cast<f32x4*>(P.base[rank] + stage_off + (size_t)vi * 32);
      dst[0] = f32x4{a[i][0], a[i][1], a[i][2], a[i][3]};
      dst[1] = f32x4{a[i][4], a[i][5], a[i][6], a[i][7]};
    }
  }
  bool ok = row_barrier(P, rank, world, 0, row, ep);
  float v[FR_MAXV][8];
  float ss = 0.f;
  if (!TWO_SHOT) {
#pragma unroll
    for (int i = 0; i < FR_MAXV; ++i) {
      const int vi = threadIdx.x + i * FR_THREADS;
      if (vi < nvec) {
        float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ok) {
          for (int p = 0; p < world; ++p) {  // rank order: identical on every rank
            float f[8];
            ld8f(P.base[p] + stage_off + (size_t)vi * 32, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += f[e];
          }
        }
        unpack8(hv[i], v[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = bf2f(f2bf(v[i][e] + bf2f(f2bf(t[e]))));
      }
    }
  } else {
    // 2a. reduce my column slice of the row over all ranks (rank order), publish it as bf16
    const int per = (nvec + world - 1) / world;
    const int s0 = min(rank * per, nvec), s1 = min(s0 + per, nvec);
    for (int vi = s0 + threadIdx.x; vi < s1; vi += FR_THREADS) {
      float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) {
        for (int p = 0; p < world; ++p) {
          float f[8];
          ld8f(P.base[p] + stage_off + (size_t)vi * 32, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += f[e];
        }
      }
      *reinterpret_cast<u32x4*>(P.base[rank] + res_off + (size_t)vi * 16) = pack8(t);
    }
    ok = row_barrier(P, rank, world, 1, row, ep) && ok;
    // 2b. gather the reduced row (slice owner = vi / per)
#pragma unroll
    for (int i = 0; i < FR_MAXV; ++i) {
      const int vi = threadIdx.x + i * FR_THREADS;
      if (vi < nvec) {
        float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ok) unpack8(ld16(P.base[vi / per] + res_off + (size_t)vi * 16), t);
        unpack8(hv[i], v[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = bf2f(f2bf(v[i][e] + t[e]));  // t already bf16-rounded
      }
    }
  }
  // 3. residual written back, RMSNorm (rmsnorm_kernel's exact order)
#pragma unroll
  for (int i = 0; i < FR_MAXV; ++i) {
    const int vi = threadIdx.x + i * FR_THREADS;
    if (vi < nvec) {
      *reinterpret_cast<u32x4*>(h + (size_t)row * ldh + vi * 8) = pack8(v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < FR_MAXV; ++i) {
    const int vi = threadIdx.x + i * FR_THREADS;
    if (vi < nvec) {
      float wv[8], o[8];
      unpack8(gv[i], wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = wv[e] * bf2f(f2bf(v[i][e] * inv));
      *reinterpret_cast<u32x4*>(out + (size_t)row * ldo + vi * 8) = pack8(o);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) mine->epoch[row] = ep;
}

// All-gather: out[p * n16 + v] = rank p's in[v] (16-byte vectors). Used for the vocab-parallel
// sampler's candidate exchange (a few KB per decode step), so tensor-parallel decode runs with no
// RCCL call at all and stays inside the captured hipGraph. Same epochs / halves as the all-reduce.
__global__ __launch_bounds__(AR_THREADS) void allgather_kernel(ArPeers P, int rank, int world, const u32x4* in,
                                                               u32x4* out, long n16, size_t data_bytes) {
  const int b = blockIdx.x;
  ArFlags* mine = reinterpret_cast<ArFlags*>(P.base[rank]);
  __shared__ unsigned s_ep;
  if (threadIdx.x == 0) s_ep = mine->epoch[b] + 1;
  __syncthreads();
  const unsigned ep = s_ep;
  const size_t stage_off = FLAG_BYTES + (size_t)(ep & 1) * data_bytes;
  const long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long v0 = min((long)b * per, n16), v1 = min(v0 + per, n16);
  u32x4* my_stage = reinterpret_cast<u32x4*>(P.base[rank] + stage_off);
  for (long v = v0 + threadIdx.x; v < v1; v += AR_THREADS) my_stage[v] = in[v];
  if (peer_barrier(P, rank, world, 0, ep, AR_SITE_GATHER))
  for (int p = 0; p < world; ++p)
    for (long v = v0 + threadIdx.x; v < v1; v += AR_THREADS) out[(long)p * n16 + v] = ld16(P.base[p] + stage_off + v * 16);
  __syncthreads();
  if (threadIdx.x == 0) mine->epoch[b] = ep;
}

struct ArHandle {
  int rank, world, blocks;
  int max_rows, max_h;  // fused row area geometry (0 = none)
  size_t data_bytes;  // capacity of one staging half (= max message bytes)
  char* local;
  unsigned* host_err;  // pinned, mapped: host view
  ArPeers peers;
  bool opened[AR_MAX_RANKS];
};

}  // namespace

// Region layout: [flags | stage0 | stage1 | result0 | result1], each stage/result = max_bytes, then
// (max_rows > 0) the fused row area [row flags | fp32 stage x2 | bf16 result x2] of max_rows x max_h.
// `blocks` (1..80) is the fixed grid of every call on this communicator (same on all ranks).
RAGK_API void* ragk_ar_create(int rank, int world, long max_bytes, int blocks, int max_rows, int max_h) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || max_bytes <= 0) return nullptr;
  if (blocks < 1 || blocks > AR_MAX_BLOCKS) return nullptr;
  if (max_rows < 0 || max_rows > AR_MAX_ROWS || max_h < 0 || max_h > 8 * FR_THREADS * FR_MAXV || max_h % 8) return nullptr;
  ArHandle* h = new ArHandle();
  memset(h, 0, sizeof(*h));
  h->rank = rank;
  h->world = world;
  h->blocks = blocks;
  h->max_rows = max_h > 0 ? max_rows : 0;
  h->max_h = max_rows > 0 ? max_h : 0;
  h->data_bytes = ((size_t)max_bytes + 4095) & ~size_t(4095);
  size_t total = FLAG_BYTES + 4 * h->data_bytes;
  if (h->max_rows) {
    h->peers.rows_off = total;
    h->peers.row_stage_bytes = ((size_t)h->max_rows * h->max_h * 4 + 4095) & ~size_t(4095);
    h->peers.row_result_bytes = ((size_t)h->max_rows * h->max_h * 2 + 4095) & ~size_t(4095);
    total += ROW_FLAG_BYTES + 2 * h->peers.row_stage_bytes + 2 * h->peers.row_result_bytes;
  }
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached) != hipSuccess) {
    delete h;
    return nullptr;
  }
  if (hipMemset(p, 0, total) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    delete h;
    return nullptr;
  }
  h->local = (char*)p;
  h->peers.base[rank] = h->local;
  h->peers.spin_limit = AR_TIMEOUT_TICKS;
  {
    const char* f = getenv("RAGK_AR_FENCES");
    h->peers.fences = (f && f[0] == '1') ? 1 : 0;
  }
  void* he = nullptr;
  if (hipHostMalloc(&he, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    h->host_err = (unsigned*)he;
    *h->host_err = 0;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, he, 0) == hipSuccess) h->peers.host_err = (unsigned*)dp;
  }
  return h;
}

RAGK_API int ragk_ar_ipc_handle(void* hp, void* out64) {
  ArHandle* h = (ArHandle*)hp;
  hipIpcMemHandle_t mh;
  hipError_t e = hipIpcGetMemHandle(&mh, h->local);
  if (e != hipSuccess) return (int)e;
  memcpy(out64, &mh, sizeof(mh));
  return 0;
}

RAGK_API int ragk_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// handles: world x ragk_ar_handle_size() bytes (own entry ignored)
RAGK_API int ragk_ar_open_peers(void* hp, const void* handles) {
  ArHandle* h = (ArHandle*)hp;
  const size_t hs = sizeof(hipIpcMemHandle_t);
  for (int p = 0; p < h->world; ++p) {
    if (p == h->rank) continue;
    hipIpcMemHandle_t mh;
    memcpy(&mh, (const char*)handles + p * hs, hs);
    void* ptr = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&ptr, mh, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    h->peers.base[p] = (char*)ptr;
    h->opened[p] = true;
  }
  return 0;
}

RAGK_API long ragk_ar_max_bytes(void* hp) { return (long)((ArHandle*)hp)->data_bytes; }

// Bound of each peer wait in microseconds (default 5 s); tests shorten it.
RAGK_API int ragk_ar_set_spin_limit(void* hp, unsigned limit_us) {
  ArHandle* h = (ArHandle*)hp;
  if (!h || limit_us == 0) return (int)hipErrorInvalidValue;
  h->peers.spin_limit = (unsigned long long)limit_us * 100ull;  // 100 MHz ticks (a 32-bit bound capped at 43 s)
  return 0;
}

// System-scope release/acquire fences around the fused row barriers: 1 on, 0 off. Required when any
// peer region is on another device (xGMI); optional for same-device probes.
RAGK_API int ragk_ar_set_fences(void* hp, int on) {
  ArHandle* h = (ArHandle*)hp;
  if (!h) return (int)hipErrorInvalidValue;
  h->peers.fences = on ? 1 : 0;
  return 0;
}

RAGK_API int ragk_ar_get_fences(void* hp) { return hp ? ((ArHandle*)hp)->peers.fences : -1; }

// Host address of the pinned error word (0 = healthy): readable at any time without a device sync.
RAGK_API void* ragk_ar_error_host_ptr(void* hp) { return ((ArHandle*)hp)->host_err; }

// in: nbytes per rank (multiple of 16, 16-byte aligned); out: world * nbytes, rank order.
RAGK_API int ragk_ar_allgather(void* hp, const void* in, void* out, long nbytes, hipStream_t st) {
  ArHandle* h = (ArHandle*)hp;
  if (!h || nbytes <= 0) return nbytes == 0 ? 0 : (int)hipErrorInvalidValue;
  if (nbytes % 16 || (size_t)nbytes > h->data_bytes || ((uintptr_t)in & 15) || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  for (int p = 0; p < h->world; ++p)
    if (!h->peers.base[p]) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(allgather_kernel, dim3(h->blocks), dim3(AR_THREADS), 0, st, h->peers, h->rank, h->world,
                     (const u32x4*)in, (u32x4*)out, nbytes / 16, h->data_bytes);
  return (int)hipGetLastError();
}

// in/out: bf16[n] (n % 8 == 0, 16-byte aligned; in == out allowed). mode 0 = one-shot, 1 = two-shot.
RAGK_API int ragk_ar_allreduce(void* hp, const void* in, void* out, long n, int mode, hipStream_t st) {
  ArHandle* h = (ArHandle*)hp;
  if (!h || n <= 0) return n == 0 ? 0 : (int)hipErrorInvalidValue;
  if (n % 8 || (size_t)n * 2 > h->data_bytes || ((uintptr_t)in & 15) || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  for (int p = 0; p < h->world; ++p)
    if (!h->peers.base[p]) return (int)hipErrorInvalidValue;  // peers not opened
  const long n8 = n / 8;
  const int blocks = h->blocks;
  if (mode == 1)
    hipLaunchKernelGGL(allreduce_kernel<true>, dim3(blocks), dim3(AR_THREADS), 0, st, h->peers, h->rank, h->world,
                       (const bf16_t*)in, (bf16_t*)out, n8, h->data_bytes);
  else
    hipLaunchKernelGGL(allreduce_kernel<false>, dim3(blocks), dim3(AR_THREADS), 0, st, h->peers, h->rank, h->world,
                       (const bf16_t*)in, (bf16_t*)out, n8, h->data_bytes);
  return (int)hipGetLastError();
}

// Fused decode reduction: P = this rank's fp32 partial slabs [S][M][H]; h [M][ldh] bf16 residual
// (updated in place), w [H] bf16 norm weight, out [M][ldo] bf16. mode 0 = one-shot, 1 = two-shot.
RAGK_API int ragk_ar_add_rmsnorm(void* hp, const float* P, int S, int M, void* hres, int ldh, const void* w, void* out,
                                 int ldo, int H, float eps, int mode, hipStream_t st) {
  ArHandle* h = (ArHandle*)hp;
  if (!h || M <= 0) return M == 0 ? 0 : (int)hipErrorInvalidValue;
  if (!h->max_rows || M > h->max_rows || H > h->max_h || H % 8 || S < 1 || ldh % 8 || ldo % 8 ||
      ((uintptr_t)P & 15) || ((uintptr_t)hres & 15) || ((uintptr_t)out & 15) || ((uintptr_t)w & 15))
    return (int)hipErrorInvalidValue;
  for (int p = 0; p < h->world; ++p)
    if (!h->peers.base[p]) return (int)hipErrorInvalidValue;
  if (mode == 1)
    hipLaunchKernelGGL(ar_add_rmsnorm_kernel<true>, dim3(M), dim3(FR_THREADS), 0, st, h->peers, h->rank, h->world, P, S,
                       M, (bf16_t*)hres, ldh, (const bf16_t*)w, (bf16_t*)out, ldo, H, eps);
  else
    hipLaunchKernelGGL(ar_add_rmsnorm_kernel<false>, dim3(M), dim3(FR_THREADS), 0, st, h->peers, h->rank, h->world, P,
                       S, M, (bf16_t*)hres, ldh, (const bf16_t*)w, (bf16_t*)out, ldo, H, eps);
  return (int)hipGetLastError();
}

RAGK_API int ragk_ar_fused_rows(void* hp) { return hp ? ((ArHandle*)hp)->max_rows : 0; }

// 1 if any bounded spin gave up since creation (a peer never arrived), else 0; < 0 on error.
RAGK_API int ragk_ar_error(void* hp) {
  ArHandle* h = (ArHandle*)hp;
  unsigned v = 0;
  if (hipMemcpy(&v, h->local + offsetof(ArFlags, error), 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

RAGK_API void ragk_ar_destroy(void* hp) {
  ArHandle* h = (ArHandle*)hp;
  if (!h) return;
  for (int p = 0; p < h->world; ++p)
    if (h->opened[p]) (void)hipIpcCloseMemHandle(h->peers.base[p]);
  (void)hipFree(h->local);
  if (h->host_err) (void)hipHostFree(h->host_err);
  delete h;
}
