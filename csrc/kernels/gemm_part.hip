// Decode GEMM v5 for gfx950: split-K partial products, reduction left to the consumer kernel.
//
// P[s][M][N] (fp32) = X[M, s*KS:(s+1)*KS] . W[N, s*KS:(s+1)*KS]^T,  M <= 16*MT <= 64, s < S = K/KS.
//
// Why: at decode batch sizes the small-N projections (qkv, o_proj, down: 33-117 MB of weights)
// are latency-bound, not bandwidth-bound: the skinny / split-K kernels ran them at 2.0-2.8 TB/s
// (profiles/rocprof_bench_r1_kernels_v2.txt) because a block issues its weight loads one chunk at a
// time and split-K blocks then serialise on a last-arriver reduction. Here
//   * a block = 8 waves = 64 output columns x one K-slice; wave w owns n-tile (w & 3) and half
//     (w >> 2) of the slice, and issues ALL of its weight loads (NKS x 16 B per lane, straight to
//     VGPRs, non-temporal) before touching anything else -> the whole matrix is in flight within
//     the first microsecond;
//   * the activation slice (16*MT rows x KS) is DMA'd once per block into LDS (XOR-swizzled rows,
//     conflict-free ds_read_b128) and shared by the 4 n-tile waves;
//   * the two K-halves meet in LDS, and the block writes its fp32 partial tile to slab s. There is
//     no inter-block synchronisation: the consumer (ragk_add_partials_rmsnorm / rope_kv_partials in
//     norm.hip) sums the S slabs while doing its own row work, so the reduction costs no extra
//     launch and no atomics (deterministic).
#include <stdlib.h>

#include "common.h"
using namespace ragk;

namespace {

constexpr int PT_THREADS = 512;
constexpr int PT_NB = 64;  // output columns per block

__device__ __forceinline__ int pswz16(int row, int chunk) { return chunk ^ (row & 15); }

// e4m3fn x 8 -> bf16 x 8, exact (3 mantissa bits fit bf16's 7; the f32 -> bf16 step truncates bits
// that are zero)
__device__ __forceinline__ unsigned pf32x2_bf16(f32x2 f) {
  return __builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u);
}
__device__ __forceinline__ bf16x8 p_fp8x8_bf16(unsigned lo, unsigned hi) {
  u32x4 r;
  r[0] = pf32x2_bf16(__builtin_amdgcn_cvt_pk_f32_fp8((int)lo, false));
  r[1] = pf32x2_bf16(__builtin_amdgcn_cvt_pk_f32_fp8((int)lo, true));
  r[2] = pf32x2_bf16(__builtin_amdgcn_cvt_pk_f32_fp8((int)hi, false));
  r[3] = pf32x2_bf16(__builtin_amdgcn_cvt_pk_f32_fp8((int)hi, true));
  return __builtin_bit_cast(bf16x8, r);
}

// FP8 (W8A16, BASELINE config 5): W is e4m3fn [N][K] bytes with one fp32 scale per row. A lane's
// 16-B load is 16 consecutive k of one row, i.e. two MFMA k-steps: lane (fr, fh) of 64-k block j
// holds k = 64j + 16fh + [0, 8) for the first MFMA and + [8, 16) for the second; the activation
// fragments are read from LDS at the same k (chunks 8j + 2fh and 8j + 2fh + 1), so both operands
// see the same permutation of K and the dot product is unchanged. Half the weight bytes of bf16 per
// K-slice; the row scale is applied to the partial before it is written.
// NORM (decode batch <= 4): X is the un-normalised residual stream h and the block applies the
// following RMSNorm itself -- out = bf16(gamma * bf16(h * rsqrt(mean(h^2) + eps))), exactly
// rmsnorm_kernel's math and reduction order (threads 0..255 sum their row vectors in the same order,
// the wave partials are added in the same order; waves 4..7 add zeros) -- so the separate norm
// launch before the qkv projection disappears. Every block reads the full rows (8 KiB each at
// K = 4096, L2-resident) for the sum of squares; its weight stream is already in flight.
// NR = rows (M), NV = 16-B row vectors per thread (threads 0..255: K = 2048 NV); NR = 0: no norm.
constexpr int NORM_MAXR = 4;

// MG (o_proj at decode batch <= 4): the activation is the split-K decode attention's UNMERGED output
// -- per (sequence, query head) max_parts partial (O, max, sum) records (attention.hip, written with the
// separate merge launch deferred) -- and every block merges the heads of its own K-slice while its
// weight stream is in flight: the attn_decode_reduce launch (~5 us of pure latency per layer at batch
// 1) disappears. The merge math is attn_decode_reduce_kernel's (max-rescaled sums, bf16(O / L)); only
// the fp32 summation order differs. Rows whose sequence used a single partition were written as bf16
// by the attention kernel itself and are read from there.
struct MergeArgs {
  const float* part_o;   // [B][Hq][max_parts][MG_D]
  const float* part_ml;  // [B][Hq][max_parts][2] (max, sum)
  const bf16_t* out;     // [B][out_stride] bf16: rows with a single partition
  int out_stride;
  const int* kv_lens;    // [B]
  int Hq, part_tiles, max_parts;
};
constexpr int MG_D = 128;    // head dim
constexpr int MG_KT = 64;    // keys per KV tile (attention.hip KT)
constexpr int MG_MAXPP = 32; // partition records merged per thread (host check)
constexpr int MG_CHUNK = 4;  // records in flight per thread
constexpr int MG_MAXR = 4;   // rows
// The merge runs on 4 EXTRA waves (threads 512..767) that issue no weight loads: vmcnt is per wave, so
// the 8 weight-streaming waves issue their whole stream at once as before and never wait behind the
// partition-record loads (merging in the weight waves themselves, ahead of their stream, was slower
// than the separate reduce launch).
constexpr int MG_THREADS = 256;
// partition groups per (row, head, 4-column) task: the merge threads split the partitions of a task
__host__ __device__ inline int mg_groups(int M, int KS) {
  const int tasks = M * (KS / MG_D) * (MG_D / 4);
  int pg = 1;
  while (pg < 8 && tasks * pg * 2 <= MG_THREADS) pg *= 2;
  return pg;
}

// SG (down projection at decode batch <= 4 under tensor parallelism): the activation is silu(gate) * up
// of the packed gate/up projection's UNREDUCED split-K partials Pgu[S1][M][2K] (gemm_part of the
// packed weight, 128-row tiles of [64 gate | 64 up], ops/reference.py pack_gate_up): each block sums
// the S1 slabs of the gate and up columns of its own K-slice, applies silu(g) * u (fp32, rounded to
// bf16 once -- the silu_mul epilogue's math) and stages the slice in LDS. The gate/up GEMM then
// streams its shard with every load in flight instead of the register-streaming skinny kernel
// (12.8 us for a 29 MB TP=8 shard, profiles/tp_decode_probe_kernels_r3.txt). One item per thread:
// row tid / CPR, 8 columns (tid % CPR) * 8; all S1 slabs' loads issued before the weight stream.
constexpr int SG_MAXS = 4;
struct SiluArgs {
  const float* pgu;  // [S1][M][2K]
  int S1;
};

template <int MT, int NKS, bool FP8 = false, int NR = 0, int NV = 1, bool MG = false, bool SG = false>
__global__ __launch_bounds__(PT_THREADS + (MG ? MG_THREADS : 0), MG ? 2 : 1) void gemm_part_kernel(const bf16_t* __restrict__ X, int ldx,
                                                                  const bf16_t* __restrict__ W, int ldw,
                                                                  float* __restrict__ P, int M, int N, int K,
                                                                  const float* __restrict__ wscale = nullptr,
                                                                  const bf16_t* __restrict__ gamma = nullptr,
                                                                  float eps = 0.f, MergeArgs mg = {},
                                                                  SiluArgs sg = {}, int wnt = 1) {
  constexpr int KS = NKS * 64;          // K-slice of the block (two halves of NKS k-steps of 32)
  constexpr int XROWS = 16 * MT;
  constexpr int ROWB = KS * 2;          // bytes per LDS row
  constexpr int XBYTES = XROWS * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[XBYTES > 16384 ? XBYTES : 16384];
  constexpr bool NORM = NR > 0;
  __shared__ float s_red[NORM ? NR * (PT_THREADS / 64) : 1];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = wid & 3, kh = wid >> 2;
  const int fr = lane & 15, fh = lane >> 4;
  const int n0 = blockIdx.x * PT_NB, s = blockIdx.y;
  const int kbase = s * KS;

  // 1) activation slice -> LDS first (so a counted vmcnt can retire it before the weights): 16-B
  //    chunk c of row r lives at chunk slot c ^ (r & 15) (source-swizzled LDS-DMA: the LDS image is
  //    lane-linear, the global address carries the XOR)
  constexpr int CPR = ROWB / 16;                 // chunks per row
  constexpr int PIECES = XBYTES / 1024;          // 1-KiB pieces (64 lanes x 16 B)
  constexpr int PPW = PIECES / (PT_THREADS / 64);
  static_assert(PIECES % (PT_THREADS / 64) == 0 && CPR >= 16, "activation slice shape");
  u32x4 hv[NORM ? NR : 1][NV];  // NORM: raw row vectors (tid & 255) + 256 i
  u32x4 gv[NV];
  if constexpr (NORM) {
    // full rows (vectors tid + 256 i, threads < 256) and gamma for the slice's vectors, issued before
    // the weight stream so the counted wait below retires them first
    // branch-free: every load is issued (addresses clamped into range) and masked afterwards, so the
    // compiler keeps them all in flight (predicated loads behind branches got a vmcnt(0) each)
    // (waves 4..7 repeat waves 0..3's addresses -- L1 hits -- and are masked at use, after the weight
    // loads are issued)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = (tid & 255) + 256 * i;
#pragma unroll
      for (int r = 0; r < NR; ++r) hv[r][i] = *reinterpret_cast<const u32x4*>(X + (size_t)r * ldx + vi * 8);
      const int gi = min(max(vi * 8, kbase), kbase + KS - 8);
      gv[i] = *reinterpret_cast<const u32x4*>(gamma + gi);
    }
  } else if constexpr (MG) {
    // merge waves: the whole merge happens here (these waves stream no weights); tasks (row r, head j
    // of the slice, columns 4 d4 .. 4 d4 + 3) in rounds of MG_THREADS / npg, partitions pg, pg + npg, ...
    // of a task on npg adjacent lanes (indices clamped, all loads of a round in flight)
    if (wid >= PT_THREADS / 64) {
      const int npg = mg_groups(M, KS);
      const int per = MG_THREADS / npg, ntask = M * (KS / 4);
      const int pg = (tid - PT_THREADS) % npg;
      for (int t0 = 0; t0 < ntask; t0 += per) {
        const int task = t0 + (tid - PT_THREADS) / npg;
        const bool act = task < ntask;
        const int tk = act ? task : 0;
        const int r = tk / (KS / 4);
        const int j = (tk / (MG_D / 4)) % (KS / MG_D), d4 = tk % (MG_D / 4);
        const int hq = kbase / MG_D + j;
        // kv_len of row r: uniform scalar loads, selected per lane
        int kvl = mg.kv_lens[0];
#pragma unroll
        for (int rr = 1; rr < MG_MAXR; ++rr) {
          const int v = mg.kv_lens[min(rr, M - 1)];
          kvl = r == rr ? v : kvl;
        }
        const int n_kt = (kvl + MG_KT - 1) / MG_KT;
        const int pt = max(mg.part_tiles, (n_kt + mg.max_parts - 1) / mg.max_parts);
        const int np = (n_kt + pt - 1) / pt;
        const size_t pb = ((size_t)r * mg.Hq + hq) * mg.max_parts;
        const uint2 one = *reinterpret_cast<const uint2*>(mg.out + (size_t)r * mg.out_stride + hq * MG_D + 4 * d4);
        // online max-rescaled merge of this lane's partitions pg, pg + npg, ... in chunks of MG_CHUNK
        // records (a chunk's loads in flight together; few registers, so two blocks fit per CU), then
        // across the task's npg lanes
        float mx = -INFINITY, l = 0.f;
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        const int mine = (np - pg + npg - 1) / npg;  // partitions of this lane
        for (int c0 = 0; c0 < mine; c0 += MG_CHUNK) {
          f32x4 po[MG_CHUNK];
          f32x2 pml[MG_CHUNK];
#pragma unroll
          for (int i = 0; i < MG_CHUNK; ++i) {
            const int p = min(pg + (c0 + i) * npg, np - 1);
            po[i] = *reinterpret_cast<const f32x4*>(mg.part_o + (pb + p) * MG_D + 4 * d4);
            pml[i] = *reinterpret_cast<const f32x2*>(mg.part_ml + (pb + p) * 2);
          }
          float cm = mx;
#pragma unroll
          for (int i = 0; i < MG_CHUNK; ++i) cm = c0 + i < mine ? fmaxf(cm, pml[i][0]) : cm;
          const float sa = mx == -INFINITY ? 0.f : exp2f(mx - cm);  // cm finite: chunk has a valid record
          l *= sa;
          o *= sa;
#pragma unroll
          for (int i = 0; i < MG_CHUNK; ++i) {
            const float sc = c0 + i < mine ? exp2f(pml[i][0] - cm) : 0.f;
            l += pml[i][1] * sc;
            o += po[i] * sc;
          }
          mx = cm;
        }
        for (int off = 1; off < npg; off <<= 1) {
          const float mo = __shfl_xor(mx, off, 64), lo = __shfl_xor(l, off, 64);
          f32x4 oo;
#pragma unroll
          for (int e = 0; e < 4; ++e) oo[e] = __shfl_xor(o[e], off, 64);
          const float mn = fmaxf(mx, mo);
          const float sa = mx == -INFINITY ? 0.f : exp2f(mx - mn), sb = mo == -INFINITY ? 0.f : exp2f(mo - mn);
          l = l * sa + lo * sb;
          o = o * sa + oo * sb;
          mx = mn;
        }
        if (act && pg == 0) {
          uint2 v = one;  // single partition: the attention kernel wrote the row itself
          if (np > 1) {
            v.x = pk2bf(l > 0.f ? o[0] / l : 0.f, l > 0.f ? o[1] / l : 0.f);
            v.y = pk2bf(l > 0.f ? o[2] / l : 0.f, l > 0.f ? o[3] / l : 0.f);
          }
          const int cc = j * (MG_D / 8) + d4 / 2;  // 16-B chunk of the slice row; 8-B half d4 & 1
          const int c = (cc & ~15) | ((cc & 15) ^ (r & 15));
          *reinterpret_cast<uint2*>(smem + r * ROWB + 16 * c + 8 * (d4 & 1)) = v;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  f32x4 sgv[SG ? SG_MAXS : 1][4];  // SG: gate lo/hi, up lo/hi of each slab
  if constexpr (SG) {
    // (loads unconditional: row / slab clamped, masked at use, so one counted vmcnt retires them)
    const int r = min(tid / CPR, M - 1), c = tid % CPR;
    const int j = kbase + 8 * c;
    const float* pg = sg.pgu + (size_t)r * 2 * K + (j >> 6) * 128 + (j & 63);
#pragma unroll
    for (int s2 = 0; s2 < SG_MAXS; ++s2) {
      const float* ps = pg + (size_t)min(s2, sg.S1 - 1) * M * 2 * K;
      sgv[s2][0] = *reinterpret_cast<const f32x4*>(ps);
      sgv[s2][1] = *reinterpret_cast<const f32x4*>(ps + 4);
      sgv[s2][2] = *reinterpret_cast<const f32x4*>(ps + 64);
      sgv[s2][3] = *reinterpret_cast<const f32x4*>(ps + 68);
    }
  } else if constexpr (!NORM && !MG) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wid * PPW + i;
      const int e = p * 64 + lane;                 // destination chunk index (lane-linear)
      const int r = e / CPR, slot = e % CPR;
      const int c = (slot & ~15) | ((slot & 15) ^ (r & 15));
      const int gr = min(r, M - 1);
      glds16(X + (size_t)gr * ldx + kbase + c * 8, smem + p * 1024);
    }
  }

  __builtin_amdgcn_sched_barrier(0);
  // 2) this wave's whole weight stream, all loads in flight: row n0 + 16nt + fr,
  //    bf16: k = kbase + kh*KS/2 + 32ks + 8fh;  fp8: k = kbase + kh*KS/2 + 64j + 16fh (16 k per load)
  constexpr int NLD = FP8 ? NKS / 2 : NKS;  // 16-B loads per lane
  static_assert(!FP8 || NKS % 2 == 0, "fp8 slices cover whole 64-k blocks");
  const int wrow = min(n0 + 16 * nt + fr, N - 1);
  const bool wwave = !MG || wid < PT_THREADS / 64;  // wave-uniform: MG's merge waves stream no weights
  bf16x8 wf[NLD];
  if (!wwave) {
  } else if constexpr (FP8) {
    const unsigned char* wp = reinterpret_cast<const unsigned char*>(W) + (size_t)wrow * ldw + kbase + kh * (KS / 2) +
                              fh * 16;
#pragma unroll
    for (int j = 0; j < NLD; ++j)
      wf[j] = wnt ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + 64 * j))
                  : *reinterpret_cast<const bf16x8*>(wp + 64 * j);
  } else {
    const bf16_t* wp = W + (size_t)wrow * ldw + kbase + kh * (KS / 2) + fh * 8;
#pragma unroll
    for (int ks = 0; ks < NLD; ++ks)
      wf[ks] = wnt ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + 32 * ks))
                   : *reinterpret_cast<const bf16x8*>(wp + 32 * ks);
  }
  // vmcnt(NLD): the DMA / row loads (older than the NLD weight loads) have landed
  __builtin_amdgcn_s_waitcnt((NLD & 15) | (((NLD >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (SG) {
    const int r = tid / CPR, c = tid % CPR;
    if (r < M) {
      f32x4 g0 = sgv[0][0], g1 = sgv[0][1], u0 = sgv[0][2], u1 = sgv[0][3];
#pragma unroll
      for (int s2 = 1; s2 < SG_MAXS; ++s2) {
        if (s2 < sg.S1) {
          g0 += sgv[s2][0];
          g1 += sgv[s2][1];
          u0 += sgv[s2][2];
          u1 += sgv[s2][3];
        }
      }
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = silu(g0[e]) * u0[e];
        o[4 + e] = silu(g1[e]) * u1[e];
      }
      *reinterpret_cast<u32x4*>(smem + r * ROWB + 16 * ((c & ~15) | ((c & 15) ^ (r & 15)))) = pack8(o);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (NORM) {
    // RMSNorm statistics (rmsnorm_kernel order), then the normalised slice -> LDS (rows >= M are
    // left as they are: their accumulator rows are never stored)
    float ss[NR];
    const u32x4 z = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      ss[r] = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        hv[r][i] = tid < 256 ? hv[r][i] : z;
        float f[8];
        unpack8(hv[r][i], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) ss[r] += f[e] * f[e];
      }
      ss[r] = wave_sum(ss[r]);
      if (lane == 0) s_red[r * (PT_THREADS / 64) + wid] = ss[r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < PT_THREADS / 64; ++w) t += s_red[r * (PT_THREADS / 64) + w];
      const float inv = rsqrtf(t / (float)K + eps);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int vi = tid + 256 * i;
        if (tid < 256 && vi * 8 >= kbase && vi * 8 < kbase + KS) {
          float f[8], g[8], o[8];
          unpack8(hv[r][i], f);
          unpack8(gv[i], g);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = g[e] * bf2f(f2bf(f[e] * inv));
          const int c = vi - kbase / 8;
          *reinterpret_cast<u32x4*>(smem + r * ROWB + 16 * ((c & ~15) | ((c & 15) ^ (r & 15)))) = pack8(o);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();  // raw: __syncthreads() would drain the weight loads too (vmcnt(0))
  __builtin_amdgcn_sched_barrier(0);

  // 3) MFMA: A = activation fragment (rows 16t + fr), B = weight fragment (cols 16nt + fr)
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto xfrag = [&](int chunk, int t) {
    const int r = 16 * t + fr;
    return *reinterpret_cast<const bf16x8*>(smem + r * ROWB + 16 * ((chunk & ~15) | ((chunk & 15) ^ (r & 15))));
  };
  if (!wwave) {
  } else if constexpr (FP8) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const u32x4 raw = __builtin_bit_cast(u32x4, wf[j]);
      const bf16x8 w0 = p_fp8x8_bf16(raw[0], raw[1]), w1 = p_fp8x8_bf16(raw[2], raw[3]);
      const int chunk = (kh * (KS / 2) + 64 * j) / 8 + 2 * fh;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xfrag(chunk, t), w0, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xfrag(chunk + 1, t), w1, acc[t], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < NLD; ++ks) {
      const int chunk = (kh * (KS / 2) + 32 * ks) / 8 + fh;
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xfrag(chunk, t), wf[ks], acc[t], 0, 0, 0);
    }
  }

  // 4) K-halves meet in LDS (the activation slice is dead), half 0 writes the partial slab
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  if (kh == 1) {
#pragma unroll
    for (int t = 0; t < MT; ++t) red[(nt * MT + t) * 64 + lane] = acc[t];
  }
  __syncthreads();
  if (kh == 0) {
    const int col = n0 + 16 * nt + fr;
    float* ps = P + (size_t)s * M * N;
    const float sc = FP8 ? wscale[min(col, N - 1)] : 1.f;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const f32x4 o = red[(nt * MT + t) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * t + 4 * fh + r;
        const float val = FP8 ? (acc[t][r] + o[r]) * sc : acc[t][r] + o[r];
        if (row < M && col < N) ps[(size_t)row * N + col] = val;
      }
    }
  }
}

template <int MT, bool FP8 = false, int NR = 0, int NV = 1, bool MG = false, bool SG = false>
int launch_part_mt(const void* X, int ldx, const void* W, int ldw, float* P, int M, int N, int K, int ks_steps,
                   hipStream_t st, const float* wscale = nullptr, const void* gamma = nullptr, float eps = 0.f,
                   MergeArgs mg = {}, SiluArgs sg = {}) {
  const int KS = ks_steps * 64;
  const dim3 grid((N + PT_NB - 1) / PT_NB, K / KS);
#define RAGK_PART(NK)                                                                                       \
  case NK:                                                                                                  \
    if constexpr (16 * MT * NK * 64 * 2 <= 128 * 1024 && (16 * MT * NK * 64 * 2) % 8192 == 0 &&           \
                  (NR == 0 || NK == 8 || NK == 16) && (!MG || NK == 4 || NK == 8) && (!SG || NK <= 16)) {   \
      hipLaunchKernelGGL((gemm_part_kernel<MT, NK, FP8, NR, NV, MG, SG>), grid, dim3(PT_THREADS + (MG ? MG_THREADS : 0)), \
                         0, st,                                                                             \
                         (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, P, M, N, K, wscale, (const bf16_t*)gamma, \
                         eps, mg, sg, 1);  /* non-temporal weight stream */                                                       \
      break;                                                                                                \
    } else {                                                                                                \
      return (int)hipErrorInvalidValue;                                                                     \
    }
  switch (ks_steps) {
    RAGK_PART(4)
    RAGK_PART(8)
    RAGK_PART(14)
    RAGK_PART(16)
    RAGK_PART(28)
    RAGK_PART(32)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef RAGK_PART
  return (int)hipGetLastError();
}

}  // namespace

// Slice choice: K-slice KS = 64 * ks_steps (ks_steps in {4, 8, 14, 16, 28, 32}; 14 / 28 divide the
// K = 14336 of Llama's down projection into 16 / 8 slabs; 4 = 256-wide slices for the narrow K of
// tensor-parallel shards: down at TP=8 has K = 1792 = 7 x 256, o_proj K = 512); S = K / KS slabs.
// Picks the largest slice that still gives >= g_part_min_blocks blocks and fits the activation slice
// in LDS, else the smallest legal slice (most blocks).
static int g_part_min_blocks = 256;
RAGK_API int ragk_gemm_part_set_min_blocks(int n) {
  g_part_min_blocks = n > 0 ? n : 256;
  return 0;
}

RAGK_API int ragk_gemm_part_ksteps(int M, int N, int K) {
  const int mt = (M + 15) / 16;
  const int nb = (N + PT_NB - 1) / PT_NB;
  int best = 0;
  for (int ks : {32, 28, 16, 14, 8, 4}) {
    const int KS = ks * 64;
    if (K % KS) continue;
    if (16 * mt * KS * 2 > 128 * 1024 || (16 * mt * KS * 2) % 8192) continue;  // LDS; 8 waves x 1-KiB DMA pieces
    if (best == 0) best = ks;  // largest legal slice
    if (nb * (K / KS) >= g_part_min_blocks) return ks;
    best = ks;
  }
  return best;
}

// P must hold (K / (64*ks_steps)) * M * N floats. M <= 64, K % (64*ks_steps) == 0.
RAGK_API int ragk_gemm_part(const void* X, int ldx, const void* W, int ldw, float* P, int M, int N, int K,
                            int ks_steps, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > 64 || ks_steps <= 0 || K % (64 * ks_steps) != 0) return (int)hipErrorInvalidValue;
  const int mt = (M + 15) / 16;
  if (16 * mt * ks_steps * 64 * 2 > 128 * 1024) return (int)hipErrorInvalidValue;
  switch (mt) {
    case 1: return launch_part_mt<1>(X, ldx, W, ldw, P, M, N, K, ks_steps, st);
    case 2: return launch_part_mt<2>(X, ldx, W, ldw, P, M, N, K, ks_steps, st);
    case 3: return launch_part_mt<3>(X, ldx, W, ldw, P, M, N, K, ks_steps, st);
    case 4: return launch_part_mt<4>(X, ldx, W, ldw, P, M, N, K, ks_steps, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// X = un-normalised rows h (M <= 4, K <= 8192); the block applies RMSNorm(h) * gamma (rmsnorm_kernel's
// exact math) before the product: P = partials of rmsnorm(h) . W^T. bf16 weights.
RAGK_API int ragk_gemm_part_norm(const void* X, int ldx, const void* gamma, float eps, const void* W, int ldw,
                                 float* P, int M, int N, int K, int ks_steps, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > NORM_MAXR || (K != 4096 && K != 8192) || !gamma || (ks_steps != 8 && ks_steps != 16) ||
      K % (64 * ks_steps) != 0)
    return (int)hipErrorInvalidValue;
#define RAGK_PN(R, V) return launch_part_mt<1, false, R, V>(X, ldx, W, ldw, P, M, N, K, ks_steps, st, nullptr, gamma, eps)
  if (K == 4096) {
    switch (M) { case 1: RAGK_PN(1, 2); case 2: RAGK_PN(2, 2); case 3: RAGK_PN(3, 2); default: RAGK_PN(4, 2); }
  }
  switch (M) { case 1: RAGK_PN(1, 4); case 2: RAGK_PN(2, 4); case 3: RAGK_PN(3, 4); default: RAGK_PN(4, 4); }
#undef RAGK_PN
}

// Down projection fed by the packed gate/up projection's split-K partials (SG above): P = partials of
// (silu(gate) * up) . W^T, gate / up = sum of the S1 slabs of pgu [S1][M][2K] (gemm_part of the packed
// [2K, H] weight). M <= 4, S1 <= SG_MAXS, K % 64 == 0, one staging item per thread (M * 8 * ks_steps <= 512).
RAGK_API int ragk_gemm_part_silu(const float* pgu, int S1, const void* W, int ldw, float* P, int M, int N, int K,
                                 int ks_steps, hipStream_t st) {
  if (M <= 0) return 0;
  if (!pgu || M > 4 || S1 < 1 || S1 > SG_MAXS || K % 64 || ks_steps <= 0 || ks_steps > 16 ||
      K % (64 * ks_steps) || M * 8 * ks_steps > PT_THREADS)
    return (int)hipErrorInvalidValue;
  return launch_part_mt<1, false, 0, 1, false, true>(nullptr, 0, W, ldw, P, M, N, K, ks_steps, st, nullptr, nullptr,
                                                      0.f, {}, SiluArgs{pgu, S1});
}

RAGK_API int ragk_gemm_part_silu_ok(int M, int S1, int K, int ks_steps) {
  return M >= 1 && M <= 4 && S1 >= 1 && S1 <= SG_MAXS && K % 64 == 0 && ks_steps > 0 && ks_steps <= 16 &&
         K % (64 * ks_steps) == 0 && M * 8 * ks_steps <= PT_THREADS;
}

// W8A16 variant: W = e4m3fn [N][K] bytes (ldw in bytes), wscale = fp32 [N]; same slabs / slices.
RAGK_API int ragk_gemm_part_fp8(const void* X, int ldx, const void* W8, int ldw, const float* wscale, float* P, int M,
                                int N, int K, int ks_steps, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > 64 || ks_steps <= 0 || ks_steps % 2 || K % (64 * ks_steps) != 0 || !wscale || ldw % 16)
    return (int)hipErrorInvalidValue;
  const int mt = (M + 15) / 16;
  if (16 * mt * ks_steps * 64 * 2 > 128 * 1024) return (int)hipErrorInvalidValue;
  switch (mt) {
    case 1: return launch_part_mt<1, true>(X, ldx, W8, ldw, P, M, N, K, ks_steps, st, wscale);
    case 2: return launch_part_mt<2, true>(X, ldx, W8, ldw, P, M, N, K, ks_steps, st, wscale);
    case 3: return launch_part_mt<3, true>(X, ldx, W8, ldw, P, M, N, K, ks_steps, st, wscale);
    case 4: return launch_part_mt<4, true>(X, ldx, W8, ldw, P, M, N, K, ks_steps, st, wscale);
    default: return (int)hipErrorInvalidValue;
  }
}

// o_proj fed by the decode attention's unmerged partitions (MG above; the attention launched with its
// merge deferred, ragk_attn_decode_set_defer). X (bf16 rows, out_stride) is the attention output buffer:
// rows whose sequence used one partition are read from it. M <= 4, head dim 128, K = Hq * 128, 8- or
// 4-step K-slices (a 16-step slice spills), at most MG_MAXPP partitions per thread. w8 / wscale: fp8 weights (ldw in bytes).
RAGK_API int ragk_gemm_part_merge(const float* part_o, const float* part_ml, const void* out, int out_stride,
                                  const int* kv_lens, int Hq, int part_tiles, int max_parts, const void* W, int ldw,
                                  const float* wscale, float* P, int M, int N, int K, int ks_steps, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > MG_MAXR || K != Hq * MG_D || (ks_steps != 8 && ks_steps != 4) || K % (64 * ks_steps) || max_parts < 2 ||
      !part_o || !part_ml || !out || !kv_lens || part_tiles < 1)
    return (int)hipErrorInvalidValue;
  const int npg = mg_groups(M, ks_steps * 64);
  if ((max_parts + npg - 1) / npg > MG_MAXPP) return (int)hipErrorInvalidValue;
  const MergeArgs mg{part_o, part_ml, (const bf16_t*)out, out_stride, kv_lens, Hq, part_tiles, max_parts};
  if (wscale) return launch_part_mt<1, true, 0, 1, true>(out, out_stride, W, ldw, P, M, N, K, ks_steps, st, wscale,
                                                          nullptr, 0.f, mg);
  return launch_part_mt<1, false, 0, 1, true>(out, out_stride, W, ldw, P, M, N, K, ks_steps, st, nullptr, nullptr,
                                              0.f, mg);
}

RAGK_API int ragk_gemm_part_merge_ok(int M, int K, int Hq, int max_parts, int ks_steps) {
  if (M <= 0 || M > MG_MAXR || K != Hq * MG_D || (ks_steps != 8 && ks_steps != 4) || max_parts < 2) return 0;
  const int npg = mg_groups(M, ks_steps * 64);
  return (max_parts + npg - 1) / npg <= MG_MAXPP;
}

