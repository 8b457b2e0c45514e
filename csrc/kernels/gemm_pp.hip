// 256x256x64 bf16 GEMM with an 8-wave "ping-pong" schedule for gfx950 (large-M prefill GEMMs).
//
// C[M,N] = A[M,K] . B[N,K]^T (+ fused epilogue), same operand layout / epilogues as gemm.hip.
//
// Structure (one 512-thread workgroup per CU, 128 KiB LDS = 2 K-tile buffers):
//   * wave w: group g = w>>2 owns output rows [128g, 128g+128), wq = w&3 owns cols [64wq, 64wq+64)
//     -> 8 x 4 tiles of mfma_f32_16x16x32_bf16 = 128 accumulator VGPRs per wave;
//   * every SIMD holds one wave of each group. Group 1 runs one barrier interval behind group 0,
//     so in every interval one wave per SIMD is in a COMPUTE segment (64 back-to-back MFMAs on
//     register fragments, setprio 1) while its partner is in a READ segment (24 ds_read_b128 of
//     the next K-tile's fragments + its share of the global->LDS DMA for a later K-tile);
//   * K-tile t lives in LDS buffer t&1; DMA for tile t+2 is issued (global_load_lds, 16 B/lane,
//     source-swizzled so the lane-linear LDS image is bank-conflict-free for ds_read_b128) in
//     interval 2t+2, after both groups have drained their reads of tile t (lgkmcnt(0) before the
//     barrier that ends every READ segment); each wave retires its own DMA with vmcnt(0) at the
//     end of interval 2t+3, one barrier before the first read of tile t+2 (interval 2t+4).
//     No __syncthreads() in the loop: raw s_barrier + explicit waits only.
//   * epilogue: the two groups stage their 128x256 fp32 halves through LDS in turn and the whole
//     workgroup writes 16-B row vectors with bias / residual / GELU / SiLU*up fused.
#include "common.h"
using namespace ragk;

namespace {

constexpr int PBM = 256, PBN = 256, PBK = 64;
constexpr int PP_THREADS = 512;
constexpr int TILE_A = PBM * PBK * 2;        // 32 KiB
constexpr int TILE_B = PBN * PBK * 2;        // 32 KiB
constexpr int BUF = TILE_A + TILE_B;         // 64 KiB per K-tile
constexpr int PEPI_LD = PBN + 4;             // padded fp32 row
constexpr int PEPI_BYTES = 128 * PEPI_LD * 4; // 133,120 B (one group's half)
constexpr int PP_LDS = (2 * BUF > PEPI_BYTES) ? 2 * BUF : PEPI_BYTES;
constexpr int PGROUP_M = 8;

__device__ __forceinline__ int pswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// 256 rows x 128 B = 32 pieces; wave w stages pieces 4w..4w+3.
__device__ __forceinline__ void pp_stage(const bf16_t* __restrict__ g, int ld, int row0, int rows_valid, int k0,
                                         char* lds, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid * 4 + i;
    const int r = q * 8 + (lane >> 3);
    const int c = pswz(r, lane & 7);
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    glds16(g + (size_t)gr * ld + k0 + c * 8, lds + q * 1024);
  }
}

__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Epilogue shared by the ping-pong kernels: each group stages its 128 x 256 fp32 half through LDS,
// then the whole workgroup writes 16-B row vectors with bias / residual / GELU / SiLU*up fused.
template <int EPI, bool OUT_F32>
__device__ __forceinline__ void pp_epilogue(const f32x4 (&acc)[8][4], char* smem, int tid, int grp, int wq, int fr,
                                            int fh, int m0, int n0, void* C, int ldc, const bf16_t* __restrict__ bias,
                                            const bf16_t* resid, int ldr, int M, int N) {
  float* sC = reinterpret_cast<float*>(smem);
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
    if (grp == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sC[(16 * i + 4 * fh + r) * PEPI_LD + wq * 64 + 16 * j + fr] = acc[i][j][r];
    }
    __syncthreads();
    const int mrow0 = m0 + h * 128;
    if constexpr (EPI == EPI_SILU_MUL) {
      // 256 packed cols = two [64 gate | 64 up] tiles -> 128 output cols
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int v = tid + it * PP_THREADS;  // 128 rows x 16 vec (2 halves x 8)
        const int row = v >> 4, hv = (v >> 3) & 1, c8 = (v & 7) * 8;
        const int gr = mrow0 + row;
        if (gr < M) {
          float o[8];
          const float* g = sC + row * PEPI_LD + hv * 128 + c8;
          const float* u = g + 64;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
          bf16_t* dst = reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + (n0 >> 1) + hv * 64 + c8;
          *reinterpret_cast<u32x4*>(dst) = pack8(o);
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int v = tid + it * PP_THREADS;  // 128 rows x 32 vec
        const int row = v >> 5, c8 = (v & 31) * 8;
        const int gr = mrow0 + row, gc = n0 + c8;
        if (gr < M && gc < N) {
          float o[8];
          const float* s = sC + row * PEPI_LD + c8;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = s[e];
          if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU ||
                        EPI == EPI_BIAS_GELU_TANH) {
            float b[8];
            unpack8(*reinterpret_cast<const u32x4*>(bias + gc), b);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += b[e];
          }
          if constexpr (EPI == EPI_RESID || EPI == EPI_BIAS_RESID) {
            float rr[8];
            unpack8(*reinterpret_cast<const u32x4*>(resid + (size_t)gr * ldr + gc), rr);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += rr[e];
          }
          if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = gelu_erf(o[e]);
          }
          if constexpr (EPI == EPI_BIAS_GELU_TANH) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = gelu_tanh(o[e]);
          }
          if constexpr (OUT_F32) {
            float* dst = reinterpret_cast<float*>(C) + (size_t)gr * ldc + gc;
            *reinterpret_cast<f32x4*>(dst) = (f32x4){o[0], o[1], o[2], o[3]};
            *reinterpret_cast<f32x4*>(dst + 4) = (f32x4){o[4], o[5], o[6], o[7]};
          } else {
            bf16_t* dst = reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + gc;
            *reinterpret_cast<u32x4*>(dst) = pack8(o);
          }
        }
      }
    }
  }
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(PP_THREADS, 1) void gemm_pp_kernel(const bf16_t* __restrict__ A, int lda,
                                                                const bf16_t* __restrict__ B, int ldb, void* C,
                                                                int ldc, const bf16_t* __restrict__ bias,
                                                                const bf16_t* resid, int ldr, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[PP_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wq = wid & 3;
  const int fr = lane & 15, fh = lane >> 4;

  const int tiles_m = (M + PBM - 1) / PBM, tiles_n = (N + PBN - 1) / PBN;
  const int nwg = tiles_m * tiles_n;
  const int logical = xcd_remap(blockIdx.x, nwg);
  const int group = logical / (PGROUP_M * tiles_n);
  const int first_m = group * PGROUP_M;
  const int gm = min(tiles_m - first_m, PGROUP_M);
  const int in_group = logical % (PGROUP_M * tiles_n);
  const int m0 = (first_m + in_group % gm) * PBM;
  const int n0 = (in_group / gm) * PBN;
  const int nk = K / PBK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[8][2], bfr[4][2];

  // prologue: tiles 0 and 1
  pp_stage(A, lda, m0, M, 0, smem, wid, lane);
  pp_stage(B, ldb, n0, N, 0, smem + TILE_A, wid, lane);
  if (nk > 1) {
    pp_stage(A, lda, m0, M, PBK, smem + BUF, wid, lane);
    pp_stage(B, ldb, n0, N, PBK, smem + BUF + TILE_A, wid, lane);
  }
  wait_vmcnt0();
  barrier_raw();       // boundary 0
  if (grp == 1) barrier_raw();  // group 1 runs one interval behind

  for (int t = 0; t < nk; ++t) {
    // ---------------- READ segment: fragments of tile t --------------------------------
    const char* sa = smem + (t & 1) * BUF;
    const char* sb = sa + TILE_A;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + fh;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int R = grp * 128 + 16 * i + fr;
        af[i][s] = *reinterpret_cast<const bf16x8*>(sa + R * 128 + 16 * pswz(R, c));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int R = wq * 64 + 16 * j + fr;
        bfr[j][s] = *reinterpret_cast<const bf16x8*>(sb + R * 128 + 16 * pswz(R, c));
      }
    }
    // group 0 issues the DMA of tile t+1's successor (t+2 is due in interval 2t+2 = this one for group 0)
    if (grp == 0 && t >= 1 && t + 1 < nk) {
      char* dst = smem + ((t + 1) & 1) * BUF;  // == buffer of tile t-1 (drained by both groups)
      pp_stage(A, lda, m0, M, (t + 1) * PBK, dst, wid, lane);
      pp_stage(B, ldb, n0, N, (t + 1) * PBK, dst + TILE_A, wid, lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp == 1) wait_vmcnt0();  // end of interval 2t+1 (odd): retire own DMA
    barrier_raw();
    // ---------------- COMPUTE segment: 64 MFMAs ----------------------------------------
    // Tile X is DMA'd by every wave in global interval 2X-2: group 0 from READ(X-1), group 1 from
    // COMPUTE(X-2) (its interval 2t+2). Both groups' reads of tile X-2 (same buffer) ended by then.
    if (grp == 1 && t + 2 < nk) {
      char* dst = smem + (t & 1) * BUF;
      pp_stage(A, lda, m0, M, (t + 2) * PBK, dst, wid, lane);
      pp_stage(B, ldb, n0, N, (t + 2) * PBK, dst + TILE_A, wid, lane);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (grp == 0) wait_vmcnt0();  // end of interval 2t+1... (group 0's compute interval is odd)
    barrier_raw();
  }
  if (grp == 0) barrier_raw();  // match group 1's extra barrier
  wait_vmcnt0();

  pp_epilogue<EPI, OUT_F32>(acc, smem, tid, grp, wq, fr, fh, m0, n0, C, ldc, bias, resid, ldr, M, N);
}


// ------------------------------------------------------------------------------------------------
// Variant 4 (experimental, A/B only): same 256x256 tile, waves and ping-pong, but 32-deep K-tiles
// in a 4-buffer ring (4 x 32 KiB). Each K-tile's DMA is issued 6 barrier intervals (3 K-tiles)
// before its first read instead of 2; waits are counted (vmcnt(8) = the two younger tiles may stay
// in flight), never 0 in steady state. Measured 8-13 % SLOWER than variant 2 on Llama-8B prefill
// shapes (1.17-1.26 vs 1.23-1.38 PF at M=16384): DMA latency was not the limiter, and the halved
// MFMA bursts (32 per interval) add barrier overhead. Kept for A/B (RAGK_PP_VARIANT=4).
//   group 0: READ(t) at global interval 2t, COMPUTE(t) at 2t+1, issues tile t+3 in READ(t);
//   group 1: one interval behind, issues tile t+4 in COMPUTE(t);
//   both halves of tile X are issued in global interval 2X-6, after group 1's READ(X-4) (the
//   buffer's previous tile) ended with lgkmcnt(0) + barrier; each wave retires its part of tile X
//   by the barrier that ends global interval 2X-1.
// 64-B LDS rows: chunk c of row R sits in 16-B slot c ^ ((R>>1)&3) -- conflict-free for the
// ds_read_b128 lane groups ({0-3,12-15,20-27}, ...).
// ------------------------------------------------------------------------------------------------
constexpr int P4K = 32;
constexpr int P4_TILE = 256 * P4K * 2;  // 16 KiB per operand tile
constexpr int P4_BUF = 2 * P4_TILE;     // 32 KiB per K-tile
constexpr int P4_NB = 4;
constexpr int P4_LDS = (P4_NB * P4_BUF > PEPI_BYTES) ? P4_NB * P4_BUF : PEPI_BYTES;

__device__ __forceinline__ int swz4(int row, int chunk) { return chunk ^ ((row >> 1) & 3); }

// one K-tile = 32 pieces of 16 rows x 64 B (A: 0-15, B: 16-31); wave w stages pieces 4w..4w+3
__device__ __forceinline__ void pp4_stage(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ B,
                                          int ldb, int m0, int M, int n0, int N, int k0, char* buf, int wid,
                                          int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid * 4 + i;
    const bool isA = q < 16;
    const int r = (q & 15) * 16 + (lane >> 2);
    const int c = swz4(r, lane & 3);
    const bf16_t* g = isA ? A : B;
    const int ld = isA ? lda : ldb;
    const int rv = isA ? M : N;
    int gr = (isA ? m0 : n0) + r;
    gr = gr < rv ? gr : rv - 1;
    glds16(g + (size_t)gr * ld + k0 + c * 8, buf + q * 1024);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}

// wait for tile `x`'s own DMA, given the newest tile this wave has issued
__device__ __forceinline__ void pp4_wait(int x, int newest) {
  const int younger = newest - x;  // tiles issued after x (each 4 glds per wave)
  if (younger >= 2) wait_vm<8>();
  else if (younger == 1) wait_vm<4>();
  else wait_vm<0>();
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(PP_THREADS, 1) void gemm_pp4_kernel(const bf16_t* __restrict__ A, int lda,
                                                                 const bf16_t* __restrict__ B, int ldb, void* C,
                                                                 int ldc, const bf16_t* __restrict__ bias,
                                                                 const bf16_t* resid, int ldr, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[P4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wq = wid & 3;
  const int fr = lane & 15, fh = lane >> 4;

  const int tiles_m = (M + PBM - 1) / PBM, tiles_n = (N + PBN - 1) / PBN;
  const int nwg = tiles_m * tiles_n;
  const int logical = xcd_remap(blockIdx.x, nwg);
  const int group = logical / (PGROUP_M * tiles_n);
  const int first_m = group * PGROUP_M;
  const int gm = min(tiles_m - first_m, PGROUP_M);
  const int in_group = logical % (PGROUP_M * tiles_n);
  const int m0 = (first_m + in_group % gm) * PBM;
  const int n0 = (in_group / gm) * PBN;
  const int nk = K / P4K;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[8], bfr[4];

  auto stage = [&](int x) {
    pp4_stage(A, lda, B, ldb, m0, M, n0, N, x * P4K, smem + (x % P4_NB) * P4_BUF, wid, lane);
  };
  // prologue: tiles 0..2 by everyone, tile 3 by group 1 (group 0 issues it in READ(0))
  int newest = -1;
#pragma unroll
  for (int x = 0; x < 3; ++x)
    if (x < nk) {
      stage(x);
      newest = x;
    }
  if (grp == 1 && 3 < nk) {
    stage(3);
    newest = 3;
  }
  pp4_wait(0, newest);
  barrier_raw();                // boundary 0
  if (grp == 1) barrier_raw();  // group 1 runs one interval behind

  for (int t = 0; t < nk; ++t) {
    // ---------------- READ segment: fragments of tile t ---------------------------------
    const char* sa = smem + (t % P4_NB) * P4_BUF;
    const char* sb = sa + P4_TILE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int R = grp * 128 + 16 * i + fr;
      af[i] = *reinterpret_cast<const bf16x8*>(sa + R * 64 + 16 * swz4(R, fh));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int R = wq * 64 + 16 * j + fr;
      bfr[j] = *reinterpret_cast<const bf16x8*>(sb + R * 64 + 16 * swz4(R, fh));
    }
    if (grp == 0 && t + 3 < nk) {
      stage(t + 3);
      newest = t + 3;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp == 1 && t + 1 < nk) pp4_wait(t + 1, newest);  // group 1's interval 2t+1 ends here
    barrier_raw();
    // ---------------- COMPUTE segment: 32 MFMAs -----------------------------------------
    if (grp == 1 && t + 4 < nk) {
      stage(t + 4);
      newest = t + 4;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (grp == 0 && t + 1 < nk) pp4_wait(t + 1, newest);  // group 0's interval 2t+1 ends here
    barrier_raw();
  }
  if (grp == 0) barrier_raw();  // match group 1's extra barrier
  wait_vmcnt0();
  pp_epilogue<EPI, OUT_F32>(acc, smem, tid, grp, wq, fr, fh, m0, n0, C, ldc, bias, resid, ldr, M, N);
}

int g_pp_variant = 2;  // 2: 2 x 64-deep buffers, 4: 4 x 32-deep ring (ragk_gemm_pp_set_variant)

template <int EPI, bool F32>
int launch_pp(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias, const void* resid,
              int ldr, int M, int N, int K, hipStream_t st) {
  const int nwg = ((M + PBM - 1) / PBM) * ((N + PBN - 1) / PBN);
  if (g_pp_variant == 4)
    hipLaunchKernelGGL((gemm_pp4_kernel<EPI, F32>), dim3(nwg), dim3(PP_THREADS), 0, st, (const bf16_t*)A, lda,
                       (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K);
  else
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, F32>), dim3(nwg), dim3(PP_THREADS), 0, st, (const bf16_t*)A, lda,
                       (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K);
  return (int)hipGetLastError();
}

}  // namespace

RAGK_API int ragk_gemm_pp_set_variant(int v) {
  if (v != 2 && v != 4) return (int)hipErrorInvalidValue;
  g_pp_variant = v;
  return 0;
}

// N = output columns (for EPI_SILU_MUL the weight has 2N rows, N % 128 == 0). Requires K % 64 == 0.
RAGK_API int ragk_gemm_pp(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                          const void* resid, int ldr, int M, int N, int K, int epi, int out_f32, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % PBK != 0) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL) {
    if (N % 128 != 0 || out_f32) return (int)hipErrorInvalidValue;
    return launch_pp<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, 2 * N, K, st);
  }
  if (N % 8 != 0) return (int)hipErrorInvalidValue;
#define RAGK_PP_CASE(E) \
  case E:               \
    return out_f32 ? launch_pp<E, true>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st) \
                   : launch_pp<E, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
  switch (epi) {
    RAGK_PP_CASE(EPI_NONE)
    RAGK_PP_CASE(EPI_BIAS)
    RAGK_PP_CASE(EPI_RESID)
    RAGK_PP_CASE(EPI_BIAS_RESID)
    RAGK_PP_CASE(EPI_BIAS_GELU)
    RAGK_PP_CASE(EPI_GELU)
    RAGK_PP_CASE(EPI_BIAS_GELU_TANH)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef RAGK_PP_CASE
}
