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


template <int EPI, bool F32>
int launch_pp(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias, const void* resid,
              int ldr, int M, int N, int K, hipStream_t st) {
  const int nwg = ((M + PBM - 1) / PBM) * ((N + PBN - 1) / PBN);
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, F32>), dim3(nwg), dim3(PP_THREADS), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K);
  return (int)hipGetLastError();
}

}  // namespace

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
