// Decode GEMM v3 for gfx950 (M <= 64 activation rows, weights streamed once from HBM).
//
// C[M,N] = X[M,K] . W[N,K]^T (+ fused epilogue). Block = 8 waves = 128 output columns (16 per
// wave, one 16x16x32 MFMA n-tile), grid = (N/128, S): K is split S ways across blocks so even
// N = 4096 projections put >= 256 workgroups on the 256 CUs.
//   * the activation K-chunk (16*MT rows x 256) is staged ONCE per block in LDS (XOR-swizzled
//     rows, conflict-free ds_read_b128) and read by all 8 waves -- 8x less activation traffic than
//     per-wave fragment loads, which capped the v1 kernel at 2-3 TB/s for M = 32..64;
//   * weights go straight to VGPRs with non-temporal loads, one 256-deep chunk prefetched;
//   * S > 1: each block writes its fp32 partial tile to a slab, then takes a ticket on the
//     n-tile's counter (plain stores -> every wave vmcnt(0) -> barrier -> lane-0 agent RELEASE
//     fence -> vmcnt(0) -> relaxed agent fetch_add); the block that draws S-1 acquires (agent
//     fence), sums the S slabs, applies the epilogue and resets the counter for the next call
//     (correct for any block -> XCD placement; counters are zeroed once at allocation).
#include "common.h"
using namespace ragk;

namespace {

constexpr int DK = 256;
constexpr int DEC_THREADS = 512;

__device__ __forceinline__ int xswz(int row, int chunk) { return chunk ^ (row & 15); }

template <int MT, int EPI, bool OUT_F32>
__global__ __launch_bounds__(DEC_THREADS, 1) void gemm_dec_kernel(
    const bf16_t* __restrict__ X, int ldx, const bf16_t* __restrict__ W, int ldw, void* C, int ldc,
    const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr, int M, int N, int K, int S, float* ws,
    int* counters) {
  constexpr bool PAIR = (EPI == EPI_SILU_MUL);
  constexpr int NACC = PAIR ? 2 : 1;
  constexpr int XROWS = 16 * MT;
  constexpr int XBUF = XROWS * DK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * XBUF + 16];
  int* s_flag = reinterpret_cast<int*>(smem + 2 * XBUF);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fh = lane >> 4;
  const int ntile = blockIdx.x, slice = blockIdx.y;
  const int col = ntile * 128 + wid * 16 + fr;
  const bf16_t* wp[NACC];
  if constexpr (PAIR) {
    const int c = min(col, N - 1);
    const int r0 = (c >> 6) * 128 + (c & 63);
    wp[0] = W + (size_t)r0 * ldw + fh * 8;
    wp[1] = W + (size_t)(r0 + 64) * ldw + fh * 8;
  } else {
    wp[0] = W + (size_t)min(col, N - 1) * ldw + fh * 8;
  }
  const int nk = (K / DK) / S;
  const int kbase = slice * nk * DK;

  f32x4 acc[NACC][MT];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[a][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 xr[MT];
  bf16x8 wA[NACC][8], wB[NACC][8];
  auto load_x = [&](int kc) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int p = tid + i * DEC_THREADS;
      const int row = p >> 5, ch = p & 31;
      xr[i] = *reinterpret_cast<const u32x4*>(X + (size_t)min(row, M - 1) * ldx + kbase + kc * DK + ch * 8);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int p = tid + i * DEC_THREADS;
      const int row = p >> 5, ch = p & 31;
      *reinterpret_cast<u32x4*>(smem + buf * XBUF + row * (DK * 2) + 16 * xswz(row, ch)) = xr[i];
    }
  };
  auto load_w = [&](int kc, bf16x8 (&w)[NACC][8]) {
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
      for (int s = 0; s < 8; ++s)
        w[a][s] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp[a] + kbase + kc * DK + 32 * s));
  };
  auto compute = [&](int buf, const bf16x8 (&w)[NACC][8]) {
    const char* xb = smem + buf * XBUF;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int row = 16 * t + fr;
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xb + row * (DK * 2) + 16 * xswz(row, 4 * s + fh));
#pragma unroll
        for (int a = 0; a < NACC; ++a)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, w[a][s], acc[a][t], 0, 0, 0);
      }
  };

  load_x(0);
  load_w(0, wA);
  store_x(0);
  __syncthreads();
  for (int i = 0; i < nk; i += 2) {
    if (i + 1 < nk) {
      load_x(i + 1);
      load_w(i + 1, wB);
    }
    compute(0, wA);
    if (i + 1 < nk) store_x(1);
    __syncthreads();
    if (i + 1 >= nk) break;
    if (i + 2 < nk) {
      load_x(i + 2);
      load_w(i + 2, wA);
    }
    compute(1, wB);
    if (i + 2 < nk) store_x(0);
    __syncthreads();
  }

  // ---------------- epilogue -----------------------------------------------------------
  auto finish = [&](int row, int c, float v, float u) {
    if constexpr (PAIR) v = silu(v) * u;
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH)
      v += bf2f(bias[c]);
    if constexpr (EPI == EPI_RESID || EPI == EPI_BIAS_RESID) v += bf2f(resid[(size_t)row * ldr + c]);
    if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) v = gelu_erf(v);
    if constexpr (EPI == EPI_BIAS_GELU_TANH) v = gelu_tanh(v);
    if constexpr (OUT_F32)
      reinterpret_cast<float*>(C)[(size_t)row * ldc + c] = v;
    else
      reinterpret_cast<bf16_t*>(C)[(size_t)row * ldc + c] = f2bf(v);
  };

  if (S == 1) {
    if (col < N) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + 4 * fh + r;
          if (row < M) finish(row, col, acc[0][t][r], PAIR ? acc[NACC - 1][t][r] : 0.f);
        }
    }
    return;
  }

  // split-K: partial slab ws[slice][a][row][N] (fp32), then last-arriver reduction
  const size_t slab = (size_t)NACC * M * N;
  if (col < N) {
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + 4 * fh + r;
          if (row < M) ws[slice * slab + ((size_t)a * M + row) * N + col] = acc[a][t][r];
        }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(counters + ntile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag[0] = (old == S - 1);
  }
  __syncthreads();
  if (!s_flag[0]) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int e = tid; e < M * 128; e += DEC_THREADS) {
    const int row = e >> 7, c = ntile * 128 + (e & 127);
    if (c >= N) continue;
    float v = 0.f, u = 0.f;
    for (int s = 0; s < S; ++s) {
      v += ws[s * slab + (size_t)row * N + c];
      if constexpr (PAIR) u += ws[s * slab + ((size_t)M + row) * N + c];
    }
    finish(row, c, v, u);
  }
  if (tid == 0) __hip_atomic_store(counters + ntile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int EPI, bool F32>
int launch_dec(const void* X, int ldx, const void* W, int ldw, void* C, int ldc, const void* bias, const void* resid,
               int ldr, int M, int N, int K, int S, float* ws, int* cnt, hipStream_t st) {
  const dim3 grid((N + 127) / 128, S);
  const int mt = (M + 15) / 16;
#define RAGK_DEC(MTV)                                                                                         \
  case MTV:                                                                                                   \
    hipLaunchKernelGGL((gemm_dec_kernel<MTV, EPI, F32>), grid, dim3(DEC_THREADS), 0, st, (const bf16_t*)X, ldx, \
                       (const bf16_t*)W, ldw, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K, S, \
                       ws, cnt);                                                                              \
    break;
  switch (mt) {
    RAGK_DEC(1)
    RAGK_DEC(2)
    RAGK_DEC(3)
    RAGK_DEC(4)
    default: return (int)hipErrorInvalidValue;
  }
#undef RAGK_DEC
  return (int)hipGetLastError();
}

}  // namespace

// Split factor chosen so that >= 256 workgroups stream the weights; S divides K/256.
RAGK_API int ragk_gemm_dec_splits(int N, int K, int epi) {
  const int nblk = (N + 127) / 128;
  const int nk = K / DK;
  int S = 1;
  while (nblk * S < 256 && nk % (2 * S) == 0 && 2 * S <= 16) S *= 2;
  (void)epi;
  return S;
}

// N = output columns (SILU_MUL: weight has 2N packed rows, N % 64 == 0). K % 256 == 0, M <= 64.
// ws must hold S * (2 if SILU_MUL else 1) * M * N floats; counters >= ceil(N/128) ints, zeroed once.
RAGK_API int ragk_gemm_dec(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                           const void* resid, int ldr, int M, int N, int K, int epi, int out_f32, int S, float* ws,
                           int* counters, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > 64 || K % DK != 0 || S < 1 || (K / DK) % S != 0) return (int)hipErrorInvalidValue;
  if (S > 1 && (ws == nullptr || counters == nullptr)) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL) {
    if (N % 64 != 0 || out_f32) return (int)hipErrorInvalidValue;
    return launch_dec<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, S, ws, counters, st);
  }
#define RAGK_DC3(E)                                                                                          \
  case E:                                                                                                    \
    return out_f32 ? launch_dec<E, true>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, S, ws, counters, st) \
                   : launch_dec<E, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, S, ws, counters, st);
  switch (epi) {
    RAGK_DC3(EPI_NONE)
    RAGK_DC3(EPI_BIAS)
    RAGK_DC3(EPI_RESID)
    RAGK_DC3(EPI_BIAS_RESID)
    RAGK_DC3(EPI_BIAS_GELU)
    RAGK_DC3(EPI_GELU)
    RAGK_DC3(EPI_BIAS_GELU_TANH)
    default: return (int)hipErrorInvalidValue;
  }
#undef RAGK_DC3
}
