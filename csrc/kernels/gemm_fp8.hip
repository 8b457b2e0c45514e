// fp8 (OCP e4m3fn) weight GEMMs for gfx950 -- BASELINE config 5 ("Llama-3.1-8B fp8 weights,
// CDNA4 fp8 MFMA"). Weights are quantized once at load with one fp32 scale per output row
// (W ≈ W8 * sw[n]); the reference runs the same GEMMs as fp32 CPU matmuls
// (/root/reference/llm/rag.py:24,172).
//
//  * quant_rows   : activations bf16 -> fp8 with one dynamic scale per row (token):
//                   sx[m] = amax(|x[m,:]|) / 448.
//  * gemm_fp8_tile: prefill (M > 64), W8A8. 128x128 block tile, 128-byte (=128 fp8) K steps
//                   staged with global_load_lds into XOR-swizzled LDS rows, and the
//                   block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit
//                   E8M0 block scales): 4x the K of the bf16 16x16x32 form at 2x its cycles,
//                   i.e. 2x bf16 throughput. Epilogue: acc * sx[m] * sw[n], then the same
//                   fused bias / residual / GELU / SiLU*up variants as the bf16 kernels.
//  * gemm_fp8_dec : decode (M <= 64), W8A16. Weight streaming at 1 byte per weight (half the
//                   HBM bytes of bf16 -- decode is bandwidth-bound); fp8 -> bf16 is exact and
//                   done in registers (v_cvt_pk_f32_fp8 + v_perm), then bf16 MFMA against
//                   the unquantized activations; acc * sw[n] in the epilogue.
#include "common.h"
using namespace ragk;

typedef int i32x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr float FP8_MAX = 448.f;

// ----------------------------------------------------------------------------- quantize
constexpr int Q_THREADS = 256;

__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  int v = 0;
  v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, v, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

// one block per row; K % 8 == 0
__global__ __launch_bounds__(Q_THREADS) void quant_rows_kernel(const bf16_t* __restrict__ x, int ldx, unsigned char* q,
                                                               int ldq, float* __restrict__ scale, int K) {
  __shared__ float red[Q_THREADS / 64];
  const int m = blockIdx.x;
  const bf16_t* row = x + (size_t)m * ldx;
  float amax = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += Q_THREADS * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(row + k), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(f[e]));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  float a = 0.f;
#pragma unroll
  for (int w = 0; w < Q_THREADS / 64; ++w) a = fmaxf(a, red[w]);
  // s = amax * fp32(1/448) then a correctly rounded 1/s: bit-identical to ops/fp8.quantize_rows
  const float s = a > 0.f ? a * (1.f / FP8_MAX) : 1.f;
  const float inv = __fdiv_rn(1.f, s);
  if (threadIdx.x == 0) scale[m] = s;
  unsigned char* qr = q + (size_t)m * ldq;
  for (int k = threadIdx.x * 8; k < K; k += Q_THREADS * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(row + k), f);
    uint2 o;
    o.x = pack4_fp8(f[0] * inv, f[1] * inv, f[2] * inv, f[3] * inv);
    o.y = pack4_fp8(f[4] * inv, f[5] * inv, f[6] * inv, f[7] * inv);
    *reinterpret_cast<uint2*>(qr + k) = o;
  }
}

// ----------------------------------------------------------------------------- prefill tile
constexpr int BM = 128, BN = 128, BKB = 128;  // BKB: K bytes (= fp8 elements) per step
constexpr int TILE_THREADS = 256;
constexpr int STAGE_BYTES = (BM + BN) * BKB;
constexpr int EPI_LD = BN + 4;
constexpr int EPI_BYTES = BM * EPI_LD * 4;
constexpr int TILE_LDS = (2 * STAGE_BYTES > EPI_BYTES) ? 2 * STAGE_BYTES : EPI_BYTES;
constexpr int GROUP_M = 8;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void stage_tile8(const unsigned char* __restrict__ g, int ld, int row0, int rows_valid,
                                            int k0, char* lds_tile, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid * 4 + i;
    const int r = q * 8 + (lane >> 3);
    const int c = swz(r, lane & 7);
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    glds16(g + (size_t)gr * ld + k0 + c * 16, lds_tile + q * 1024);
  }
}

// lane (fr, fh) holds A[row fr][k = 32 fh + j], j = 0..31: chunks 2fh, 2fh+1 of the 128-B row
__device__ __forceinline__ i32x8 frag8(const char* tile, int R, int fh) {
  const u32x4 lo = *reinterpret_cast<const u32x4*>(tile + R * 128 + 16 * swz(R, 2 * fh));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(tile + R * 128 + 16 * swz(R, 2 * fh + 1));
  return (i32x8){(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(TILE_THREADS, 2) void gemm_fp8_tile_kernel(
    const unsigned char* __restrict__ A, int lda, const float* __restrict__ sa, const unsigned char* __restrict__ B,
    int ldb, const float* __restrict__ sb, void* C, int ldc, const bf16_t* __restrict__ bias, const bf16_t* resid,
    int ldr, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[TILE_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int logical = xcd_remap(blockIdx.x, nwg);
  const int group = logical / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gm = min(tiles_m - first_m, GROUP_M);
  const int in_group = logical % (GROUP_M * tiles_n);
  const int tm = first_m + in_group % gm;
  const int tn = in_group / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / BKB;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  stage_tile8(A, lda, m0, M, 0, smem, wid_u, lane);
  stage_tile8(B, ldb, n0, N, 0, smem + BM * BKB, wid_u, lane);
  wait_vmcnt0();
  __syncthreads();

  const int fr = lane & 15, fh = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
      stage_tile8(A, lda, m0, M, (kt + 1) * BKB, nxt, wid_u, lane);
      stage_tile8(B, ldb, n0, N, (kt + 1) * BKB, nxt + BM * BKB, wid_u, lane);
    }
    const char* ta = smem + cur * STAGE_BYTES;
    const char* tb = ta + BM * BKB;
    i32x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag8(ta, wr * 64 + 16 * i + fr, fh);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag8(tb, wc * 64 + 16 * j + fr, fh);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    wait_vmcnt0();
    __syncthreads();
  }

  // ---- epilogue: dequant scales -> padded f32 LDS tile -> fused epilogue -> 16-B stores
  float* sC = reinterpret_cast<float*>(smem);
  float scb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) scb[j] = sb[min(n0 + wc * 64 + 16 * j + fr, N - 1)];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wr * 64 + 16 * i + 4 * fh + r;
      const float s = sa[min(m0 + row, M - 1)];
#pragma unroll
      for (int j = 0; j < 4; ++j) sC[row * EPI_LD + wc * 64 + 16 * j + fr] = acc[i][j][r] * s * scb[j];
    }
  __syncthreads();

  if constexpr (EPI == EPI_SILU_MUL) {
    const int ocol0 = tn * 64;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int v = tid + it * TILE_THREADS;
      const int row = v >> 3, c8 = (v & 7) * 8;
      const int gr = m0 + row;
      if (gr < M) {
        float o[8];
        const float* g = sC + row * EPI_LD + c8;
        const float* u = g + 64;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
        *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + ocol0 + c8) = pack8(o);
      }
    }
  } else {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int v = tid + it * TILE_THREADS;
      const int row = v >> 4, c8 = (v & 15) * 8;
      const int gr = m0 + row, gc = n0 + c8;
      if (gr < M && gc < N) {
        float o[8];
        const float* s = sC + row * EPI_LD + c8;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = s[e];
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH) {
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
          *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + gc) = pack8(o);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------- decode
constexpr int DW = 8;  // waves per block, split K

// 8 fp8 (one uint2) -> 8 bf16, exact (every e4m3 value is a bf16 value): v_cvt_pk_f32_fp8 to
// f32 pairs, then the upper halves packed with one v_perm per pair.
__device__ __forceinline__ unsigned f32pair_to_bf16x2(f32x2 f) {
  return __builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u);
}

__device__ __forceinline__ bf16x8 fp8x8_to_bf16(uint2 w) {
  u32x4 r;
  r[0] = f32pair_to_bf16x2(__builtin_amdgcn_cvt_pk_f32_fp8((int)w.x, false));
  r[1] = f32pair_to_bf16x2(__builtin_amdgcn_cvt_pk_f32_fp8((int)w.x, true));
  r[2] = f32pair_to_bf16x2(__builtin_amdgcn_cvt_pk_f32_fp8((int)w.y, false));
  r[3] = f32pair_to_bf16x2(__builtin_amdgcn_cvt_pk_f32_fp8((int)w.y, true));
  return __builtin_bit_cast(bf16x8, r);
}

// Block = DW waves on one 16-column output tile; waves take interleaved 128-deep K blocks.
// Inside a K block lane group fh owns k in [32 fh, 32 fh + 32) (its 32 weight bytes are
// contiguous: two 16-B loads); MFMA s consumes k = 32 fh + 8 s + j on both operands.
template <int MT, int EPI, bool OUT_F32>
__global__ __launch_bounds__(DW * 64) void gemm_fp8_dec_kernel(const bf16_t* __restrict__ X, int ldx,
                                                               const unsigned char* __restrict__ W, int ldw,
                                                               const float* __restrict__ sw, void* C, int ldc,
                                                               const bf16_t* __restrict__ bias, const bf16_t* resid,
                                                               int ldr, int M, int N, int K) {
  constexpr bool PAIR = (EPI == EPI_SILU_MUL);
  constexpr int NACC = PAIR ? 2 : 1;
  __shared__ __attribute__((aligned(16))) f32x4 red[DW][NACC * MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fh = lane >> 4;
  const int n0 = blockIdx.x * 16;
  int wrow0, wrow1 = 0;
  if constexpr (PAIR) {
    const int g = n0 + fr;
    wrow0 = (g >> 6) * 128 + (g & 63);
    wrow1 = wrow0 + 64;
  } else {
    wrow0 = min(n0 + fr, N - 1);
  }
  const unsigned char* w0 = W + (size_t)wrow0 * ldw + 32 * fh;
  const unsigned char* w1 = W + (size_t)wrow1 * ldw + 32 * fh;
  const bf16_t* xr[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xr[t] = X + (size_t)min(t * 16 + fr, M - 1) * ldx + 32 * fh;

  f32x4 acc[NACC][MT];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[a][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nkb = K >> 7;
  for (int kb = wid; kb < nkb; kb += DW) {
    const int k = kb * 128;
    uint2 wv[NACC][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w0 + k + 16 * h));
      wv[0][2 * h] = make_uint2(a[0], a[1]);
      wv[0][2 * h + 1] = make_uint2(a[2], a[3]);
      if constexpr (PAIR) {
        const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w1 + k + 16 * h));
        wv[1][2 * h] = make_uint2(b[0], b[1]);
        wv[1][2 * h + 1] = make_uint2(b[2], b[3]);
      }
    }
    bf16x8 xf[MT][4];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(xr[t] + k + 8 * s);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 wf[NACC];
#pragma unroll
      for (int a = 0; a < NACC; ++a) wf[a] = fp8x8_to_bf16(wv[a][s]);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int a = 0; a < NACC; ++a)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[t][s], wf[a], acc[a][t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) red[wid][a * MT + t][lane] = acc[a][t];
  __syncthreads();

  for (int e = threadIdx.x; e < MT * 64 * 4; e += DW * 64) {
    const int t = e >> 8, ln = (e >> 2) & 63, r = e & 3;
    const int row = t * 16 + 4 * (ln >> 4) + r;
    const int col = n0 + (ln & 15);
    if (row >= M || col >= N) continue;
    float v = 0.f, u = 0.f;
#pragma unroll
    for (int w = 0; w < DW; ++w) {
      v += red[w][t][ln][r];
      if constexpr (PAIR) u += red[w][MT + t][ln][r];
    }
    if constexpr (PAIR) {
      const int g = col;
      const int pr = (g >> 6) * 128 + (g & 63);
      v = silu(v * sw[pr]) * (u * sw[pr + 64]);
    } else {
      v *= sw[col];
    }
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH)
      v += bf2f(bias[col]);
    if constexpr (EPI == EPI_RESID || EPI == EPI_BIAS_RESID) v += bf2f(resid[(size_t)row * ldr + col]);
    if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) v = gelu_erf(v);
    if constexpr (EPI == EPI_BIAS_GELU_TANH) v = gelu_tanh(v);
    if constexpr (OUT_F32)
      reinterpret_cast<float*>(C)[(size_t)row * ldc + col] = v;
    else
      reinterpret_cast<bf16_t*>(C)[(size_t)row * ldc + col] = f2bf(v);
  }
}

template <int EPI, bool F32>
hipError_t launch_tile8(const void* A, int lda, const float* sa, const void* B, int ldb, const float* sb, void* C,
                        int ldc, const void* bias, const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_fp8_tile_kernel<EPI, F32>), dim3(tiles), dim3(TILE_THREADS), 0, st,
                     (const unsigned char*)A, lda, sa, (const unsigned char*)B, ldb, sb, C, ldc, (const bf16_t*)bias,
                     (const bf16_t*)resid, ldr, M, N, K);
  return hipGetLastError();
}

template <int MT, int EPI, bool F32>
hipError_t launch_dec8(const void* X, int ldx, const void* W, int ldw, const float* sw, void* C, int ldc,
                       const void* bias, const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL((gemm_fp8_dec_kernel<MT, EPI, F32>), dim3((N + 15) / 16), dim3(DW * 64), 0, st,
                     (const bf16_t*)X, ldx, (const unsigned char*)W, ldw, sw, C, ldc, (const bf16_t*)bias,
                     (const bf16_t*)resid, ldr, M, N, K);
  return hipGetLastError();
}

template <int EPI, bool F32>
hipError_t dispatch_dec8(const void* X, int ldx, const void* W, int ldw, const float* sw, void* C, int ldc,
                         const void* bias, const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  switch ((M + 15) / 16) {
    case 1: return launch_dec8<1, EPI, F32>(X, ldx, W, ldw, sw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 2: return launch_dec8<2, EPI, F32>(X, ldx, W, ldw, sw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 3: return launch_dec8<3, EPI, F32>(X, ldx, W, ldw, sw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 4: return launch_dec8<4, EPI, F32>(X, ldx, W, ldw, sw, C, ldc, bias, resid, ldr, M, N, K, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

RAGK_API int ragk_quant_fp8_rows(const void* x, int ldx, void* q, int ldq, float* scale, int M, int K,
                                 hipStream_t st) {
  if (M <= 0) return 0;
  if (K % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(quant_rows_kernel, dim3(M), dim3(Q_THREADS), 0, st, (const bf16_t*)x, ldx, (unsigned char*)q, ldq,
                     scale, K);
  return (int)hipGetLastError();
}

// Prefill W8A8: C = epi((A8 * sa) . (B8 * sb)^T); A8 [M,K] fp8 (row scale sa), B8 [N or 2N,K] fp8 (row scale sb).
// Decode W8A16 (M <= 64, x_bf16 != null): C = epi(x . (B8 * sb)^T); A8/sa ignored.
// N = output columns; for EPI_SILU_MUL the weight has 2N rows in the packed [64 gate | 64 up] tile layout.
RAGK_API int ragk_gemm_fp8(const void* x_bf16, int ldx, const void* A8, int lda, const float* sa, const void* B8,
                           int ldb, const float* sb, void* C, int ldc, const void* bias, const void* resid, int ldr,
                           int M, int N, int K, int epi, int out_f32, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % 128) return (int)hipErrorInvalidValue;
  const bool dec = x_bf16 != nullptr;
  if (dec && M > 64) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL) {
    if (N % 64 || out_f32) return (int)hipErrorInvalidValue;
    return dec ? (int)dispatch_dec8<EPI_SILU_MUL, false>(x_bf16, ldx, B8, ldb, sb, C, ldc, bias, resid, ldr, M, N, K,
                                                         st)
               : (int)launch_tile8<EPI_SILU_MUL, false>(A8, lda, sa, B8, ldb, sb, C, ldc, bias, resid, ldr, M, 2 * N,
                                                        K, st);
  }
  if (!dec && N % 8) return (int)hipErrorInvalidValue;
#define RAGK_FP8_CASE(E)                                                                                          \
  case E:                                                                                                         \
    if (dec)                                                                                                      \
      return out_f32 ? (int)dispatch_dec8<E, true>(x_bf16, ldx, B8, ldb, sb, C, ldc, bias, resid, ldr, M, N, K, st) \
                     : (int)dispatch_dec8<E, false>(x_bf16, ldx, B8, ldb, sb, C, ldc, bias, resid, ldr, M, N, K, st); \
    return out_f32 ? (int)launch_tile8<E, true>(A8, lda, sa, B8, ldb, sb, C, ldc, bias, resid, ldr, M, N, K, st)   \
                   : (int)launch_tile8<E, false>(A8, lda, sa, B8, ldb, sb, C, ldc, bias, resid, ldr, M, N, K, st);
  switch (epi) {
    RAGK_FP8_CASE(EPI_NONE)
    RAGK_FP8_CASE(EPI_BIAS)
    RAGK_FP8_CASE(EPI_RESID)
    RAGK_FP8_CASE(EPI_BIAS_RESID)
    RAGK_FP8_CASE(EPI_BIAS_GELU)
    RAGK_FP8_CASE(EPI_GELU)
    RAGK_FP8_CASE(EPI_BIAS_GELU_TANH)
    default: return (int)hipErrorInvalidValue;
  }
#undef RAGK_FP8_CASE
}
