// bf16 GEMM family for gfx950: C[M,N] = A[M,K] . B[N,K]^T  (+ fused epilogue)
//
// B is the HF weight layout [out_features, in_features], so both operands are
// K-contiguous and every MFMA fragment is one 16-byte load.
//
// Two kernels:
//  * gemm_tile   : prefill / encoder GEMMs (M >= 64). 128x128x64 block tile,
//                  4 waves (2x2) of 64x64, mfma_f32_16x16x32_bf16, operands
//                  staged global->LDS with global_load_lds (16 B/lane), XOR
//                  swizzled rows (conflict-free ds_read_b128), double-buffered,
//                  XCD-aware grouped tile order, LDS-staged vectorised epilogue
//                  (bias / residual / GELU / SiLU*up fused).
//  * gemm_skinny : decode GEMMs (M <= 64). Weight-streaming: every weight byte is
//                  read exactly once straight into VGPRs (no LDS round trip), 8
//                  waves per block split K, MFMA with the activations as the A
//                  operand, cross-wave reduction through LDS, fused epilogue.
//
// Replaces reference ops K3/K7/K8/K9/K10/K11 (the reference
// runs them as fp32 ATen CPU matmuls inside transformers' LlamaForCausalLM,
// /root/reference/llm/rag.py:24,172) and encoder ops E2/E4/E5/E6.
#include <stdlib.h>

#include "common.h"
using namespace ragk;

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_THREADS = 256;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;         // one buffer: A + B = 32 KiB
constexpr int EPI_LD = BN + 4;                          // padded f32 row (conflict-free C-layout writes)
constexpr int EPI_BYTES = BM * EPI_LD * 4;              // 67,584 B
constexpr int TILE_LDS = (2 * STAGE_BYTES > EPI_BYTES) ? 2 * STAGE_BYTES : EPI_BYTES;
constexpr int GROUP_M = 8;

// 128-byte LDS rows (64 bf16): 8 x 16-B chunks. XOR the chunk with (row>>1)&7 so the
// 16 lanes of each ds_read_b128 lane-group land on 16 distinct 16-B bank slots.
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, int ld, int row0, int rows_valid,
                                           int k0, char* lds_tile, int wid, int lane) {
  // 128 rows x 128 B = 16 x 1 KiB glds pieces, 4 per wave. Lane-linear LDS
  // destination; the swizzle is applied to the per-lane SOURCE address.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid * 4 + i;
    const int r = q * 8 + (lane >> 3);
    const int p = lane & 7;
    const int c = swz(r, p);
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;  // clamp: rows past the edge are never stored
    const bf16_t* src = g + (size_t)gr * ld + k0 + c * 8;
    glds16(src, lds_tile + q * 1024);
  }
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(TILE_THREADS, 2) void gemm_tile_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ B, int ldb, void* C, int ldc,
    const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr, int M, int N, int K) {
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

  const int nk = K / BK;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  stage_tile(A, lda, m0, M, 0, smem, wid_u, lane);
  stage_tile(B, ldb, n0, N, 0, smem + BM * BK * 2, wid_u, lane);
  wait_vmcnt0();
  __syncthreads();

  const int fr = lane & 15, fh = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
      stage_tile(A, lda, m0, M, (kt + 1) * BK, nxt, wid_u, lane);
      stage_tile(B, ldb, n0, N, (kt + 1) * BK, nxt + BM * BK * 2, wid_u, lane);
    }
    const char* sa = smem + cur * STAGE_BYTES;
    const char* sb = sa + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
      const int c = 4 * s + fh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int R = wr * 64 + 16 * i + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + R * 128 + 16 * swz(R, c));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int R = wc * 64 + 16 * j + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + R * 128 + 16 * swz(R, c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // ---- epilogue: accumulators -> padded f32 LDS tile -> 16-B row stores ----
  float* sC = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[(wr * 64 + 16 * i + 4 * fh + r) * EPI_LD + wc * 64 + 16 * j + fr] = acc[i][j][r];
  __syncthreads();

  if constexpr (EPI == EPI_SILU_MUL) {
    // packed tile = [64 gate cols | 64 up cols] -> 64 output cols
    const int ocol0 = tn * 64;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int v = tid + it * TILE_THREADS;  // 128 rows x 8 vec
      const int row = v >> 3, c8 = (v & 7) * 8;
      const int gr = m0 + row;
      if (gr < M) {
        float o[8];
        const float* g = sC + row * EPI_LD + c8;
        const float* u = g + 64;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
        bf16_t* dst = reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + ocol0 + c8;
        *reinterpret_cast<u32x4*>(dst) = pack8(o);
      }
    }
  } else {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int v = tid + it * TILE_THREADS;  // 128 rows x 16 vec
      const int row = v >> 4, c8 = (v & 15) * 8;
      const int gr = m0 + row, gc = n0 + c8;
      if (gr < M && gc < N) {
        float o[8];
        const float* s = sC + row * EPI_LD + c8;
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

// ------------------------------------------------------------------------------------
// Skinny (decode) GEMM. Block = WAVES waves handling one 16-column output tile; the
// waves take interleaved 128-deep K blocks (4 MFMA k-steps each), so the block
// streams each of its 16 weight rows front-to-back exactly once.
// ------------------------------------------------------------------------------------
constexpr int SK_WAVES = 8;

// (16 waves per block measured slower on the batch-1 down projection: more waves lengthen the LDS
// reduction and the per-block tail more than the extra loads in flight gain; two K blocks in flight per
// wave and non-temporal weight loads were slower at C=1 too -- profiles/c1_skinny_*_ab_r4.log.)
template <int MT, int EPI, bool OUT_F32>
__global__ __launch_bounds__(SK_WAVES * 64) void gemm_skinny_kernel(
    const bf16_t* __restrict__ X, int ldx, const bf16_t* __restrict__ W, int ldw, void* C, int ldc,
    const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr, int M, int N, int K) {
  constexpr int WV = SK_WAVES;
  constexpr bool PAIR = (EPI == EPI_SILU_MUL);
  constexpr int NACC = PAIR ? 2 : 1;
  __shared__ __attribute__((aligned(16))) f32x4 red[WV][NACC * MT][64];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fh = lane >> 4;
  const int n0 = blockIdx.x * 16;
  // weight rows for this lane's output column (packed gate/up layout for SILU_MUL:
  // 128-row tiles = [64 gate | 64 up])
  int wrow0, wrow1 = 0;
  if constexpr (PAIR) {
    const int g = n0 + fr;
    wrow0 = (g >> 6) * 128 + (g & 63);
    wrow1 = wrow0 + 64;
  } else {
    wrow0 = min(n0 + fr, N - 1);
  }
  const bf16_t* w0 = W + (size_t)wrow0 * ldw + fh * 8;
  const bf16_t* w1 = W + (size_t)wrow1 * ldw + fh * 8;
  const bf16_t* xr[MT];
  bool xv[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + fr;
    xv[t] = m < M;
    xr[t] = X + (size_t)(xv[t] ? m : 0) * ldx + fh * 8;
  }

  f32x4 acc[NACC][MT];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[a][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nkb = K >> 7;  // 128-deep K blocks
  const bf16x8 zero = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int U = 1;  // K blocks per wave per iteration (default cache policy for the weights)
  for (int kb = wid; kb < nkb; kb += U * WV) {
    bf16x8 wf[U][NACC][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kb + u * WV, nkb - 1) * 128;  // clamped: a missing second block is loaded, not used
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        wf[u][0][s] = *reinterpret_cast<const bf16x8*>(w0 + k + 32 * s);
        if constexpr (PAIR) wf[u][1][s] = *reinterpret_cast<const bf16x8*>(w1 + k + 32 * s);
      }
    }
    bf16x8 xf[U][MT][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kb + u * WV, nkb - 1) * 128;
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          xf[u][t][s] = xv[t] ? *reinterpret_cast<const bf16x8*>(xr[t] + k + 32 * s) : zero;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kb + u * WV >= nkb) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int a = 0; a < NACC; ++a)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[u][t][s], wf[u][a][s], acc[a][t], 0, 0, 0);
    }
  }

#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) red[wid][a * MT + t][lane] = acc[a][t];
  __syncthreads();

  // reduce over waves; element e = (t, lane, r): row = 16t + 4*(lane>>4) + r, col = n0 + (lane&15)
  for (int e = threadIdx.x; e < MT * 64 * 4; e += WV * 64) {
    const int t = e >> 8, ln = (e >> 2) & 63, r = e & 3;
    const int row = t * 16 + 4 * (ln >> 4) + r;
    const int col = n0 + (ln & 15);
    if (row >= M || col >= N) continue;
    float v = 0.f, u = 0.f;
#pragma unroll
    for (int w = 0; w < WV; ++w) {
      v += red[w][t][ln][r];
      if constexpr (PAIR) u += red[w][MT + t][ln][r];
    }
    if constexpr (PAIR) v = silu(v) * u;
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU ||
                  EPI == EPI_BIAS_GELU_TANH)
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

// ------------------------------------------------------------------------------------
// Pipelined weight-streaming GEMV/GEMM for decode (M <= 64), v2.
//  * software pipeline: the next 128-deep K block's weights + activations are loaded into a
//    second register set while the MFMAs of the current one run (the v1 loop was latency-bound:
//    load -> wait -> 4 MFMAs, ~4 iterations per wave);
//  * weights are streamed with non-temporal loads (read exactly once);
//  * NT n-tiles per wave reuse each activation fragment NT times (cuts the L2 activation
//    traffic that dominated at M = 32..64);
//  * rows >= M read a clamped (valid) row: their outputs are garbage but never stored, so no
//    per-element select sits between a load and its MFMA.
// ------------------------------------------------------------------------------------
template <int MT, int NT, int NACC>
struct GemvFrags {
  bf16x8 w[NACC][NT][4];
  bf16x8 x[MT][4];
};

template <int MT, int NT, int EPI, bool OUT_F32>
__global__ __launch_bounds__(SK_WAVES * 64) void gemm_gemv_kernel(
    const bf16_t* __restrict__ X, int ldx, const bf16_t* __restrict__ W, int ldw, void* C, int ldc,
    const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr, int M, int N, int K) {
  constexpr bool PAIR = (EPI == EPI_SILU_MUL);
  constexpr int NACC = PAIR ? 2 : 1;
  __shared__ __attribute__((aligned(16))) f32x4 red[SK_WAVES][NACC * NT * MT][64];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fh = lane >> 4;
  const int nbase = blockIdx.x * 16 * NT;
  const bf16_t* wp[NACC][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = nbase + 16 * j + fr;
    if constexpr (PAIR) {
      const int r0 = (col >> 6) * 128 + (col & 63);
      wp[0][j] = W + (size_t)r0 * ldw + fh * 8;
      wp[1][j] = W + (size_t)(r0 + 64) * ldw + fh * 8;
    } else {
      wp[0][j] = W + (size_t)min(col, N - 1) * ldw + fh * 8;
    }
  }
  const bf16_t* xp[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xp[t] = X + (size_t)min(t * 16 + fr, M - 1) * ldx + fh * 8;

  f32x4 acc[NACC][NT][MT];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[a][j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto load = [&](GemvFrags<MT, NT, NACC>& f, int kb) {
    const int k = kb * 128;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          f.w[a][j][s] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp[a][j] + k + 32 * s));
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) f.x[t][s] = *reinterpret_cast<const bf16x8*>(xp[t] + k + 32 * s);
  };
  auto compute = [&](const GemvFrags<MT, NT, NACC>& f) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int a = 0; a < NACC; ++a)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[a][j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.x[t][s], f.w[a][j][s], acc[a][j][t], 0, 0, 0);
  };

  const int nkb = K >> 7;
  GemvFrags<MT, NT, NACC> fa, fb;
  int kb = wid;
  if (kb < nkb) load(fa, kb);
  for (; kb < nkb; kb += 2 * SK_WAVES) {
    const int kb2 = kb + SK_WAVES;
    if (kb2 < nkb) load(fb, kb2);
    compute(fa);
    const int kb3 = kb2 + SK_WAVES;
    if (kb3 < nkb) load(fa, kb3);
    if (kb2 < nkb) compute(fb);
  }

#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t) red[wid][(a * NT + j) * MT + t][lane] = acc[a][j][t];
  __syncthreads();

  // element e = (j, t, lane, r): row = 16t + 4*(lane>>4) + r, col = nbase + 16j + (lane&15)
  for (int e = threadIdx.x; e < NT * MT * 64 * 4; e += SK_WAVES * 64) {
    const int j = e / (MT * 256), rem = e % (MT * 256);
    const int t = rem >> 8, ln = (rem >> 2) & 63, r = rem & 3;
    const int row = t * 16 + 4 * (ln >> 4) + r;
    const int col = nbase + 16 * j + (ln & 15);
    if (row >= M || col >= N) continue;
    float v = 0.f, u = 0.f;
#pragma unroll
    for (int w = 0; w < SK_WAVES; ++w) {
      v += red[w][j * MT + t][ln][r];
      if constexpr (PAIR) u += red[w][(NT + j) * MT + t][ln][r];
    }
    if constexpr (PAIR) v = silu(v) * u;
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

template <int MT, int NT, int EPI, bool F32>
hipError_t launch_gemv(const void* X, int ldx, const void* W, int ldw, void* C, int ldc, const void* bias,
                       const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL((gemm_gemv_kernel<MT, NT, EPI, F32>), dim3((N + 16 * NT - 1) / (16 * NT)), dim3(SK_WAVES * 64),
                     0, st, (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, C, ldc, (const bf16_t*)bias,
                     (const bf16_t*)resid, ldr, M, N, K);
  return hipGetLastError();
}

// NT=2 when it still leaves >= 2 blocks per CU (and PAIR needs N % 32 for whole tiles)
template <int EPI, bool F32>
hipError_t dispatch_gemv(const void* X, int ldx, const void* W, int ldw, void* C, int ldc, const void* bias,
                         const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  const int mt = (M + 15) / 16;
  const bool nt2 = M > 16 && N >= 32 * 512 && (EPI != EPI_SILU_MUL || N % 32 == 0);
#define RAGK_GV(MTV)                                                                                         \
  case MTV:                                                                                                  \
    if (nt2 && MTV <= 2)                                                                                     \
      return launch_gemv<MTV, (MTV <= 2 ? 2 : 1), EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st); \
    return launch_gemv<MTV, 1, EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st);
  switch (mt) {
    RAGK_GV(1)
    RAGK_GV(2)
    RAGK_GV(3)
    RAGK_GV(4)
    default: return hipErrorInvalidValue;
  }
#undef RAGK_GV
}

template <int EPI, bool F32>
hipError_t launch_tile(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                       const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_tile_kernel<EPI, F32>), dim3(nwg), dim3(TILE_THREADS), 0, st,
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias,
                     (const bf16_t*)resid, ldr, M, N, K);
  return hipGetLastError();
}

template <int MT, int EPI, bool F32>
hipError_t launch_skinny(const void* X, int ldx, const void* W, int ldw, void* C, int ldc, const void* bias,
                         const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, EPI, F32>), dim3((N + 15) / 16), dim3(SK_WAVES * 64), 0, st,
                     (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, C, ldc, (const bf16_t*)bias,
                     (const bf16_t*)resid, ldr, M, N, K);
  return hipGetLastError();
}

template <int EPI, bool F32>
hipError_t dispatch_skinny(const void* X, int ldx, const void* W, int ldw, void* C, int ldc, const void* bias,
                           const void* resid, int ldr, int M, int N, int K, hipStream_t st) {
  const int mt = (M + 15) / 16;
  switch (mt) {
    case 1: return launch_skinny<1, EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 2: return launch_skinny<2, EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 3: return launch_skinny<3, EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st);
    case 4: return launch_skinny<4, EPI, F32>(X, ldx, W, ldw, C, ldc, bias, resid, ldr, M, N, K, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// N here is the number of OUTPUT columns. For EPI_SILU_MUL the weight has 2*N rows
// in the packed [64 gate | 64 up] tile layout and N must be a multiple of 64.
RAGK_API int ragk_gemm(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                       const void* resid, int ldr, int M, int N, int K, int epi, int out_f32, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % 128 != 0) return (int)hipErrorInvalidValue;
  const bool skinny = M <= 64;
  if (epi == EPI_SILU_MUL) {
    if (N % 64 != 0 || out_f32) return (int)hipErrorInvalidValue;
    if (skinny) return (int)dispatch_skinny<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
    return (int)launch_tile<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, 2 * N, K, st);
  }
  if (!skinny && N % 8 != 0) return (int)hipErrorInvalidValue;
#define RAGK_GEMM_CASE(E)                                                                               \
  case E:                                                                                               \
    if (skinny)                                                                                         \
      return out_f32 ? (int)dispatch_skinny<E, true>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st) \
                     : (int)dispatch_skinny<E, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st); \
    return out_f32 ? (int)launch_tile<E, true>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st)     \
                   : (int)launch_tile<E, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
  switch (epi) {
    RAGK_GEMM_CASE(EPI_NONE)
    RAGK_GEMM_CASE(EPI_BIAS)
    RAGK_GEMM_CASE(EPI_RESID)
    RAGK_GEMM_CASE(EPI_BIAS_RESID)
    RAGK_GEMM_CASE(EPI_BIAS_GELU)
    RAGK_GEMM_CASE(EPI_GELU)
    RAGK_GEMM_CASE(EPI_BIAS_GELU_TANH)
    default: return (int)hipErrorInvalidValue;
  }
#undef RAGK_GEMM_CASE
}

// Force a specific path (tests / benchmarks): path 0 = tile, 1 = skinny v1, 3 = pipelined gemv v2.
RAGK_API int ragk_gemm_path(int path, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                            const void* bias, const void* resid, int ldr, int M, int N, int K, int epi,
                            hipStream_t st) {
  if (K % 128 != 0) return (int)hipErrorInvalidValue;
  if (path == 1 || path == 3) {
    if (M > 64) return (int)hipErrorInvalidValue;
    if (path == 3) {
      if (epi == EPI_SILU_MUL) return (int)dispatch_gemv<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
      if (epi == EPI_NONE) return (int)dispatch_gemv<EPI_NONE, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
      if (epi == EPI_RESID) return (int)dispatch_gemv<EPI_RESID, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
      return (int)hipErrorInvalidValue;
    }
    if (epi == EPI_SILU_MUL) return (int)dispatch_skinny<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
    if (epi == EPI_NONE) return (int)dispatch_skinny<EPI_NONE, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
    if (epi == EPI_RESID) return (int)dispatch_skinny<EPI_RESID, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
    return (int)hipErrorInvalidValue;
  }
  if (epi == EPI_SILU_MUL) return (int)launch_tile<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, 2 * N, K, st);
  if (epi == EPI_NONE) return (int)launch_tile<EPI_NONE, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
  if (epi == EPI_RESID) return (int)launch_tile<EPI_RESID, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
  return (int)hipErrorInvalidValue;
}
