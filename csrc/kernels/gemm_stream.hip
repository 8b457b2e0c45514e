// Decode GEMM v4 ("stream") for gfx950: M <= 64 activation rows, weights streamed from HBM
// through a multi-stage global_load_lds ring. Serves bf16 and fp8 (e4m3fn, per-row scale) weights.
//
// Why: at decode batch 32 the register-streaming kernels (gemm.hip skinny, gemm_fp8 dec) reach
// only 2-3.4 TB/s -- every 16-column block re-reads the whole activation block from L2 and each
// wave keeps just one or two K-blocks of loads in flight. Here
//   * block = 4 waves x 32 columns = 128 weight rows; the activation tile (16*MT rows) is staged
//     ONCE per block per K-step and shared by all 128 rows;
//   * both operands go global -> LDS with global_load_lds (no VGPRs held by loads in flight), in
//     an NS-stage ring (NS-1 K-steps in flight per block: ~64-80 KB per CU), XOR-swizzled rows;
//   * one raw s_barrier per K-step (explicit vmcnt/lgkmcnt; no __syncthreads so the compiler
//     never drains the ring);
//   * K is split S ways across grid.y when N alone cannot fill 256 CUs (fp32 slabs + atomic
//     ticket; the last-arriving block reduces and runs the epilogue -- agent-scope release /
//     acquire, any block->XCD placement);
//   * fp8 weights (W8A16): the tile holds 128 fp8 k per 128-byte row; fragments are converted
//     exactly to bf16 in registers; per-row scales applied in the epilogue.
// Epilogues: none / bias / resid / bias_resid / gelu variants / SiLU*up on the packed
// [64 gate | 64 up] 128-row weight tiles (same layout as every other GEMM here).
#include <stdlib.h>

#include "common.h"
using namespace ragk;

namespace {

constexpr int ST_THREADS = 256;
constexpr int WROWS = 128;  // weight rows per block
#ifndef STREAM_LDS_KB
#define STREAM_LDS_KB 150
#endif

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

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

template <int MT, bool FP8, int ROWS = WROWS>
struct StreamGeom {
  static constexpr int KSTEP = FP8 ? 128 : 64;      // k elements per pipeline step
  static constexpr int XROW = 2 * KSTEP;            // activation row bytes per step (bf16)
  static constexpr int XROWS = 16 * MT;
  static constexpr int WBYTES = ROWS * 128;         // ROWS rows x 128 B
  static constexpr int XBYTES = XROWS * XROW;       // MT x 2 KB (bf16) or MT x 4 KB (fp8 case)
  static constexpr int STAGE = WBYTES + XBYTES;
  // ring depth: as many stages as ~STREAM_LDS_KB of LDS per CU allow (NS - 1 K-steps of weights in
  // flight; a pure streaming read needs ~128 KB in flight per CU for 5.7 TB/s, tools/read_roofline.py).
  // 64-row tiles run two blocks per CU, each with half the LDS.
  static constexpr int BPC = ROWS == 64 ? 2 : 1;
  static constexpr int NS_CAP = STREAM_LDS_KB * 1024 / BPC / STAGE;
  static constexpr int NS = NS_CAP >= 8 ? 8 : (NS_CAP < 4 ? 4 : NS_CAP);
  static constexpr int XPIECES = XBYTES / 1024;     // 1 KB glds pieces (64 lanes x 16 B)
  static constexpr int XP = (XPIECES + 3) / 4;      // per wave (duplicates pad the last round)
  static constexpr int WPW = ROWS / 32;             // weight pieces (8 rows) per wave per stage
  static constexpr int LOADS = WPW + XP;            // glds per wave per stage
  static constexpr int EPI_LD = ROWS + 4;
  static constexpr int J = ROWS / 64;               // 16-row weight fragments per wave
};

// Packed weight row of local tile row r. The SiLU*up weights are packed [64 gate | 64 up] per 128
// rows; a 64-row tile of a pair GEMM takes gate rows h*32..h*32+31 and the matching up rows of
// group g (tile = 2g + h), so every tile still holds whole (gate, up) pairs.
template <int ROWS, bool PAIR>
__device__ __forceinline__ int stream_row(int tile, int r) {
  if constexpr (ROWS == 64 && PAIR) {
    const int g = tile >> 1, h = tile & 1;
    return g * 128 + (r < 32 ? h * 32 + r : 64 + h * 32 + (r - 32));
  } else {
    return tile * ROWS + r;
  }
}

// Weight-stream LDS-DMA with the non-temporal policy (aux = 2): each weight row is read by exactly
// one block once per decode step, from a stream far larger than the Infinity Cache.
__device__ __forceinline__ void glds16_nt(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 2);
}

template <int MT, bool FP8, bool NT, int ROWS, bool PAIR, bool NOX = false>
__device__ __forceinline__ void stage_load(const bf16_t* __restrict__ X, int ldx, int M,
                                           const unsigned char* __restrict__ Wb, int ldw_bytes, int Nrows, int tile,
                                           int kel, char* st, int wid, int lane) {
  using G = StreamGeom<MT, FP8, ROWS>;
  // weights: ROWS rows x 128 B; wave w issues pieces WPW*w .. WPW*w + WPW-1 (8 rows each)
  const size_t kbyte = FP8 ? (size_t)kel : (size_t)kel * 2;
#pragma unroll
  for (int i = 0; i < G::WPW; ++i) {
    const int q = wid * G::WPW + i;
    const int r = q * 8 + (lane >> 3);
    const int c = swz(r, lane & 7);
    const int gr = min(stream_row<ROWS, PAIR>(tile, r), Nrows - 1);
    if constexpr (NT) glds16_nt(Wb + (size_t)gr * ldw_bytes + kbyte + c * 16, st + q * 1024);
    else glds16(Wb + (size_t)gr * ldw_bytes + kbyte + c * 16, st + q * 1024);
  }
  // activations: XROWS rows x XROW bytes, as 128-B half-rows for the fp8 (256-B) case
  if constexpr (NOX) return;
  char* xs = st + G::WBYTES;
#pragma unroll
  for (int i = 0; i < G::XP; ++i) {
    const int q = (wid + 4 * i) % G::XPIECES;
    const int slot = q * 64 + lane;                 // 16-B slot index in the X tile
    int row, c, half;
    if constexpr (FP8) {  // 256-B rows: slot -> (half, row, chunk); sub-tile h = k in [64h, 64h+64)
      half = slot / (G::XROWS * 8);
      const int s2 = slot % (G::XROWS * 8);
      row = s2 >> 3;
      c = swz(row, s2 & 7);
    } else {
      half = 0;
      row = slot >> 3;
      c = swz(row, slot & 7);
    }
    const int gm = min(row, M - 1);
    glds16(X + (size_t)gm * ldx + kel + half * 64 + c * 8, xs + q * 1024);
  }
}

// SLAB: split-K partial mode for the decode consumers (add_partials_rmsnorm / rope_kv_partials / the
// decode attention's qkv staging): every block writes its fp32 partial tile to P[slice][row][col]
// ([S][M][N], gemm_part's layout) and exits -- no ticket, no in-kernel reduction (the release / acquire
// of the last-arriver form made the 8-way split down projection 56 us at batch 32; gemm_part's
// register-streaming blocks need 114 KB of LDS for its activation slice there and run in two rounds).
// DG = 1 (diagnostic, tools/stream_gemm_probe.py): the ring, its waits and barriers, no fragment reads or MFMA
// (results meaningless) -- how fast the weight stream itself runs in this kernel's structure. DG = 2: also
// no activation staging (weights only); DG = 3: as 2 without the per-stage barrier.
template <int MT, int EPI, bool OUT_F32, bool FP8, bool NT = false, int ROWS = WROWS, bool SLAB = false, int DG = 0>
__global__ __launch_bounds__(ST_THREADS, ROWS == 64 ? 2 : 1) void gemm_stream_kernel(
    const bf16_t* __restrict__ X, int ldx, const void* __restrict__ Wv, int ldw, const float* __restrict__ wscale,
    void* C, int ldc, const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr, int M, int N, int K, int S,
    float* ws, int* counters) {
  using G = StreamGeom<MT, FP8, ROWS>;
  constexpr bool PAIR = (EPI == EPI_SILU_MUL);
  constexpr int NS = G::NS, J = G::J;
  __shared__ __attribute__((aligned(16))) char smem[NS * G::STAGE + 16];  // one object: see trap (a)
  int& s_flag = *reinterpret_cast<int*>(smem + NS * G::STAGE);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int fr = lane & 15, fh = lane >> 4;
  const int ntile = blockIdx.x, slice = blockIdx.y, ntiles = gridDim.x;
  const int Nrows = PAIR ? 2 * N : N;
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(Wv);
  const int ldw_bytes = FP8 ? ldw : ldw * 2;
  const int steps_total = K / G::KSTEP;
  const int nst = steps_total / S;
  const int k0 = slice * nst * G::KSTEP;

  f32x4 acc[MT][J];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: NS-1 stages in flight
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nst)
      stage_load<MT, FP8, NT, ROWS, PAIR, (DG >= 2)>(X, ldx, M, Wb, ldw_bytes, Nrows, ntile, k0 + p * G::KSTEP,
                                          smem + p * G::STAGE, wid_u, lane);

  for (int t = 0; t < nst; ++t) {
    // stage t landed (this wave's part): at most the later stages' loads still outstanding
    const int ahead = min(nst - 1 - t, NS - 2);
    constexpr int LD = DG >= 2 ? G::WPW : G::LOADS;  // LDS-DMAs per wave per stage
    if (ahead >= NS - 2) wait_vm<(NS - 2) * LD>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (DG != 3) barrier_raw();  // every wave's part of stage t landed; every wave finished reading stage t-1
    if (t + NS - 1 < nst)
      stage_load<MT, FP8, NT, ROWS, PAIR, (DG >= 2)>(X, ldx, M, Wb, ldw_bytes, Nrows, ntile, k0 + (t + NS - 1) * G::KSTEP,
                                          smem + ((t + NS - 1) % NS) * G::STAGE, wid_u, lane);
    const char* wt = smem + (t % NS) * G::STAGE;
    const char* xt = wt + G::WBYTES;
    if constexpr (DG == 1) {
      continue;
    } else if constexpr (!FP8) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 4 * s + fh;
        bf16x8 wf[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int R = wid * (ROWS / 4) + 16 * j + fr;
          wf[j] = *reinterpret_cast<const bf16x8*>(wt + R * 128 + 16 * swz(R, c));
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int R = 16 * m + fr;
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xt + R * 128 + 16 * swz(R, c));
#pragma unroll
          for (int j = 0; j < J; ++j) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wf[j], acc[m][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {  // k = 32 s + 8 fh + j
        bf16x8 wf[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int R = wid * (ROWS / 4) + 16 * j + fr;
          const uint2 raw = *reinterpret_cast<const uint2*>(wt + R * 128 + 16 * swz(R, 2 * s + (fh >> 1)) +
                                                            8 * (fh & 1));
          wf[j] = fp8x8_to_bf16(raw);
        }
        const char* xh = xt + (s >> 1) * (G::XROWS * 128);
        const int c = 4 * (s & 1) + fh;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int R = 16 * m + fr;
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xh + R * 128 + 16 * swz(R, c));
#pragma unroll
          for (int j = 0; j < J; ++j) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wf[j], acc[m][j], 0, 0, 0);
        }
      }
    }
  }

  // ---------------- epilogue: partial tile -> LDS [16 MT][ROWS] f32 ----------------------
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wait_vm<0>();
  barrier_raw();
  float* sC = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[(16 * m + 4 * fh + r) * G::EPI_LD + wid * (ROWS / 4) + 16 * j + fr] = acc[m][j][r];
  __syncthreads();
  if constexpr (SLAB) {
    float* ps = reinterpret_cast<float*>(C) + (size_t)slice * M * N;
    for (int e = tid; e < M * (ROWS / 4); e += ST_THREADS) {
      const int row = e / (ROWS / 4), c4 = (e % (ROWS / 4)) * 4;
      const int col = ntile * ROWS + c4;
      if (col < N) {  // N % 4 == 0 (host check)
        const float* src = sC + row * G::EPI_LD + c4;
        *reinterpret_cast<f32x4*>(ps + (size_t)row * N + col) = (f32x4){src[0], src[1], src[2], src[3]};
      }
    }
    return;
  }

  auto finish = [&](int row, int c, float v) {  // c = output column
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
  constexpr int OUTC = PAIR ? ROWS / 2 : ROWS;
  // final value of local column cc (pair: gate cc with up cc + ROWS/2) for activation row `row`
  auto emit = [&](int row, int cc) {
    const int gp = stream_row<ROWS, PAIR>(ntile, cc);  // packed weight row (the gate row of a pair)
    if (gp >= Nrows) return;
    float v = sC[row * G::EPI_LD + cc];
    if constexpr (PAIR) {
      float u = sC[row * G::EPI_LD + cc + ROWS / 2];
      if constexpr (FP8) {
        v *= wscale[gp];
        u *= wscale[gp + 64];
      }
      finish(row, (gp >> 7) * 64 + (gp & 63), silu(v) * u);
    } else {
      if constexpr (FP8) v *= wscale[gp];
      finish(row, gp, v);
    }
  };

  if (S == 1) {
    for (int e = tid; e < M * OUTC; e += ST_THREADS) emit(e / OUTC, e % OUTC);
    return;
  }
  // split-K: slab ws[slice][tile][row][ROWS] fp32 (16-B stores), then the last-arriving block reduces
  const size_t slab = (size_t)ntiles * M * ROWS;
  const size_t tbase = (size_t)ntile * M * ROWS;
  for (int e = tid; e < M * (ROWS / 4); e += ST_THREADS) {
    const int row = e / (ROWS / 4), c4 = (e % (ROWS / 4)) * 4;
    const float* src = sC + row * G::EPI_LD + c4;
    *reinterpret_cast<f32x4*>(ws + slice * slab + tbase + (size_t)row * ROWS + c4) =
        (f32x4){src[0], src[1], src[2], src[3]};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(counters + ntile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag = (old == S - 1);
  }
  __syncthreads();
  if (!s_flag) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // reduce the S slabs of this tile into sC (all loads of a round issued before any use), then
  // run the epilogue from LDS exactly as the S == 1 path
  const float* __restrict__ wsr = ws;
  for (int e = tid; e < M * (ROWS / 4); e += ST_THREADS) {
    const int row = e / (ROWS / 4), c4 = (e % (ROWS / 4)) * 4;
    const size_t off = tbase + (size_t)row * ROWS + c4;
    f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < S) v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(wsr + q * slab + off));
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < S) a += v[q];
    for (int q = 8; q < S; ++q) a += *reinterpret_cast<const f32x4*>(wsr + q * slab + off);
    float* d = sC + row * G::EPI_LD + c4;
    d[0] = a[0]; d[1] = a[1]; d[2] = a[2]; d[3] = a[3];
  }
  __syncthreads();
  for (int e = tid; e < M * OUTC; e += ST_THREADS) emit(e / OUTC, e % OUTC);
  if (tid == 0) __hip_atomic_store(counters + ntile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Weight-stream cache policy for the SiLU*up (gate/up) instantiations: 1 = non-temporal.
int g_stream_nt = 1;
// diagnostic build of the SiLU*up 64-row kernel (DG above; A/B tooling only)
int g_stream_diag = 0;
// Tile rows for the SiLU*up GEMM: 64 = two blocks per CU over 64-row (32 gate + 32 up) tiles, so the
// 28672-row Llama gate/up grid (448 tiles) occupies all 256 CUs; 128 = one block per CU, 224 tiles.
int g_stream_pair_rows = 64;

inline int stream_rows(int epi) { return (epi == EPI_SILU_MUL && g_stream_pair_rows == 64) ? 64 : WROWS; }

template <int MT, int EPI, bool F32, bool FP8>
int launch_stream(const void* X, int ldx, const void* W, int ldw, const float* wscale, void* C, int ldc,
                  const void* bias, const void* resid, int ldr, int M, int N, int K, int S, float* ws, int* cnt,
                  hipStream_t st) {
  const int Nrows = EPI == EPI_SILU_MUL ? 2 * N : N;
  if constexpr (EPI == EPI_SILU_MUL) {
#define RAGK_ST_PAIR(NTV, R)                                                                                         \
  hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI, F32, FP8, NTV, R>), dim3((Nrows + R - 1) / R, S), dim3(ST_THREADS), \
                     0, st, (const bf16_t*)X, ldx, W, ldw, wscale, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid,  \
                     ldr, M, N, K, S, ws, cnt)
    if (g_stream_pair_rows == 64 && g_stream_diag && !FP8) {
#define RAGK_ST_DG(DGV)                                                                                              \
  hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI, F32, FP8, true, 64, false, DGV>), dim3((Nrows + 63) / 64, S),       \
                     dim3(ST_THREADS), 0, st, (const bf16_t*)X, ldx, W, ldw, wscale, C, ldc, (const bf16_t*)bias,     \
                     (const bf16_t*)resid, ldr, M, N, K, S, ws, cnt)
      if (g_stream_diag == 1) RAGK_ST_DG(1);
      else if (g_stream_diag == 2) RAGK_ST_DG(2);
      else RAGK_ST_DG(3);
#undef RAGK_ST_DG
    } else if (g_stream_pair_rows == 64) {
      if (g_stream_nt) RAGK_ST_PAIR(true, 64);
      else RAGK_ST_PAIR(false, 64);
    } else {
      if (g_stream_nt) RAGK_ST_PAIR(true, 128);
      else RAGK_ST_PAIR(false, 128);
    }
#undef RAGK_ST_PAIR
    return (int)hipGetLastError();
  }
  const dim3 grid((Nrows + WROWS - 1) / WROWS, S);
  if (g_stream_nt && Nrows >= 65536)  // vocab-sized weights, read once per step: non-temporal
    hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI, F32, FP8, true>), grid, dim3(ST_THREADS), 0, st, (const bf16_t*)X,
                       ldx, W, ldw, wscale, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K, S, ws, cnt);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI, F32, FP8>), grid, dim3(ST_THREADS), 0, st, (const bf16_t*)X, ldx,
                       W, ldw, wscale, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K, S, ws, cnt);
  return (int)hipGetLastError();
}

template <int MT>
int launch_stream_slab(const void* X, int ldx, const void* W, int ldw, float* P, int M, int N, int K, int S, int rows,
                       hipStream_t st) {
  const dim3 grid((N + rows - 1) / rows, S);
  // non-temporal weight stream (each weight byte is read once per step)
  if (rows == 64)
    hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI_NONE, true, false, true, 64, true>), grid, dim3(ST_THREADS), 0, st,
                       (const bf16_t*)X, ldx, W, ldw, nullptr, P, N, nullptr, nullptr, 0, M, N, K, S, nullptr, nullptr);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<MT, EPI_NONE, true, false, true, WROWS, true>), grid, dim3(ST_THREADS), 0,
                       st, (const bf16_t*)X, ldx, W, ldw, nullptr, P, N, nullptr, nullptr, 0, M, N, K, S, nullptr,
                       nullptr);
  return (int)hipGetLastError();
}

template <int EPI, bool F32, bool FP8>
int dispatch_stream(const void* X, int ldx, const void* W, int ldw, const float* wscale, void* C, int ldc,
                    const void* bias, const void* resid, int ldr, int M, int N, int K, int S, float* ws, int* cnt,
                    hipStream_t st) {
  switch ((M + 15) / 16) {
    case 1: return launch_stream<1, EPI, F32, FP8>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, cnt, st);
    case 2: return launch_stream<2, EPI, F32, FP8>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, cnt, st);
    case 3: return launch_stream<3, EPI, F32, FP8>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, cnt, st);
    case 4: return launch_stream<4, EPI, F32, FP8>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, cnt, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// Split count for the stream decode GEMM: enough blocks for 256 CUs (one block per CU), at least
// 8 K-steps per block, S | K-steps.
RAGK_API int ragk_gemm_stream_set_diag(int dg) {
  g_stream_diag = (dg >= 1 && dg <= 3) ? dg : 0;
  return 0;
}

RAGK_API int ragk_gemm_stream_set_nt(int nt) {
  g_stream_nt = nt ? 1 : 0;
  return 0;
}

RAGK_API int ragk_gemm_stream_set_pair_rows(int rows) {
  if (rows != 64 && rows != 128) return (int)hipErrorInvalidValue;
  g_stream_pair_rows = rows;
  return 0;
}

RAGK_API int ragk_gemm_stream_splits(int N, int K, int epi, int fp8) {
  const int Nrows = epi == EPI_SILU_MUL ? 2 * N : N;
  const int rows = stream_rows(epi);
  const int tiles = (Nrows + rows - 1) / rows;
  const int steps = K / (fp8 ? 128 : 64);
  int S = 1;
  const int slots = rows == 64 ? 640 : 320;  // 64-row tiles: two blocks per CU
  while (tiles * S * 2 <= slots && steps % (S * 2) == 0 && steps / (S * 2) >= 8) S *= 2;
  return S;
}

// C[M,N] = epi(X[M,K] . W^T): W bf16 [Nrows, K] (wscale == null) or fp8 e4m3 [Nrows, K] with per-row
// fp32 scales. M <= 64. ws/counters: split-K workspace (S * M * ceil(Nrows/128)*128 floats, Nrows/64
// zeroed ints).
RAGK_API int ragk_gemm_stream(const void* X, int ldx, const void* W, int ldw, const float* wscale, void* C, int ldc,
                              const void* bias, const void* resid, int ldr, int M, int N, int K, int epi, int out_f32,
                              int S, float* ws, int* counters, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  const bool fp8 = wscale != nullptr;
  const int kstep = fp8 ? 128 : 64;
  if (M > 64 || K % kstep || S < 1 || (K / kstep) % S) return (int)hipErrorInvalidValue;
  if (S > 1 && (!ws || !counters)) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL) {
    if (N % 64 || out_f32) return (int)hipErrorInvalidValue;
    return fp8 ? dispatch_stream<EPI_SILU_MUL, false, true>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K,
                                                            S, ws, counters, st)
               : dispatch_stream<EPI_SILU_MUL, false, false>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N,
                                                             K, S, ws, counters, st);
  }
#define RAGK_ST_CASE(E)                                                                                             \
  case E:                                                                                                           \
    if (fp8)                                                                                                        \
      return out_f32 ? dispatch_stream<E, true, true>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, \
                                                      counters, st)                                                 \
                     : dispatch_stream<E, false, true>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S,  \
                                                       ws, counters, st);                                           \
    return out_f32 ? dispatch_stream<E, true, false>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, \
                                                     counters, st)                                                  \
                   : dispatch_stream<E, false, false>(X, ldx, W, ldw, wscale, C, ldc, bias, resid, ldr, M, N, K, S, ws, \
                                                      counters, st);
  switch (epi) {
    RAGK_ST_CASE(EPI_NONE)
    RAGK_ST_CASE(EPI_BIAS)
    RAGK_ST_CASE(EPI_RESID)
    RAGK_ST_CASE(EPI_BIAS_RESID)
    RAGK_ST_CASE(EPI_GELU)
    RAGK_ST_CASE(EPI_BIAS_GELU)
    RAGK_ST_CASE(EPI_BIAS_GELU_TANH)
    default: return (int)hipErrorInvalidValue;
  }
#undef RAGK_ST_CASE
}

// Split-K partial slabs P[S][M][N] (fp32) of X[M,K] . W[N,K]^T through the LDS-DMA weight ring (SLAB
// above): bf16 weights, M <= 64, N % 4 == 0, S | K / 64, rows = 64 (two blocks per CU) or 128.
RAGK_API int ragk_gemm_stream_part(const void* X, int ldx, const void* W, int ldw, float* P, int M, int N, int K,
                                   int S, int rows, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 64 || K % 64 || S < 1 || (K / 64) % S || N % 4 || (rows != 64 && rows != 128) || ldx % 8 || ldw % 8)
    return (int)hipErrorInvalidValue;
  switch ((M + 15) / 16) {
    case 1: return launch_stream_slab<1>(X, ldx, W, ldw, P, M, N, K, S, rows, st);
    case 2: return launch_stream_slab<2>(X, ldx, W, ldw, P, M, N, K, S, rows, st);
    case 3: return launch_stream_slab<3>(X, ldx, W, ldw, P, M, N, K, S, rows, st);
    case 4: return launch_stream_slab<4>(X, ldx, W, ldw, P, M, N, K, S, rows, st);
    default: return (int)hipErrorInvalidValue;
  }
}
