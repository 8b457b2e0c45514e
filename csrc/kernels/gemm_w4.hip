// 256x256x64 bf16 GEMM, 4 waves x (128x128) per workgroup, one wave per SIMD (large-M prefill GEMMs).
//
// C[M,N] = A[M,K] . B[N,K]^T (+ fused epilogue); same operands / epilogues as gemm.hip / gemm_pp.hip.
//
// Why a second 256x256 design next to the 8-wave ping-pong (gemm_pp.hip): rocprofv3 PMC on the
// Llama-8B prefill shapes (profiles/pmc_gemm_r1.txt) put the ping-pong at 64 % MFMA-pipe utilisation
// vs 75 % for hipBLASLt's 256x256x64 4-wave kernel at the same clock. The ping-pong pays one
// workgroup barrier per 64 MFMAs per SIMD, gives its K-tile DMA only ~1 interval (~1k cycles) to land
// before a vmcnt(0), and re-reads every A fragment from LDS for each of 4 column waves (192 KiB of
// ds_read per K-tile). Here each wave owns a 128x128 output tile (8 x 8 mfma_f32_16x16x32_bf16
// accumulators = 256 AGPRs), so per K-tile (64-deep) and SIMD: 128 MFMAs, one barrier, 128 KiB of
// LDS reads per CU, and each DMA is issued 128 MFMAs (~2k cycles) before its wait.
//
// Per-wave software pipeline, one K-tile per iteration (fragment sets F0 = k 0..31, F1 = k 32..63;
// tile t lives in LDS buffer t&1, lane-linear image, source-swizzled as gemm_pp):
//   seg 1: ds_read F1(t), one per MFMA | MFMA F0 #0..23           -> lgkmcnt(0); barrier 1
//   seg 2: 16 buffer-DMAs of tile t+2 -> buffer t&1 (every wave finished reading tile t before
//          barrier 1), one per 5 MFMAs | MFMA F0 #24..63, F1 #0..47 -> vmcnt(16) [tile t+1 landed,
//          t+2 in flight]; barrier 2
//   seg 3: ds_read F0(t+1) from buffer (t+1)&1, one per MFMA | MFMA F1 #48..63
// A DMA is issued 1-1.7 K-tiles (2-3.5k cycles) before the wait that retires it, and DMA issue is
// spread over the MFMA stream: with one wave per SIMD nothing else hides its issue cost (a first
// version that issued all 16 back to back ran at 49-61 % MFMA utilisation). The DMA is
// buffer_load ... lds with per-lane byte offsets precomputed once (16 VGPRs) and the K position in
// an SGPR (as hipBLASLt's gfx950 256x256 kernels do), so no address VALU in the loop.
//
// Build note: the loop is written in its final instruction order and this file is compiled with
// `-mllvm -enable-misched=0 -mllvm -disable-post-ra` (_build.py EXTRA_FLAGS), so neither machine
// scheduler reorders it (the post-RA one bunched the DMAs at the end of segment 2).
#include <stdlib.h>

#include <utility>

#include "common.h"
using namespace ragk;

namespace {

constexpr int WBM = 256, WBN = 256, WBK = 64;
constexpr int W4_THREADS = 256;
constexpr int W_TILE_A = WBM * WBK * 2;  // 32 KiB
constexpr int W_TILE_B = WBN * WBK * 2;  // 32 KiB
constexpr int W_BUF = W_TILE_A + W_TILE_B;
constexpr int W4_LDS = 2 * W_BUF;  // two K-tile buffers; the epilogue needs no LDS
constexpr int WGROUP_M = 8;

__device__ __forceinline__ int wswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <typename F, int... Ms>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Ms...>) {
  (f(std::integral_constant<int, Ms>{}), ...);
}
// f(integral_constant<int, m>) for m = 0..N-1, every m a compile-time constant
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// 256 rows x 128 B = 32 pieces of 8 rows; wave w stages pieces 8w..8w+7 of each operand. Per-lane
// byte offsets of those 8 pieces (row clamped to the last valid row, chunk source-swizzled).
__device__ __forceinline__ void w4_offsets(int ld, int row0, int rows_valid, int wid, int lane, int (&off)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = (wid * 8 + i) * 8 + (lane >> 3);
    const int c = wswz(r, lane & 7);
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    off[i] = gr * ld * 2 + c * 16;
  }
}

__device__ __forceinline__ void w4_stage(i32x4 srd, const int (&off)[8], int k0, char* lds, int wid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) blds16(srd, off[i], k0 * 2, lds + (wid * 8 + i) * 1024);
}

__device__ __forceinline__ void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// fragments of one 32-deep sub-step: A rows wr*128 + 16i + fr, B rows wc*128 + 16j + fr, chunk 4s + fh
__device__ __forceinline__ void w4_read(const char* buf, int s, int wr, int wc, int fr, int fh, bf16x8 (&a)[8],
                                        bf16x8 (&b)[8]) {
  const char* sa = buf;
  const char* sb = buf + W_TILE_A;
  const int c = 4 * s + fh;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int R = wr * 128 + 16 * i + fr;
    a[i] = *reinterpret_cast<const bf16x8*>(sa + R * 128 + 16 * wswz(R, c));
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int R = wc * 128 + 16 * j + fr;
    b[j] = *reinterpret_cast<const bf16x8*>(sb + R * 128 + 16 * wswz(R, c));
  }
}

// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int W_LGKM0 = 0xC07F;  // lgkmcnt(0), others don't-care
constexpr int W_VM0 = 0x0F70;    // vmcnt(0), others don't-care
constexpr int W_VM16 = 0x4F70;   // vmcnt(16)

// Vector-memory ops one wave issues in w4_epilogue_reg on a full tile (no row/column guard): the
// persistent loop's wait for the next tile's first K-tile counts them as younger than its DMA.
// bf16 outputs of full tiles use the widened store epilogue (w4_epilogue_wide: 16 B per lane),
// fp32 outputs the 4-column one (w4_epilogue_reg).
template <int EPI, bool OUT_F32>
constexpr int w4_epi_vmem() {
  if constexpr (EPI == EPI_SILU_MUL) return 16;
  constexpr bool RES = (EPI == EPI_RESID || EPI == EPI_BIAS_RESID);
  constexpr bool BIAS = (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU ||
                         EPI == EPI_BIAS_GELU_TANH);
  return (OUT_F32 ? 64 : 32) + (RES ? 64 : 0) + (BIAS ? 8 : 0);  // bf16: 32 x 16-B stores
}

__device__ __forceinline__ void w4_store4(void* C, size_t idx, const float (&o)[4], bool f32) {
  if (f32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + idx) = (f32x4){o[0], o[1], o[2], o[3]};
  } else {
    const unsigned lo = pk2bf(o[0], o[1]);
    const unsigned hi = pk2bf(o[2], o[3]);
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(C) + idx) = make_uint2(lo, hi);
  }
}

__device__ __forceinline__ void unpack4(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

// Epilogue straight from the (transposed) accumulators, no LDS and no barrier: lane (fr, fh) writes
// 4 consecutive columns (8 B bf16 / 16 B fp32) of row 16i + fr for each of its 64 fragments. LDS is
// left to the next tile's K-tile DMAs, which the persistent loop issues before this runs. FULL: the
// tile lies inside [M, N], every lane stores unguarded (exactly w4_epi_vmem ops per wave).
// resid may alias C: every element is read and written by the same lane.
template <int EPI, bool OUT_F32, bool FULL>
__device__ __forceinline__ void w4_epilogue_reg(const f32x4 (&acc)[8][8], int wr, int wc, int fr, int fh, int m0,
                                                int n0, void* C, int ldc, const bf16_t* __restrict__ bias,
                                                const bf16_t* resid, int ldr, int M, int N) {
  const int row0 = m0 + wr * 128 + fr;
  if constexpr (EPI == EPI_SILU_MUL) {
    // packed columns: this wave's 128 = [64 gate | 64 up] -> 64 output columns; gate fragment j
    // and up fragment j + 4 hold the same output columns in the same lane
    const int col0 = (n0 >> 1) + wc * 64 + 4 * fh;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gr = row0 + 16 * i;
      if (FULL || gr < M) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = silu(acc[i][j][r]) * acc[i][j + 4][r];
          w4_store4(C, (size_t)gr * ldc + col0 + 16 * j, o, false);
        }
      }
    }
  } else {
    constexpr bool RES = (EPI == EPI_RESID || EPI == EPI_BIAS_RESID);
    constexpr bool BIAS = (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU ||
                           EPI == EPI_BIAS_GELU_TANH);
    const int col0 = n0 + wc * 128 + 4 * fh;
    uint2 bv[BIAS ? 8 : 1];
    if constexpr (BIAS) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bv[j] = *reinterpret_cast<const uint2*>(bias + (FULL ? col0 + 16 * j : min(col0 + 16 * j, N - 4)));
    }
    // the whole residual tile of this lane is requested before the first use (one memory latency).
    // Loads are never predicated (edge tiles clamp the address instead): a load under a branch
    // makes hipcc's waitcnt pass drain vmcnt(0) at every join.
    uint2 rv[RES ? 64 : 1];
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int gr = FULL ? row0 + 16 * i : min(row0 + 16 * i, M - 1);
          const int gc = FULL ? col0 + 16 * j : min(col0 + 16 * j, N - 4);
          rv[8 * i + j] = *reinterpret_cast<const uint2*>(resid + (size_t)gr * ldr + gc);
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gr = row0 + 16 * i;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gc = col0 + 16 * j;
        if (FULL || (gr < M && gc < N)) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r];
          if constexpr (BIAS) {
            float b[4];
            unpack4(bv[j], b);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] += b[r];
          }
          if constexpr (RES) {
            float rr[4];
            unpack4(rv[8 * i + j], rr);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] += rr[r];
          }
          if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = gelu_erf(o[r]);
          }
          if constexpr (EPI == EPI_BIAS_GELU_TANH) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = gelu_tanh(o[r]);
          }
          w4_store4(C, (size_t)gr * ldc + gc, o, OUT_F32);
        }
      }
    }
  }
}

// Widened full-tile epilogue for bf16 outputs (T21 for the 16x16 layout): lane (fr, fh) of acc[i][j]
// holds 4 consecutive columns 16j + 4fh.. of row 16i + fr, so the plain store is 64 x 8 B per lane,
// each instruction touching 16 rows x 32 B -- an issue-bound tail of ~30k cycles per 256x256 tile in
// which no MFMA runs. Packed to bf16 first (same fp32 epilogue math and single rounding as
// w4_epilogue_reg), tiles j and j+1 are paired with v_permlane16_swap (odd 16-lane rows of the
// first operand <-> even rows of the second): afterwards lanes fh = 0 / 2 hold columns 0-7 / 8-15
// of tile j and lanes fh = 1 / 3 those of tile j+1, so each pair is ONE 16-byte store per lane,
// half the store instructions for the same bytes.
__device__ __forceinline__ void w4_swap_store(bf16_t* row, int col_j, int fh, unsigned (&x)[2], unsigned (&y)[2]) {
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    auto r = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
  const int col = col_j + 16 * (fh & 1) + 8 * (fh >> 1);
  *reinterpret_cast<uint4*>(row + col) = make_uint4(x[0], x[1], y[0], y[1]);
}

template <int EPI>
__device__ __forceinline__ void w4_epilogue_wide(const f32x4 (&acc)[8][8], int wr, int wc, int fr, int fh, int m0,
                                                 int n0, void* C, int ldc, const bf16_t* __restrict__ bias,
                                                 const bf16_t* resid, int ldr) {
  const int row0 = m0 + wr * 128 + fr;
  bf16_t* Cb = reinterpret_cast<bf16_t*>(C);
  if constexpr (EPI == EPI_SILU_MUL) {
    const int colb = (n0 >> 1) + wc * 64;  // output tiles j = 0..3: gate acc[i][j], up acc[i][j + 4]
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16_t* row = Cb + (size_t)(row0 + 16 * i) * ldc;
#pragma unroll
      for (int jp = 0; jp < 4; jp += 2) {
        unsigned x[2], y[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float a[4], b[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a[r] = silu(acc[i][jp][r]) * acc[i][jp + 4][r];
            b[r] = silu(acc[i][jp + 1][r]) * acc[i][jp + 5][r];
          }
          x[h] = pk2bf(a[2 * h], a[2 * h + 1]);
          y[h] = pk2bf(b[2 * h], b[2 * h + 1]);
        }
        w4_swap_store(row, colb + 16 * jp, fh, x, y);
      }
    }
  } else {
    constexpr bool RES = (EPI == EPI_RESID || EPI == EPI_BIAS_RESID);
    constexpr bool BIAS = (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU ||
                           EPI == EPI_BIAS_GELU_TANH);
    const int col0 = n0 + wc * 128 + 4 * fh;  // this lane's pre-swap columns in tile j: col0 + 16j
    uint2 bv[BIAS ? 8 : 1];
    if constexpr (BIAS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = *reinterpret_cast<const uint2*>(bias + col0 + 16 * j);
    }
    uint2 rv[RES ? 64 : 1];
    if constexpr (RES) {  // whole residual tile of this lane in flight before the first use
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rv[8 * i + j] = *reinterpret_cast<const uint2*>(resid + (size_t)(row0 + 16 * i) * ldr + col0 + 16 * j);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16_t* row = Cb + (size_t)(row0 + 16 * i) * ldc;
#pragma unroll
      for (int jp = 0; jp < 8; jp += 2) {
        unsigned pk[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = jp + q;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r];
          if constexpr (BIAS) {
            float b[4];
            unpack4(bv[j], b);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] += b[r];
          }
          if constexpr (RES) {
            float rr[4];
            unpack4(rv[8 * i + j], rr);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] += rr[r];
          }
          if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = gelu_erf(o[r]);
          }
          if constexpr (EPI == EPI_BIAS_GELU_TANH) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = gelu_tanh(o[r]);
          }
          pk[q][0] = pk2bf(o[0], o[1]);
          pk[q][1] = pk2bf(o[2], o[3]);
        }
        w4_swap_store(row, n0 + wc * 128 + 16 * jp, fh, pk[0], pk[1]);
      }
    }
  }
}

// MFMA #m (= 8i + j) of a sub-step. Inline asm with the accumulator tied in an AGPR ("+a"): with the
// builtin, hipcc picks dst != srcC for the loop-carried accumulators and adds 84-500 v_accvgpr copies
// per K-tile. volatile + "memory" keep the statement in source order relative to the LDS reads and
// DMAs around it (the loop is written in its final order). Hazards the compiler no longer pads:
// acc init -> first MFMA and last MFMA -> epilogue reads (w4_pin_acc below); the accumulate chain
// itself (same acc every 64 MFMAs) and ds_read -> srcA/B (s_waitcnt, inserted by hipcc) need none.
// The weight fragment is srcA and the activation fragment srcB, so the accumulator comes out
// transposed: lane (fr, fh) of acc[i][j] holds C[16i + fr][16j + 4fh .. 16j + 4fh + 3] -- four
// consecutive output columns of one row, stored straight from registers by w4_epilogue_reg.
__device__ __forceinline__ void w4_mfma(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8], int m) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %1, %0"
               : "+a"(acc[m >> 3][m & 7])
               : "v"(a[m >> 3]), "v"(b[m & 7])
               : "memory");
}

// Orders every accumulator access after an s_nop pad (>= 16 wait states covers MFMA D -> VALU/DS read
// and v_accvgpr_write -> MFMA srcC).
__device__ __forceinline__ void w4_pin_acc(f32x4 (&acc)[8][8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 1" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j])::"memory");
}

// Fragment q (0..15) of a sub-step in the order the next MFMAs consume them: a[0], b[0..7], a[1..7].
__device__ __forceinline__ void w4_read_frag(const char* buf, int s, int q, int wr, int wc, int fr, int fh,
                                             bf16x8 (&a)[8], bf16x8 (&b)[8]) {
  const int c = 4 * s + fh;
  if (q == 0 || q > 8) {
    const int i = q == 0 ? 0 : q - 8;
    const int R = wr * 128 + 16 * i + fr;
    a[i] = *reinterpret_cast<const bf16x8*>(buf + R * 128 + 16 * wswz(R, c));
  } else {
    const int j = q - 1;
    const int R = wc * 128 + 16 * j + fr;
    b[j] = *reinterpret_cast<const bf16x8*>(buf + W_TILE_A + R * 128 + 16 * wswz(R, c));
  }
}

// One K-tile, written in final instruction order (file built with -enable-misched=0).
// STAGE: issue tile t+2's DMA; READ: read F0(t+1). The 128 MFMAs (m < 64: F0, m >= 64: F1) are split
// S1 | 128-S1-S3 | S3 by the two barriers; the 16 F1 reads go 1:1 into the first MFMAs of segment 1,
// the 16 DMAs evenly through segment 2, the 16 F0(t+1) reads evenly through segment 3. The split
// was set from the stamp build's cycle anatomy (tools/gemm_stamps.py).
constexpr int W4_S1 = 32, W4_S3 = 16;
constexpr int W4_SCHED = 0;  // production schedule: 0 = w4_iter (S1/S3 split), 2 = w4_iter2
#ifndef RAGK_W4_WIDE_EPI
#define RAGK_W4_WIDE_EPI 1
#endif
constexpr bool W4_WIDE_EPI = RAGK_W4_WIDE_EPI;  // widened 16-B store epilogue for bf16 outputs

// j-major variants (SCHED 3): MFMA #m of a sub-step is acc[m & 7][m >> 3], so srcA (the weight
// fragment b[j]) stays the same register quad for 8 consecutive MFMAs (as in hipBLASLt's loop);
// reads come in consumption order b[0], a[0..7], b[1..7].
__device__ __forceinline__ void w4_mfma_jm(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8], int m) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %1, %0"
               : "+a"(acc[m & 7][m >> 3])
               : "v"(a[m & 7]), "v"(b[m >> 3])
               : "memory");
}

__device__ __forceinline__ void w4_read_frag_jm(const char* buf, int s, int q, int wr, int wc, int fr, int fh,
                                                bf16x8 (&a)[8], bf16x8 (&b)[8]) {
  const int c = 4 * s + fh;
  if (q == 0 || q > 8) {
    const int j = q == 0 ? 0 : q - 8;
    const int R = wc * 128 + 16 * j + fr;
    b[j] = *reinterpret_cast<const bf16x8*>(buf + W_TILE_A + R * 128 + 16 * wswz(R, c));
  } else {
    const int i = q - 1;
    const int R = wr * 128 + 16 * i + fr;
    a[i] = *reinterpret_cast<const bf16x8*>(buf + R * 128 + 16 * wswz(R, c));
  }
}

__device__ __forceinline__ void w4_mfma_m(f32x4 (&acc)[8][8], const bf16x8 (&a0)[8], const bf16x8 (&b0)[8],
                                          const bf16x8 (&a1)[8], const bf16x8 (&b1)[8], int m) {
  if (m < 64) w4_mfma(acc, a0, b0, m);
  else w4_mfma(acc, a1, b1, m - 64);
}

template <bool STAGE, bool READ, bool STAMP = false, int S1 = W4_S1, int S3 = W4_S3>
__device__ __forceinline__ void w4_iter(char* smem, int t, i32x4 srd_a, i32x4 srd_b, const int (&off_a)[8],
                                        const int (&off_b)[8], int wid, int wr, int wc, int fr, int fh,
                                        f32x4 (&acc)[8][8], bf16x8 (&a0)[8], bf16x8 (&b0)[8], bf16x8 (&a1)[8],
                                        bf16x8 (&b1)[8], unsigned long long (&stp)[5]) {
  static_assert(S1 >= 16 && S1 <= 64 && S3 >= 16 && S3 <= 64, "segment split");
  constexpr int N2 = 128 - S1 - S3;
  char* buf = smem + (t & 1) * W_BUF;
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
  // ---------------- seg 1: read F1(t), one per MFMA | MFMA #0..S1-1 ------------------------
#pragma unroll
  for (int m = 0; m < S1; ++m) {
    if (m < 16) w4_read_frag(buf, 1, m, wr, wc, fr, fh, a1, b1);
    w4_mfma_m(acc, a0, b0, a1, b1, m);
  }
  if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
  // builtin (not inline-asm) waits: hipcc's waitcnt pass sees them and adds no redundant waits
  __builtin_amdgcn_s_waitcnt(W_LGKM0);  // every read of buffer t&1 retired
  w4_barrier();
  if constexpr (STAMP) t2 = __builtin_amdgcn_s_memtime();
  // ---------------- seg 2: 16 DMAs of tile t+2 -> buffer t&1 (spread) | MFMA #S1..127-S3 -----
  static_assert(N2 % 16 == 0 && (S3 == 16 || S3 == 24 || S3 == 32), "segment split");
  constexpr int DSTEP = N2 / 16;  // MFMAs per DMA
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    if constexpr (STAGE) {
      if (i % DSTEP == 0) {
        const int q = i / DSTEP;
        if (q < 8) blds16(srd_a, off_a[q], (t + 2) * WBK * 2, buf + (wid * 8 + q) * 1024);
        else blds16(srd_b, off_b[q - 8], (t + 2) * WBK * 2, buf + W_TILE_A + (wid * 8 + q - 8) * 1024);
      }
    }
    w4_mfma_m(acc, a0, b0, a1, b1, S1 + i);
  }
  if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
  if constexpr (STAGE) __builtin_amdgcn_s_waitcnt(W_VM16);  // tile t+1 landed (t+2's 16 in flight)
  else __builtin_amdgcn_s_waitcnt(W_VM0);
  w4_barrier();
  if constexpr (STAMP) {
    const unsigned long long t4 = __builtin_amdgcn_s_memtime();
    stp[0] += t1 - t0;  // seg 1 issue
    stp[1] += t2 - t1;  // lgkmcnt(0) + barrier 1
    stp[2] += t3 - t2;  // seg 2 issue
    stp[3] += t4 - t3;  // vmcnt(16) + barrier 2
  }
  // ---------------- seg 3: read F0(t+1) from buffer (t+1)&1 (spread) | MFMA #128-S3..127 ----
  const char* nbuf = smem + ((t + 1) & 1) * W_BUF;
#pragma unroll
  for (int i = 0; i < S3; ++i) {
    if constexpr (READ) {
      if constexpr (S3 == 16) {
        w4_read_frag(nbuf, 0, i, wr, wc, fr, fh, a0, b0);
      } else if constexpr (S3 == 32) {
        if (i % 2 == 0) w4_read_frag(nbuf, 0, i / 2, wr, wc, fr, fh, a0, b0);
      } else {  // 24: two reads per three MFMAs
        if (i % 3 < 2) w4_read_frag(nbuf, 0, 2 * (i / 3) + i % 3, wr, wc, fr, fh, a0, b0);
      }
    }
    w4_mfma_m(acc, a0, b0, a1, b1, 128 - S3 + i);
  }
  if constexpr (STAMP) stp[4] += __builtin_amdgcn_s_memtime() - t0;  // whole iteration
}

// Single-barrier iteration (S3 == 0 selects it): one barrier per K-tile retires both the F1(t) reads
// (lgkmcnt(0)) and this wave's DMA of tile t+1 (vmcnt(0)); after it the 16 DMAs of tile t+2 go
// through the first 32 MFMAs of segment 2 (F0 #S1..63) and the 16 F0(t+1) reads through the 64 F1
// MFMAs (a0/b0 are dead once F0 #63 has issued). No third segment, no second barrier.
template <bool STAGE, bool READ, bool STAMP, int S1>
__device__ __forceinline__ void w4_iter1(char* smem, int t, i32x4 srd_a, i32x4 srd_b, const int (&off_a)[8],
                                         const int (&off_b)[8], int wid, int wr, int wc, int fr, int fh,
                                         f32x4 (&acc)[8][8], bf16x8 (&a0)[8], bf16x8 (&b0)[8], bf16x8 (&a1)[8],
                                         bf16x8 (&b1)[8], unsigned long long (&stp)[5]) {
  static_assert(S1 >= 16 && S1 <= 48, "segment split");
  constexpr int NF0 = 64 - S1;  // F0 MFMAs after the barrier
  char* buf = smem + (t & 1) * W_BUF;
  const char* nbuf = smem + ((t + 1) & 1) * W_BUF;
  unsigned long long t0 = 0, t1 = 0, t2 = 0;
  if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int m = 0; m < S1; ++m) {
    if (m < 16) w4_read_frag(buf, 1, m, wr, wc, fr, fh, a1, b1);
    w4_mfma(acc, a0, b0, m);
  }
  if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(W_LGKM0);  // F1(t) in registers: buffer t&1 free
  __builtin_amdgcn_s_waitcnt(W_VM0);    // this wave's part of tile t+1 landed
  w4_barrier();
  if constexpr (STAMP) t2 = __builtin_amdgcn_s_memtime();
  // F0 #S1..63 with the 16 DMAs spread over them
#pragma unroll
  for (int i = 0; i < NF0; ++i) {
    if constexpr (STAGE) {
      if ((i * 16) % NF0 < 16) {
        const int q = (i * 16) / NF0;
        if (q < 8) blds16(srd_a, off_a[q], (t + 2) * WBK * 2, buf + (wid * 8 + q) * 1024);
        else blds16(srd_b, off_b[q - 8], (t + 2) * WBK * 2, buf + W_TILE_A + (wid * 8 + q - 8) * 1024);
      }
    }
    w4_mfma(acc, a0, b0, S1 + i);
  }
  // F1 #0..63 with the 16 F0(t+1) reads, one per 4 MFMAs
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if constexpr (READ) {
      if (i % 4 == 0) w4_read_frag(nbuf, 0, i / 4, wr, wc, fr, fh, a0, b0);
    }
    w4_mfma(acc, a1, b1, i);
  }
  if constexpr (STAMP) {
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    stp[0] += t1 - t0;
    stp[1] += t2 - t1;
    stp[2] += t3 - t2;
    stp[4] += t3 - t0;
  }
}

// Spread two-barrier iteration (SCHED 2), the read/DMA placement of hipBLASLt's gfx950 256x256x64
// direct-to-LDS kernel (studied from its disassembly: LDS fragment reads ~one per two MFMAs and
// issued a full sub-step ahead of their use, DMAs one per few MFMAs): the old schedule (w4_iter)
// bunched its 32 fragment reads into 32 of the 128 MFMAs (one read per 16-cycle MFMA gap: the LDS
// saturates with 4 waves) and issued F0(t+1) right before the MFMAs that consume it.
//   m 0..BA-1 : 16 reads of F1(t) (buffer t&1), spread          [F0 MFMAs]
//   m = BA    : lgkmcnt(0) + barrier A: every wave holds F1(t), buffer t&1 is free
//   m BA..    : 16 DMAs of tile t+2 -> buffer t&1, one per DS MFMAs
//   m = 64    : vmcnt(#DMAs issued so far) (= tile t+1 landed) + barrier B
//   m 64..95  : 16 reads of F0(t+1) (buffer (t+1)&1), one per 2 MFMAs   [F1 MFMAs]
//   m 96..127 : MFMA only (the F0(t+1) reads land 32+ MFMAs before their use)
template <bool STAGE, bool READ, bool STAMP, int BA, int DS, bool JM = false, int RW = 2>
__device__ __forceinline__ void w4_iter2(char* smem, int t, i32x4 srd_a, i32x4 srd_b, const int (&off_a)[8],
                                         const int (&off_b)[8], int wid, int wr, int wc, int fr, int fh,
                                         f32x4 (&acc)[8][8], bf16x8 (&a0)[8], bf16x8 (&b0)[8], bf16x8 (&a1)[8],
                                         bf16x8 (&b1)[8], unsigned long long (&stp)[5]) {
  static_assert(BA >= 16 && BA <= 64 && BA % 16 == 0, "barrier A position");
  static_assert(BA + 15 * DS < 128, "DMA window");
  constexpr int RSA = BA / 16;                         // MFMAs per F1(t) read
  constexpr int NB = (64 - BA + DS - 1) / DS;         // DMAs issued before barrier B
  constexpr int VB = NB > 15 ? 15 : NB;
  char* buf = smem + (t & 1) * W_BUF;
  const char* nbuf = smem + ((t + 1) & 1) * W_BUF;
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
  // compile-time m (a #pragma unroll over this body is not always honoured: a runtime m would put
  // the accumulator array in scratch)
  static_for<128>([&](auto mc) __attribute__((always_inline)) {
    constexpr int m = decltype(mc)::value;
    if constexpr (m == BA) {
      if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_waitcnt(W_LGKM0);  // F1(t) in registers
      w4_barrier();                         // every wave: buffer t&1 no longer read
      if constexpr (STAMP) t2 = __builtin_amdgcn_s_memtime();
    }
    if constexpr (m == 64) {
      if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
      if constexpr (STAGE) __builtin_amdgcn_s_waitcnt((VB & 15) | (0x7 << 4) | (0xF << 8));  // vmcnt(VB)
      else __builtin_amdgcn_s_waitcnt(W_VM0);
      w4_barrier();  // tile t+1 landed for every wave
      if constexpr (STAMP) {
        const unsigned long long t4 = __builtin_amdgcn_s_memtime();
        stp[0] += t1 - t0;
        stp[1] += t2 - t1;
        stp[2] += t3 - t2;
        stp[3] += t4 - t3;
      }
    }
    if constexpr (m < BA && m % RSA == 0) {
      if constexpr (JM) w4_read_frag_jm(buf, 1, m / RSA, wr, wc, fr, fh, a1, b1);
      else w4_read_frag(buf, 1, m / RSA, wr, wc, fr, fh, a1, b1);
    }
    if constexpr (STAGE && m >= BA && (m - BA) % DS == 0 && (m - BA) / DS < 16) {
      constexpr int q = (m - BA) / DS;
      if constexpr (q < 8) blds16(srd_a, off_a[q], (t + 2) * WBK * 2, buf + (wid * 8 + q) * 1024);
      else blds16(srd_b, off_b[q - 8], (t + 2) * WBK * 2, buf + W_TILE_A + (wid * 8 + q - 8) * 1024);
    }
    if constexpr (READ && m >= 64 && m < 64 + 16 * RW && (m - 64) % RW == 0) {
      if constexpr (JM) w4_read_frag_jm(nbuf, 0, (m - 64) / RW, wr, wc, fr, fh, a0, b0);
      else w4_read_frag(nbuf, 0, (m - 64) / RW, wr, wc, fr, fh, a0, b0);
    }
    if constexpr (JM) {
      if constexpr (m < 64) w4_mfma_jm(acc, a0, b0, m);
      else w4_mfma_jm(acc, a1, b1, m - 64);
    } else {
      w4_mfma_m(acc, a0, b0, a1, b1, m);
    }
  });
  if constexpr (STAMP) stp[4] += __builtin_amdgcn_s_memtime() - t0;
}

// Output tile `tile` (of nwg) -> origin. Tiles are numbered so that the 8 XCDs each own a contiguous
// range (xcd_remap; a persistent block keeps its XCD since the grid is a multiple of 8), grouped
// WGROUP_M M-tiles deep for L2 reuse of the weight tiles.
__device__ __forceinline__ void w4_origin(int tile, int nwg, int tiles_m, int tiles_n, int& m0, int& n0) {
  const int logical = xcd_remap(tile, nwg);
  const int group = logical / (WGROUP_M * tiles_n);
  const int first_m = group * WGROUP_M;
  const int gm = min(tiles_m - first_m, WGROUP_M);
  const int in_group = logical % (WGROUP_M * tiles_n);
  m0 = (first_m + in_group % gm) * WBM;
  n0 = (in_group / gm) * WBN;
}

__device__ __forceinline__ void w4_zero(f32x4 (&acc)[8][8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
}

// Persistent: block b computes tiles b, b + G, b + 2G, ... (G = gridDim.x; G = nwg gives the plain
// one-tile-per-block launch). Between two tiles, LDS is free as soon as the K-loop's last barrier has
// passed, so the next tile's first two K-tiles are DMA'd BEFORE this tile's epilogue runs: the DMA
// latency that a fresh block pays in its prologue hides behind the epilogue's stores.
template <int EPI, bool OUT_F32, bool STAMP = false, int S1 = W4_S1, int S3 = W4_S3, int SCHED = W4_SCHED,
          bool WIDE = W4_WIDE_EPI>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4_kernel(const bf16_t* __restrict__ A, int lda,
                                                                const bf16_t* __restrict__ B, int ldb, void* C,
                                                                int ldc, const bf16_t* __restrict__ bias,
                                                                const bf16_t* resid, int ldr, int M, int N, int K,
                                                                unsigned long long* dbg) {
  __shared__ __attribute__((aligned(16))) char smem[W4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fh = lane >> 4;

  const int tiles_m = (M + WBM - 1) / WBM, tiles_n = (N + WBN - 1) / WBN;
  const int nwg = tiles_m * tiles_n;
  const int nk = K / WBK;

  // byte offsets are 32-bit: the launcher guarantees rows * ld * 2 < 2^31 for both operands
  const i32x4 srd_a = make_srd(A, (unsigned)M * (unsigned)lda * 2u);
  const i32x4 srd_b = make_srd(B, (unsigned)N * (unsigned)ldb * 2u);

  int tile = blockIdx.x;
  int m0, n0;
  w4_origin(tile, nwg, tiles_m, tiles_n, m0, n0);
  int off_a[8], off_b[8];
  w4_offsets(lda, m0, M, wid, lane, off_a);
  w4_offsets(ldb, n0, N, wid, lane, off_b);
  // prologue: K-tiles 0 and 1 in flight
  w4_stage(srd_a, off_a, 0, smem, wid);
  w4_stage(srd_b, off_b, 0, smem + W_TILE_A, wid);
  if (nk > 1) {
    w4_stage(srd_a, off_a, WBK, smem + W_BUF, wid);
    w4_stage(srd_b, off_b, WBK, smem + W_BUF + W_TILE_A, wid);
  }

  f32x4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  unsigned long long stp[5] = {0, 0, 0, 0, 0};
  // vector-memory ops issued after the current tile's K-tile-0 DMA: its 16 K-tile-1 DMAs, plus the
  // previous tile's full-tile epilogue (0 = none, or a guarded epilogue that drained itself)
  int younger_epi = 0, done = 0;
  unsigned long long tl_loop = 0, tl_epi = 0;  // STAMP: per-tile K-loop / epilogue cycles (sums)
  for (;;) {
    unsigned long long tt0 = 0;
    if constexpr (STAMP) tt0 = __builtin_amdgcn_s_memtime();
    w4_zero(acc);
    w4_pin_acc(acc);
    if (nk == 1) {
      __builtin_amdgcn_s_waitcnt(W_VM0);
    } else if (younger_epi == 0) {
      __builtin_amdgcn_s_waitcnt(W_VM16);
    } else {
      constexpr int E = 16 + w4_epi_vmem<EPI, OUT_F32 || !WIDE>() + ((!OUT_F32 && !WIDE && EPI == EPI_SILU_MUL) ? 16 : 0);
      constexpr int V = E > 63 ? 63 : E;
      __builtin_amdgcn_s_waitcnt((V & 15) | (((V >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
    }
    w4_barrier();
    w4_read(smem, 0, wr, wc, fr, fh, a0, b0);
    __builtin_amdgcn_s_waitcnt(W_LGKM0);
    __builtin_amdgcn_sched_barrier(0);

    int t = 0;
    if constexpr (SCHED >= 2) {  // S1 = barrier-A position, S3 = MFMAs per DMA
      constexpr bool JM = SCHED == 3;
      constexpr int RW = SCHED == 4 ? 4 : 2;  // MFMAs per F0(t+1) read
      for (; t + 2 < nk; ++t)
        w4_iter2<true, true, STAMP, S1, S3, JM, RW>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                            a1, b1, stp);
      if (t + 1 < nk) {
        w4_iter2<false, true, false, S1, S3, JM, RW>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                             a1, b1, stp);
        ++t;
      }
      // last K-tile: barrier A retires every wave's last reads, barrier B follows it
      w4_iter2<false, false, false, S1, S3, JM, RW>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                            a1, b1, stp);
    } else if constexpr (S3 == 0) {
      for (; t + 2 < nk; ++t)
        w4_iter1<true, true, STAMP, S1>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0, a1,
                                        b1, stp);
      if (t + 1 < nk) {
        w4_iter1<false, true, false, S1>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0, a1,
                                         b1, stp);
        ++t;
      }
      w4_iter1<false, false, false, S1>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0, a1,
                                        b1, stp);
      // w4_iter1 has no barrier after its last LDS reads: every wave must be done with them before
      // the next tile's DMAs overwrite the buffers
      w4_barrier();
    } else {
      for (; t + 2 < nk; ++t)
        w4_iter<true, true, STAMP, S1, S3>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                           a1, b1, stp);
      if (t + 1 < nk) {
        w4_iter<false, true, false, S1, S3>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                            a1, b1, stp);
        ++t;
      }
      // last K-tile: its F1 reads retire before its barrier 1, its segment 3 reads nothing, so
      // after its barrier 2 no wave touches LDS again for this tile
      w4_iter<false, false, false, S1, S3>(smem, t, srd_a, srd_b, off_a, off_b, wid, wr, wc, fr, fh, acc, a0, b0,
                                           a1, b1, stp);
    }

    unsigned long long tt1 = 0;
    if constexpr (STAMP) tt1 = __builtin_amdgcn_s_memtime();
    const int next = tile + (int)gridDim.x;
    if (next < nwg) {
      int nm0, nn0;
      w4_origin(next, nwg, tiles_m, tiles_n, nm0, nn0);
      // opaque copy of the lane id: keeps hipcc from hoisting the lane-only half of the offset math
      // out of the tile loop (it did, and spilled those 16 values to scratch at 256 VGPRs)
      int ln;  // == lane, recomputed here (volatile: not hoisted)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      w4_offsets(lda, nm0, M, wid, ln, off_a);
      w4_offsets(ldb, nn0, N, wid, ln, off_b);
      w4_stage(srd_a, off_a, 0, smem, wid);
      w4_stage(srd_b, off_b, 0, smem + W_TILE_A, wid);
      if (nk > 1) {
        w4_stage(srd_a, off_a, WBK, smem + W_BUF, wid);
        w4_stage(srd_b, off_b, WBK, smem + W_BUF + W_TILE_A, wid);
      }
    }
    w4_pin_acc(acc);
    if (m0 + WBM <= M && n0 + WBN <= N) {
      if constexpr (OUT_F32 || !WIDE)
        w4_epilogue_reg<EPI, OUT_F32, true>(acc, wr, wc, fr, fh, m0, n0, C, ldc, bias, resid, ldr, M, N);
      else
        w4_epilogue_wide<EPI>(acc, wr, wc, fr, fh, m0, n0, C, ldc, bias, resid, ldr);
      younger_epi = 1;
    } else {
      w4_epilogue_reg<EPI, OUT_F32, false>(acc, wr, wc, fr, fh, m0, n0, C, ldc, bias, resid, ldr, M, N);
      __builtin_amdgcn_s_waitcnt(W_VM0);  // guarded stores: count unknown, drain them here
      younger_epi = 0;
    }
    ++done;
    if constexpr (STAMP) {
      const unsigned long long tt2 = __builtin_amdgcn_s_memtime();
      tl_loop += tt1 - tt0;
      tl_epi += tt2 - tt1;
    }
    if (next >= nwg) break;
    tile = next;
    w4_origin(tile, nwg, tiles_m, tiles_n, m0, n0);
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = dbg + ((size_t)blockIdx.x * 4 + wid) * 8;
#pragma unroll
      for (int i = 0; i < 5; ++i) d[i] = stp[i];
      d[5] = (unsigned long long)done * (unsigned long long)(nk - 2);  // steady-state iterations
      d[6] = tl_loop;  // per tile: zero + prologue wait + K-loop
      d[7] = tl_epi;   // per tile: next tile's staging + epilogue
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Continuous K-stream variant (gemm_w4c_kernel). The persistent kernel above pays, per output tile,
// ~7.5k cycles of prologue (acc zeroing, waiting for the new tile's first K-tile, reading its first
// fragments with no MFMA to hide behind) plus the next tile's 32 DMA issues inside the ~13k-cycle
// epilogue window (tools/gemm_epi_probe.py: 12-13k cycles per tile at any grid size, so it is issue /
// latency, not the store burst). Here the block's K-tiles form ONE stream across its tiles: the last two
// iterations of tile i stage K-tiles 0 and 1 of tile i+1 (with that tile's row offsets) into the ring
// slots the stream would have used, the last iteration's segment 3 reads tile i+1's first fragments,
// and the first iteration of a tile writes its accumulators with srcC = 0 (no zeroing pass). Between
// the tiles only the register epilogue remains; its stores are counted into the first iteration's
// vmcnt. Ring slot = running K-tile index g & 1 (not t & 1: K-tile counts may be odd).
__device__ __forceinline__ void w4_mfma0(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8], int m) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %1, 0"
               : "=a"(acc[m >> 3][m & 7])
               : "v"(a[m >> 3]), "v"(b[m & 7])
               : "memory");
}

template <bool ZERO>
__device__ __forceinline__ void w4_mfma_z(f32x4 (&acc)[8][8], const bf16x8 (&a0)[8], const bf16x8 (&b0)[8],
                                          const bf16x8 (&a1)[8], const bf16x8 (&b1)[8], int m) {
  if (m < 64) {
    if (ZERO) w4_mfma0(acc, a0, b0, m);
    else w4_mfma(acc, a0, b0, m);
  } else {
    w4_mfma(acc, a1, b1, m - 64);
  }
}

// w4_iter with: ring slot from g, DMA source offsets / K-tile passed in (sa/sb at K-tile kst: this
// tile's t+2 or the next tile's 0 / 1), ZERO = F0 MFMAs start the accumulators, VMW = vmcnt bound at
// the end of segment 2 when a DMA was issued (16 + vector-memory ops issued after the slot's DMA).
template <bool STAGE, bool READ, bool ZERO, int VMW, bool STAMP>
__device__ __forceinline__ void w4_iter_c(char* smem, int g, i32x4 srd_a, i32x4 srd_b, const int (&sa)[8],
                                          const int (&sb)[8], int kst, int wid, int wr, int wc, int fr, int fh,
                                          f32x4 (&acc)[8][8], bf16x8 (&a0)[8], bf16x8 (&b0)[8], bf16x8 (&a1)[8],
                                          bf16x8 (&b1)[8], unsigned long long (&stp)[5]) {
  constexpr int S1 = W4_S1, S3 = W4_S3, N2 = 128 - S1 - S3, DSTEP = N2 / 16;
  static_assert(S1 == 32 && S3 == 16, "continuous schedule uses the production split");
  static_assert(VMW >= 16 && VMW <= 63, "vmcnt bound");
  char* buf = smem + (g & 1) * W_BUF;
  unsigned long long t0 = 0;
  if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int m = 0; m < S1; ++m) {
    if (m < 16) w4_read_frag(buf, 1, m, wr, wc, fr, fh, a1, b1);
    w4_mfma_z<ZERO>(acc, a0, b0, a1, b1, m);
  }
  __builtin_amdgcn_s_waitcnt(W_LGKM0);
  w4_barrier();
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    if constexpr (STAGE) {
      if (i % DSTEP == 0) {
        const int q = i / DSTEP;
        if (q < 8) blds16(srd_a, sa[q], kst * WBK * 2, buf + (wid * 8 + q) * 1024);
        else blds16(srd_b, sb[q - 8], kst * WBK * 2, buf + W_TILE_A + (wid * 8 + q - 8) * 1024);
      }
    }
    w4_mfma_z<ZERO>(acc, a0, b0, a1, b1, S1 + i);
  }
  if constexpr (STAGE) __builtin_amdgcn_s_waitcnt((VMW & 15) | (((VMW >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
  else __builtin_amdgcn_s_waitcnt(W_VM0);
  w4_barrier();
  const char* nbuf = smem + ((g + 1) & 1) * W_BUF;
#pragma unroll
  for (int i = 0; i < S3; ++i) {
    if constexpr (READ) w4_read_frag(nbuf, 0, i, wr, wc, fr, fh, a0, b0);
    w4_mfma_z<false>(acc, a0, b0, a1, b1, 128 - S3 + i);
  }
  if constexpr (STAMP) stp[4] += __builtin_amdgcn_s_memtime() - t0;
}

// ---------------------------------------------------------------------------------------------------
// Three-barrier K-tile schedule (w4_iter_h), the instruction placement of hipBLASLt's gfx950 256x256x64
// kernel as read from its disassembly: per K-tile and wave, 128 MFMAs (m = 8i + j per 32-deep sub-step,
// the activation fragment a[i] held for 8 MFMAs, the weight fragment b[j] cycling) with
//   m  0..14 : 8 reads b1[j] (weights, sub-step 1 of tile t), one per 2 MFMAs
//   m 21/22  : lgkmcnt(0), barrier X        -> every wave is done with the weight half of buffer t&1
//   m 22..58 : 8 weight DMAs of tile t+2 into it; reads a1[i] at m 24..42 between them
//   m 51/52  : lgkmcnt(0), barrier Y        -> the activation half of buffer t&1 is free
//   m 61..125: 8 activation DMAs of tile t+2
//   m 92/93  : vmcnt(13) (the 13 DMAs of this tile are the youngest), barrier: tile t+1 landed
//   m 93..124: the 16 F0 reads of tile t+1 (8 weight, then 8 activation fragments, spread)
//   m 127    : lgkmcnt(0): the next iteration opens on MFMAs whose operands are all in registers.
// What differs from w4_iter: the reads are never bunched one per MFMA (16 ds_read_b128 per 16-cycle
// MFMA gap saturate the CU's LDS with four waves), the F0(t+1) reads start 35 MFMAs (not 16) before
// their first use, and the DMAs start after a barrier that retires only the half of the buffer they
// overwrite. Reads and DMAs are inline asm so hipcc's waitcnt pass adds nothing: the three waits
// above are the only ones in the loop (its lgkmcnt(14)s stalled the head of every w4_iter). M0 is
// set once per DMA group and post-incremented after the next MFMA (no s_nop between M0 and the DMA).
__device__ __forceinline__ void h_read(bf16x8& d, unsigned addr, int off_imm) {
  // off_imm is a compile-time constant at every call site (fully unrolled schedule)
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(off_imm) : "memory");
}
__device__ __forceinline__ void h_dma(i32x4 srd, int voff, int soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(srd), "s"(soff) : "memory");
}
__device__ __forceinline__ void h_m0_set(unsigned lds) { asm volatile("s_mov_b32 m0, %0" ::"s"(lds) : "memory"); }
__device__ __forceinline__ void h_m0_inc() { asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory"); }

// DMA slots (MFMA index after which piece q is issued) and read slots of the schedule above
constexpr int H_DX[8] = {22, 25, 28, 31, 34, 52, 55, 58};     // weight pieces (operand B)
constexpr int H_DY[8] = {61, 64, 85, 87, 89, 96, 99, 125};    // activation pieces (operand A)
constexpr int H_RB1[8] = {0, 2, 4, 6, 8, 10, 12, 14};         // b1[j]
constexpr int H_RA1[8] = {24, 27, 30, 33, 36, 38, 40, 42};    // a1[i]
constexpr int H_RB0[8] = {93, 94, 95, 97, 98, 100, 101, 102}; // b0[j] of tile t+1
constexpr int H_RA0[8] = {104, 107, 110, 113, 116, 119, 121, 123};  // a0[i] of tile t+1
constexpr int H_VM = 13;  // DMAs of this iteration issued before the m = 92 wait

constexpr int h_find(const int (&s)[8], int m) {
  for (int q = 0; q < 8; ++q)
    if (s[q] == m) return q;
  return -1;
}

// One K-tile of the continuous kernel in the three-barrier schedule. g = running K-tile index (ring
// slot g & 1); sa / sb = DMA source offsets at K-tile kst (this tile's t+2 or the next tile's 0 / 1);
// ZERO = the F0 MFMAs start the accumulators (srcC = 0); VMW = the m = 92 vmcnt bound (H_VM plus the
// vector-memory ops issued between the previous iteration's DMAs and this one's, i.e. an epilogue).
// rbA / rbB: this lane's read bases (sub-step s, buffer 0) for the activation / weight fragments.
template <bool ZERO, int VMW>
__device__ __forceinline__ void w4_iter_h(char* smem, int g, i32x4 srd_a, i32x4 srd_b, const int (&sa)[8],
                                          const int (&sb)[8], int kst, int wid, const unsigned (&rbA)[2],
                                          const unsigned (&rbB)[2], f32x4 (&acc)[8][8], bf16x8 (&a0)[8],
                                          bf16x8 (&b0)[8], bf16x8 (&a1)[8], bf16x8 (&b1)[8]) {
  static_assert(VMW >= H_VM && VMW <= 63, "vmcnt bound");
  const unsigned cur = (unsigned)(g & 1) * W_BUF, nxt = (unsigned)((g + 1) & 1) * W_BUF;
  const unsigned lds_cur = (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)smem + cur;
  const unsigned mX = __builtin_amdgcn_readfirstlane(lds_cur + W_TILE_A + wid * 8192);  // weight pieces
  const unsigned mY = __builtin_amdgcn_readfirstlane(lds_cur + wid * 8192);             // activation pieces
  const int kb = kst * WBK * 2;
  const unsigned rb1 = rbB[1] + cur, ra1 = rbA[1] + cur, rb0 = rbB[0] + nxt, ra0 = rbA[0] + nxt;
  static_for<128>([&](auto mc) __attribute__((always_inline)) {
    constexpr int m = decltype(mc)::value;
    if constexpr (m == 21) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (m == 22 || m == 52) w4_barrier();
    if constexpr (m == 92) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMW) : "memory");
    }
    if constexpr (m == 93) w4_barrier();
    if constexpr (m == 51 || m == 127) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // MFMA m
    if constexpr (m < 64) {
      if constexpr (ZERO) w4_mfma0(acc, a0, b0, m);
      else w4_mfma(acc, a0, b0, m);
    } else {
      w4_mfma(acc, a1, b1, m - 64);
    }
    // post-increment M0 one MFMA after each piece; M0 for a DMA group one MFMA (or more) ahead of its
    // first piece
    if constexpr (h_find(H_DX, m - 1) >= 0 || h_find(H_DY, m - 1) >= 0) h_m0_inc();
    if constexpr (m == 21) h_m0_set(mX);
    if constexpr (m == 59) h_m0_set(mY);
    constexpr int qx = h_find(H_DX, m), qy = h_find(H_DY, m);
    if constexpr (qx >= 0) h_dma(srd_b, sb[qx], kb);
    if constexpr (qy >= 0) h_dma(srd_a, sa[qy], kb);
    constexpr int r1b = h_find(H_RB1, m), r1a = h_find(H_RA1, m), r0b = h_find(H_RB0, m), r0a = h_find(H_RA0, m);
    if constexpr (r1b >= 0) h_read(b1[r1b], rb1, r1b * 2048);
    if constexpr (r1a >= 0) h_read(a1[r1a], ra1, r1a * 2048);
    if constexpr (r0b >= 0) h_read(b0[r0b], rb0, r0b * 2048);
    if constexpr (r0a >= 0) h_read(a0[r0a], ra0, r0a * 2048);
  });
}

// Requires K / 64 >= 4 (the launcher falls back to gemm_w4_kernel below that).
// KSPLIT: split-K over nsplit K-slabs of K columns each in ONE persistent launch -- work item
// t = z * tiles + tile writes the fp32 partial tile of slab z to C + z * M * ldc (the consumer, e.g.
// add_partials_rmsnorm, sums the slabs). For prefill shapes whose 256x256 tile count fills only
// ~1.3 waves of the CUs (o_proj / down at M ~ 5k: 336 tiles on 256 CUs), two slabs make 2.6 waves.
template <int EPI, bool OUT_F32, bool STAMP = false, bool KSPLIT = false, bool H = false>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4c_kernel(const bf16_t* __restrict__ A, int lda,
                                                                 const bf16_t* __restrict__ B, int ldb, void* C,
                                                                 int ldc, const bf16_t* __restrict__ bias,
                                                                 const bf16_t* resid, int ldr, int M, int N, int K,
                                                                 unsigned long long* dbg, int nsplit = 1) {
  __shared__ __attribute__((aligned(16))) char smem[W4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fh = lane >> 4;
  const int tiles_m = (M + WBM - 1) / WBM, tiles_n = (N + WBN - 1) / WBN;
  const int nwg = tiles_m * tiles_n;
  const int nwt = KSPLIT ? nwg * nsplit : nwg;  // work items
  const int nk = K / WBK;
  const i32x4 srd_a = make_srd(A, (unsigned)M * (unsigned)lda * 2u);
  const i32x4 srd_b = make_srd(B, (unsigned)N * (unsigned)ldb * 2u);

  // epilogue vector-memory ops younger than the next tile's K-tile-1 DMA at its first vmcnt
  constexpr int EV = w4_epi_vmem<EPI, OUT_F32 || !W4_WIDE_EPI>() +
                     ((!OUT_F32 && !W4_WIDE_EPI && EPI == EPI_SILU_MUL) ? 16 : 0);
  constexpr int VMW0 = 16 + EV > 63 ? 63 : 16 + EV;

  int tile = blockIdx.x;
  int z = KSPLIT ? tile / nwg : 0;
  int m0, n0;
  w4_origin(tile - z * nwg, nwg, tiles_m, tiles_n, m0, n0);
  int off_a[8], off_b[8];
  w4_offsets(lda, m0, M, wid, lane, off_a);
  w4_offsets(ldb, n0, N, wid, lane, off_b);
  if constexpr (KSPLIT) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      off_a[i] += z * K * 2;
      off_b[i] += z * K * 2;
    }
  }
  w4_stage(srd_a, off_a, 0, smem, wid);
  w4_stage(srd_b, off_b, 0, smem + W_TILE_A, wid);
  w4_stage(srd_a, off_a, WBK, smem + W_BUF, wid);
  w4_stage(srd_b, off_b, WBK, smem + W_BUF + W_TILE_A, wid);
  __builtin_amdgcn_s_waitcnt(W_VM0);  // K-tiles 0 and 1: the first iteration's vmcnt then only covers K-tile 2
  w4_barrier();
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  w4_read(smem, 0, wr, wc, fr, fh, a0, b0);
  __builtin_amdgcn_s_waitcnt(W_LGKM0);
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[8][8];
  unsigned long long stp[5] = {0, 0, 0, 0, 0};
  unsigned long long tl_loop = 0, tl_epi = 0;
  // w4_iter_h read bases (buffer 0): fragment i / j of sub-step s at base[s] + 2048 i (swizzle independent of i)
  unsigned rbA[2], rbB[2];
  {
    const unsigned l0 = (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)smem;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const unsigned cs = (unsigned)(((4 * s2 + fh) ^ ((fr >> 1) & 7)) * 16);
      rbA[s2] = l0 + (unsigned)((wr * 128 + fr) * 128) + cs;
      rbB[s2] = l0 + W_TILE_A + (unsigned)((wc * 128 + fr) * 128) + cs;
    }
  }
  constexpr int VMH0 = H_VM + EV > 63 ? 63 : H_VM + EV;
  int g = 0, done = 0;
  for (;;) {
    unsigned long long tt0 = 0;
    if constexpr (STAMP) tt0 = __builtin_amdgcn_s_memtime();
    const int next = tile + (int)gridDim.x;
    const bool has_next = next < nwt;
    if constexpr (H)
      w4_iter_h<true, VMH0>(smem, g, srd_a, srd_b, off_a, off_b, 2, wid, rbA, rbB, acc, a0, b0, a1, b1);
    else
      w4_iter_c<true, true, true, VMW0, false>(smem, g, srd_a, srd_b, off_a, off_b, 2, wid, wr, wc, fr, fh, acc, a0,
                                               b0, a1, b1, stp);
    ++g;
    for (int t = 1; t + 2 < nk; ++t, ++g) {
      if constexpr (H)
        w4_iter_h<false, H_VM>(smem, g, srd_a, srd_b, off_a, off_b, t + 2, wid, rbA, rbB, acc, a0, b0, a1, b1);
      else
        w4_iter_c<true, true, false, 16, STAMP>(smem, g, srd_a, srd_b, off_a, off_b, t + 2, wid, wr, wc, fr, fh, acc,
                                                a0, b0, a1, b1, stp);
    }
    // The last two iterations stage (and read the first fragments of) the next tile; on the block's
    // last tile they re-stage this tile's K-tiles 0 / 1 instead (valid addresses, never read), so both
    // cases run the same straight-line code: a branch around the MFMA iterations made the register
    // allocator split the accumulators across the two paths and spill them.
    int nm0, nn0;
    const int ntile = has_next ? next : tile;
    const int nz = KSPLIT ? ntile / nwg : 0;
    w4_origin(ntile - nz * nwg, nwg, tiles_m, tiles_n, nm0, nn0);
    {
      int ln;  // == lane; opaque so the lane-only offset math is not hoisted out of the loop
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      // this tile's DMAs are all issued: its offset registers take the next tile's
      w4_offsets(lda, nm0, M, wid, ln, off_a);
      w4_offsets(ldb, nn0, N, wid, ln, off_b);
      if constexpr (KSPLIT) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          off_a[i] += nz * K * 2;
          off_b[i] += nz * K * 2;
        }
      }
    }
    if constexpr (H) {
      w4_iter_h<false, H_VM>(smem, g, srd_a, srd_b, off_a, off_b, 0, wid, rbA, rbB, acc, a0, b0, a1, b1);
      ++g;
      w4_iter_h<false, H_VM>(smem, g, srd_a, srd_b, off_a, off_b, 1, wid, rbA, rbB, acc, a0, b0, a1, b1);
      ++g;
    } else {
      w4_iter_c<true, true, false, 16, false>(smem, g, srd_a, srd_b, off_a, off_b, 0, wid, wr, wc, fr, fh, acc, a0,
                                              b0, a1, b1, stp);
      ++g;
      w4_iter_c<true, true, false, 16, false>(smem, g, srd_a, srd_b, off_a, off_b, 1, wid, wr, wc, fr, fh, acc, a0,
                                              b0, a1, b1, stp);
      ++g;
    }
    unsigned long long tt1 = 0;
    if constexpr (STAMP) tt1 = __builtin_amdgcn_s_memtime();
    w4_pin_acc(acc);
    void* Cz = KSPLIT ? (void*)(reinterpret_cast<float*>(C) + (size_t)z * M * ldc) : C;
    if (m0 + WBM <= M && n0 + WBN <= N) {
      if constexpr (OUT_F32 || !W4_WIDE_EPI)
        w4_epilogue_reg<EPI, OUT_F32, true>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr, M, N);
      else
        w4_epilogue_wide<EPI>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr);
    } else {
      w4_epilogue_reg<EPI, OUT_F32, false>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr, M, N);
      __builtin_amdgcn_s_waitcnt(W_VM0);  // guarded: count unknown, drain (the next K-tile 1 lands too)
    }
    // epilogue accumulator reads -> the next tile's srcC = 0 MFMA writes
    asm volatile("s_nop 7" ::: "memory");
    ++done;
    if constexpr (STAMP) {
      const unsigned long long tt2 = __builtin_amdgcn_s_memtime();
      tl_loop += tt1 - tt0;
      tl_epi += tt2 - tt1;
    }
    if (!has_next) {
      __builtin_amdgcn_s_waitcnt(W_VM0);  // the re-staged K-tiles land before the block's LDS is released
      break;
    }
    tile = next;
    m0 = nm0;
    n0 = nn0;
    z = nz;
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* d = dbg + ((size_t)blockIdx.x * 4 + wid) * 8;
#pragma unroll
      for (int i = 0; i < 5; ++i) d[i] = stp[i];
      d[5] = (unsigned long long)done * (unsigned long long)(nk - 3);  // stamped steady-state iterations
      d[6] = tl_loop;
      d[7] = tl_epi;
    }
  }
}

// Persistent grid: one block per CU (the kernel holds 128 KiB of LDS and 4 waves x 512 registers,
// so a CU never runs two), rounded down to a multiple of 8 so a block keeps its XCD across tiles.
// RAGK_W4_GRID=0 launches one block per tile instead (A/B), N > 0 caps the grid at N.
static int g_w4_grid = -1;
static int w4_grid(int nwg) {
  if (g_w4_grid < 0) {
    const char* e = getenv("RAGK_W4_GRID");
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    g_w4_grid = e ? atoi(e) : (cus / 8) * 8;
    if (g_w4_grid < 0) g_w4_grid = 0;
  }
  return (g_w4_grid == 0 || g_w4_grid >= nwg) ? nwg : g_w4_grid;
}

// K-loop schedule by K (tools/gemm_sched_ab.py, profiles/gemm_sched_ab_r2.txt): long K (the down
// projection, K = 14336) runs the spread schedule w4_iter2 (F1 reads in the first 16 MFMAs, one DMA
// per 7 MFMAs, F0(t+1) reads one per 4 MFMAs; -2.6 %), K = 4096 the S1/S3 split (within 1 %).
static int g_w4_sched_k = -1;
static int w4_sched_min_k() {
  if (g_w4_sched_k < 0) {
    const char* e = getenv("RAGK_W4_SPREAD_MIN_K");
    g_w4_sched_k = e ? atoi(e) : 8192;
  }
  return g_w4_sched_k;
}

// Continuous K-stream kernel for K < the spread-schedule threshold (RAGK_W4_CONT=0 -> gemm_w4_kernel).
// 2 = the continuous kernel with the three-barrier schedule (w4_iter_h) for every K.
static int g_w4_cont = -1;
static int w4_cont() {
  if (g_w4_cont < 0) {
    const char* e = getenv("RAGK_W4_CONT");
    g_w4_cont = e ? atoi(e) : 1;
  }
  return g_w4_cont;
}

template <int EPI, bool F32>
int launch_w4(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias, const void* resid,
              int ldr, int M, int N, int K, hipStream_t st) {
  const int nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  const int grid = w4_grid(nwg);
  if (K / WBK >= 4 && w4_cont() == 2)
    hipLaunchKernelGGL((gemm_w4c_kernel<EPI, F32, false, false, true>), dim3(grid), dim3(W4_THREADS), 0, st,
                       (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid,
                       ldr, M, N, K, nullptr);
  else if (K < w4_sched_min_k() && K / WBK >= 4 && w4_cont())
    hipLaunchKernelGGL((gemm_w4c_kernel<EPI, F32>), dim3(grid), dim3(W4_THREADS), 0, st, (const bf16_t*)A, lda,
                       (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K,
                       nullptr);
  else if (K >= w4_sched_min_k())
    hipLaunchKernelGGL((gemm_w4_kernel<EPI, F32, false, 16, 7, 4>), dim3(grid), dim3(W4_THREADS), 0, st,
                       (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid,
                       ldr, M, N, K, nullptr);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<EPI, F32>), dim3(grid), dim3(W4_THREADS), 0, st, (const bf16_t*)A, lda,
                       (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K,
                       nullptr);
  return (int)hipGetLastError();
}

}  // namespace

// Persistent-grid override (tests / A/B): 0 = one block per tile, g > 0 = at most g blocks (a
// multiple of 8 keeps each block on one XCD), < 0 = back to the CU count.
RAGK_API int ragk_gemm_w4_set_grid(int g) {
  g_w4_grid = g < 0 ? -1 : g;
  return 0;
}

// Continuous-K-stream override (tests / A/B): 1 = gemm_w4c_kernel for K < the spread threshold, 0 = off,
// < 0 = back to RAGK_W4_CONT / the default (on).
RAGK_API int ragk_gemm_w4_set_cont(int on) {
  g_w4_cont = on < 0 ? -1 : on;
  return 0;
}

// N = output columns (for EPI_SILU_MUL the weight has 2N rows, N % 128 == 0). Requires K % 64 == 0.
RAGK_API int ragk_gemm_w4(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                          const void* resid, int ldr, int M, int N, int K, int epi, int out_f32, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % WBK != 0) return (int)hipErrorInvalidValue;
  const long long rows_b = (epi == EPI_SILU_MUL) ? 2LL * N : (long long)N;
  if ((long long)M * lda * 2 >= (1LL << 31) || rows_b * ldb * 2 >= (1LL << 31))
    return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  if (epi == EPI_SILU_MUL) {
    if (N % 128 != 0 || out_f32) return (int)hipErrorInvalidValue;
    return launch_w4<EPI_SILU_MUL, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, 2 * N, K, st);
  }
  if (N % 8 != 0) return (int)hipErrorInvalidValue;
#define RAGK_W4_CASE(E) \
  case E:               \
    return out_f32 ? launch_w4<E, true>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st) \
                   : launch_w4<E, false>(A, lda, B, ldb, C, ldc, bias, resid, ldr, M, N, K, st);
  switch (epi) {
    RAGK_W4_CASE(EPI_NONE)
    RAGK_W4_CASE(EPI_BIAS)
    RAGK_W4_CASE(EPI_RESID)
    RAGK_W4_CASE(EPI_BIAS_RESID)
    RAGK_W4_CASE(EPI_BIAS_GELU)
    RAGK_W4_CASE(EPI_GELU)
    RAGK_W4_CASE(EPI_BIAS_GELU_TANH)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef RAGK_W4_CASE
}

// Split-K prefill GEMM into fp32 slabs: P[z][M][N] = A[:, z*Ks:(z+1)*Ks] . B[:, z*Ks:(z+1)*Ks]^T,
// Ks = K / nsplit, one persistent gemm_w4c launch over nsplit x tiles work items (see KSPLIT).
RAGK_API int ragk_gemm_w4_splitk(const void* A, int lda, const void* B, int ldb, float* P, int M, int N, int K,
                                 int nsplit, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (nsplit < 1 || K % nsplit || (K / nsplit) % WBK || (K / nsplit) / WBK < 4 || N % 8 || !P)
    return (int)hipErrorInvalidValue;
  if ((long long)M * lda * 2 >= (1LL << 31) || (long long)N * ldb * 2 >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  hipLaunchKernelGGL((gemm_w4c_kernel<EPI_NONE, true, false, true>), dim3(w4_grid(nwg * nsplit)), dim3(W4_THREADS), 0,
                     st, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, (void*)P, N, nullptr, nullptr, 0, M, N,
                     K / nsplit, nullptr, nsplit);
  return (int)hipGetLastError();
}

// Diagnostic / tuning builds of the EPI_NONE kernel (tools/gemm_stamps.py). variant selects the
// segment split (S1, S3); stamp != 0 adds s_memtime stamps around the K-loop segments, dbg:
// [nwg][4 waves][8] u64 = seg1, barrier1, seg2, barrier2, whole iteration (sums over the
// steady-state iterations), iteration count, per-tile K-loop cycles, per-tile epilogue cycles (sums).
template <bool STAMP, int S1, int S3, int SCHED = 0, bool WIDE = W4_WIDE_EPI>
int launch_w4_diag(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                   unsigned long long* dbg, hipStream_t st) {
  const int nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_NONE, false, STAMP, S1, S3, SCHED, WIDE>), dim3(w4_grid(nwg)), dim3(W4_THREADS), 0, st,
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, nullptr, nullptr, 0, M, N, K, dbg);
  return (int)hipGetLastError();
}

RAGK_API int ragk_gemm_w4_diag(int variant, int stamp, const void* A, int lda, const void* B, int ldb, void* C,
                               int ldc, int M, int N, int K, unsigned long long* dbg, hipStream_t st) {
  if (K % WBK != 0 || N % 8 != 0 || (long long)M * lda * 2 >= (1LL << 31) || (long long)N * ldb * 2 >= (1LL << 31))
    return (int)hipErrorInvalidValue;
  if (stamp && dbg == nullptr) return (int)hipErrorInvalidValue;
#define RAGK_W4D(V, S1, S3)                                                                                  \
  case V:                                                                                                    \
    return stamp ? launch_w4_diag<true, S1, S3>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)                    \
                 : launch_w4_diag<false, S1, S3>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
#define RAGK_W4D2(V, BA, DS)                                                                               \
  case V:                                                                                                  \
    return stamp ? launch_w4_diag<true, BA, DS, 2>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)                \
                 : launch_w4_diag<false, BA, DS, 2>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
  switch (variant) {
    RAGK_W4D(0, 32, 16)
    RAGK_W4D(1, 24, 24)
    RAGK_W4D(2, 40, 24)
    RAGK_W4D(3, 32, 32)
    RAGK_W4D(4, 48, 16)
    RAGK_W4D(5, 56, 24)
    RAGK_W4D(6, 32, 0)
    RAGK_W4D(7, 24, 0)
    RAGK_W4D(8, 40, 0)
    RAGK_W4D2(9, 32, 4)
    RAGK_W4D2(10, 32, 5)
    RAGK_W4D2(11, 32, 6)
    RAGK_W4D2(12, 48, 4)
    RAGK_W4D2(13, 16, 6)
    case 14:  // production schedule with the 8-byte-store epilogue (A/B of the widened one)
      return stamp ? launch_w4_diag<true, 32, 16, 0, false>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 16, 0, false>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 16:  // w4_iter2 (32, 6), j-major MFMA order
      return stamp ? launch_w4_diag<true, 32, 6, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 6, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 17:  // w4_iter2 (32, 4), j-major MFMA order
      return stamp ? launch_w4_diag<true, 32, 4, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 4, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 18:
      return stamp ? launch_w4_diag<true, 32, 6, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 6, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 19:
      return stamp ? launch_w4_diag<true, 32, 4, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 4, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 20:
      return stamp ? launch_w4_diag<true, 16, 7, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 16, 7, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 21:
      return stamp ? launch_w4_diag<true, 48, 5, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 48, 5, 4, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    case 22:  // continuous K-stream kernel (production for K < 8192)
    {
      if (K / WBK < 4) return (int)hipErrorInvalidValue;
      const dim3 grid(w4_grid(((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN)));
      if (stamp)
        hipLaunchKernelGGL((gemm_w4c_kernel<EPI_NONE, false, true>), grid, dim3(W4_THREADS), 0, st, (const bf16_t*)A,
                           lda, (const bf16_t*)B, ldb, C, ldc, nullptr, nullptr, 0, M, N, K, dbg);
      else
        hipLaunchKernelGGL((gemm_w4c_kernel<EPI_NONE, false, false>), grid, dim3(W4_THREADS), 0, st,
                           (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, nullptr, nullptr, 0, M, N, K, dbg);
      return (int)hipGetLastError();
    }
    case 15:  // w4_iter2 (32, 6) + widened epilogue
      return stamp ? launch_w4_diag<true, 32, 6, 2, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st)
                   : launch_w4_diag<false, 32, 6, 2, true>(A, lda, B, ldb, C, ldc, M, N, K, dbg, st);
    default:
      return (int)hipErrorInvalidValue;
  }
#undef RAGK_W4D
#undef RAGK_W4D2
}
