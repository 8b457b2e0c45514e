// 256x256x64 bf16 GEMM for the large-M prefill projections: 4 waves x (128x128) per workgroup, one
// wave per SIMD, one persistent workgroup per CU streaming its tiles' K-tiles as ONE continuous ring.
//
// C[M,N] = A[M,K] . B[N,K]^T (+ fused epilogue: bias / residual / GELU / SiLU*up / fp32 split-K slabs).
// A = activations (row-major, K contiguous), B = weights (nn.Linear layout [N][K]).
//
// Per K-tile (64 deep) and wave: 128 v_mfma_f32_16x16x32_bf16 into 8 x 8 accumulators (256 AGPRs),
// 16 LDS-DMA pieces (buffer_load_dwordx4 ... lds, 1 KiB each) of K-tile t+2 and 32 ds_read_b128
// fragment reads. Two 64 KiB LDS buffers (tile t & 1), lane-linear image, source-swizzled.
//
// K-loop schedule (w4_iter_h, the placement of hipBLASLt's gfx950 256x256x64 direct-to-LDS kernel as
// read from its disassembly, rebuilt here with our LDS image and epilogues): three barriers per K-tile,
// one per LDS hazard -- the weight half of buffer t&1 free (DMAs of t+2 may start), the activation half
// free, tile t+1 landed -- with the fragment reads spread one per 2-3 MFMAs (four waves reading one
// fragment per 16-cycle MFMA gap saturate the CU's LDS) and the next tile's first fragments read
// 35 MFMAs before their use. Reads, DMAs and the three waits are inline asm, so hipcc's waitcnt pass
// adds none of its own (its lgkmcnt(14)s stalled the head of every K-tile of the previous schedule).
// Measured against the previous two-barrier schedule (same box, M = 32768, profiles/gemm_probe_r5*.log):
// qkv 1140 -> 1103 us, o_proj+resid 810 -> 796, gate/up+SiLU 5218 -> 5173, down+resid 2709 -> 2602.
//
// Continuous K-stream: the last two iterations of tile i stage K-tiles 0 and 1 of tile i+1 (its own
// row offsets) into the ring slots the stream would have used, the last iteration reads tile i+1's
// first fragments, and the first iteration of a tile writes its accumulators with srcC = 0. Between
// two tiles only the register epilogue remains; its memory ops are counted into the first iteration's
// vmcnt. The grid is one block per CU (multiple of 8: a block keeps its XCD), tiles numbered so each
// XCD owns a contiguous range grouped WGROUP_M M-tiles deep (the XCD's L2 reuses the weight panels).
//
// Epilogue: the weight rows are loaded in a permuted order (w4_perm) so that each lane's accumulators
// of tiles j, j+1 hold EIGHT consecutive output columns: every bf16 store (and residual / bias load)
// is one 16-byte access straight from registers.
//
// Build note: this file is compiled with `-mllvm -disable-post-ra` (_build.py EXTRA_FLAGS): the loop
// is written in its final instruction order and the post-RA scheduler bunched the DMAs.
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
constexpr int W4_MIN_KT = 3;  // K-tiles per tile the continuous ring needs (K >= 192)

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

// Weight-row permutation inside each 128-row wave tile: LDS row q (MFMA tile j = q >> 4, column
// c = q & 15 = 4 fh + k) holds global row w4_perm(q) = 32 (j >> 1) + 8 fh + 4 (j & 1) + k. With the
// weight fragment as srcA the accumulator comes out transposed (lane (fr, fh) of acc[i][j] holds four
// consecutive output columns of row 16 i + fr), so after the permutation the lane's columns of tiles
// j and j + 1 (j even) are eight consecutive output columns. For the packed gate/up weight
// ([64 gate | 64 up] per 128 rows) gate tile j and up tile j + 4 still map to the same output columns.
__device__ __forceinline__ int w4_perm(int q) {
  const int j = q >> 4, fh = (q >> 2) & 3, k = q & 3;
  return 32 * (j >> 1) + 8 * fh + 4 * (j & 1) + k;
}

// 256 rows x 128 B = 32 pieces of 8 rows; wave w stages pieces 8w..8w+7 of each operand. Per-lane
// byte offsets of those 8 pieces (row clamped to the last valid row, chunk source-swizzled; PERM: the
// weight operand's rows in w4_perm order within each 128-row half).
template <bool PERM>
__device__ __forceinline__ void w4_offsets(int ld, int row0, int rows_valid, int wid, int lane, int (&off)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = (wid * 8 + i) * 8 + (lane >> 3);
    const int c = wswz(r, lane & 7);
    int gr = row0 + (PERM ? (r & ~127) + w4_perm(r & 127) : r);
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

// fragments of one 32-deep sub-step (prologue only): A rows wr*128 + 16i + fr, B rows wc*128 + 16j + fr
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

// MFMA #m (= 8i + j) of a sub-step. Inline asm with the accumulator tied in an AGPR ("+a"): with the
// builtin, hipcc picks dst != srcC for the loop-carried accumulators and adds 84-500 v_accvgpr copies
// per K-tile. volatile + "memory" keep the statement in source order relative to the LDS reads and
// DMAs around it. Hazards the compiler no longer pads: acc init -> first MFMA and last MFMA ->
// epilogue reads (w4_pin_acc below). The weight fragment is srcA and the activation fragment srcB, so
// the accumulator comes out transposed: lane (fr, fh) of acc[i][j] holds C[16i + fr][4 consecutive
// output columns] (which ones: w4_perm).
__device__ __forceinline__ void w4_mfma(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8], int m) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %1, %0"
               : "+a"(acc[m >> 3][m & 7])
               : "v"(a[m >> 3]), "v"(b[m & 7])
               : "memory");
}
// the same with srcC = 0 (first K-tile of a tile: no zeroing pass)
__device__ __forceinline__ void w4_mfma0(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8], int m) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %1, 0"
               : "=a"(acc[m >> 3][m & 7])
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

// ---------------------------------------------------------------------------------------------------
// Epilogue, straight from the accumulators (no LDS, no barrier: LDS already holds the next tile's first
// K-tiles). FULL: the tile lies inside [M, N], no guards, exactly w4_epi_vmem vector-memory ops per wave
// (the next tile's first vmcnt counts them). Loads are never predicated (edge tiles clamp addresses):
// a load under a branch makes hipcc's waitcnt pass drain vmcnt(0) at every join. resid may alias C:
// every element is read and written by the same lane.
constexpr bool epi_res(int e) { return e == EPI_RESID || e == EPI_BIAS_RESID; }
constexpr bool epi_bias(int e) {
  return e == EPI_BIAS || e == EPI_BIAS_RESID || e == EPI_BIAS_GELU || e == EPI_BIAS_GELU_TANH;
}

template <int EPI, bool OUT_F32>
constexpr int w4_epi_vmem() {
  if constexpr (EPI == EPI_ROPE_KV) return 63;    // loads + stores over the counter's range: the bound clamps
  if constexpr (EPI == EPI_SILU_MUL) return 16;  // 8 rows x 2 pairs of 16-B stores
  if constexpr (OUT_F32) return 64 + (epi_res(EPI) ? 64 : 0) + (epi_bias(EPI) ? 8 : 0);
  return 32 + (epi_res(EPI) ? 32 : 0) + (epi_bias(EPI) ? 4 : 0);
}

template <int EPI>
__device__ __forceinline__ float w4_act(float v) {
  if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_GELU) return gelu_erf(v);
  if constexpr (EPI == EPI_BIAS_GELU_TANH) return gelu_tanh(v);
  return v;
}

__device__ __forceinline__ void unpack4(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

// Full tile, bf16 output: per row 16i + fr and column pair p (tiles 2p, 2p+1), eight consecutive
// columns n0 + wc*128 + 32p + 8fh .. +7, one 16-B store (SiLU*up: gate pair (2p, 2p+1), up pair
// (2p+4, 2p+5), output columns (n0 >> 1) + wc*64 + 32p + 8fh).
template <int EPI>
__device__ __forceinline__ void w4_epilogue_full_bf16(const f32x4 (&acc)[8][8], int wr, int wc, int fr, int fh,
                                                      int m0, int n0, void* C, int ldc,
                                                      const bf16_t* __restrict__ bias, const bf16_t* resid, int ldr) {
  const int row0 = m0 + wr * 128 + fr;
  bf16_t* Cb = reinterpret_cast<bf16_t*>(C);
  if constexpr (EPI == EPI_SILU_MUL) {
    const int colw = (n0 >> 1) + wc * 64 + 8 * fh;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = silu(acc[i][2 * p][k]) * acc[i][2 * p + 4][k];
          o[4 + k] = silu(acc[i][2 * p + 1][k]) * acc[i][2 * p + 5][k];
        }
        *reinterpret_cast<u32x4*>(Cb + (size_t)(row0 + 16 * i) * ldc + colw + 32 * p) = pack8(o);
        // one 8-column group at a time: interleaving all 16 groups' VALU raised the register peak past
        // the budget (spills, and a vmcnt(0) drain per tile for the reload)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    constexpr bool RES = epi_res(EPI), BIAS = epi_bias(EPI);
    const int colw = n0 + wc * 128 + 8 * fh;
    u32x4 bv[BIAS ? 4 : 1];
    if constexpr (BIAS) {
#pragma unroll
      for (int p = 0; p < 4; ++p) bv[p] = *reinterpret_cast<const u32x4*>(bias + colw + 32 * p);
    }
    u32x4 rv[RES ? 32 : 1];
    if constexpr (RES) {  // the lane's whole residual tile in flight before the first use
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int p = 0; p < 4; ++p)
          rv[4 * i + p] = *reinterpret_cast<const u32x4*>(resid + (size_t)(row0 + 16 * i) * ldr + colw + 32 * p);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = acc[i][2 * p][k];
          o[4 + k] = acc[i][2 * p + 1][k];
        }
        if constexpr (BIAS) {
          float b[8];
          unpack8(bv[p], b);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += b[k];
        }
        if constexpr (RES) {
          float r[8];
          unpack8(rv[4 * i + p], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = w4_act<EPI>(o[k]);
        *reinterpret_cast<u32x4*>(Cb + (size_t)(row0 + 16 * i) * ldc + colw + 32 * p) = pack8(o);
      }
    }
  }
}

// EPI_ROPE_KV: the qkv projection's epilogue does rope_kv's work (norm.hip rope_kv_kernel, the same bf16
// rounding of every op, the same cos / sin tables: bit-identical): a wave's 128 columns are one head; lane
// (fr, fh) holds, per row, columns 8fh + 32p + 0..7 (p = 0..3), so the rotate_half pairs d / d + 64 are
// p / p + 2 of the same lane. q heads: rotated into C; k heads: rotated into C and the paged cache at the
// row's slot; v heads: C and the cache. Rows two at a time (cos / sin in registers: 64 values), loads
// never predicated (rows past M clamp; only the stores are guarded).
struct RopeKV {
  const int* pos;
  const int* slot;
  const float* cos_t;  // [positions][64]
  const float* sin_t;
  bf16_t* kc;          // [blocks][Hkv][BS][128]
  bf16_t* vc;
  int Hq, Hkv, BS;
};

template <bool FULL>
__device__ __forceinline__ void w4_epilogue_rope(const f32x4 (&acc)[8][8], int wr, int wc, int fr, int fh, int m0,
                                                 int n0, bf16_t* C, int ldc, const RopeKV& rk, int M) {
  const int row0 = m0 + wr * 128 + fr;
  const int hd = (n0 + wc * 128) >> 7;
  const int d0 = 8 * fh;
  const bool isq = hd < rk.Hq, isk = !isq && hd < rk.Hq + rk.Hkv, rot = hd < rk.Hq + rk.Hkv;
  const int kvh = isk ? hd - rk.Hq : hd - rk.Hq - rk.Hkv;
  bf16_t* cache = isk ? rk.kc : rk.vc;
  int pos[8], slot[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = FULL ? row0 + 16 * i : min(row0 + 16 * i, M - 1);
    pos[i] = rk.pos[r];
    slot[i] = rk.slot[r];
  }
#pragma unroll
  for (int i2 = 0; i2 < 8; i2 += 2) {
    u32x4 cv[2][2][2], sv[2][2][2];  // [row][p][half]
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float* ct = rk.cos_t + (size_t)pos[i2 + u] * 64 + d0 + 32 * p;
        const float* st = rk.sin_t + (size_t)pos[i2 + u] * 64 + d0 + 32 * p;
        cv[u][p][0] = *reinterpret_cast<const u32x4*>(ct);
        cv[u][p][1] = *reinterpret_cast<const u32x4*>(ct + 4);
        sv[u][p][0] = *reinterpret_cast<const u32x4*>(st);
        sv[u][p][1] = *reinterpret_cast<const u32x4*>(st + 4);
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i2 + u;
      const int gr = row0 + 16 * i;
      float o[4][8];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[p][k] = bf2f(f2bf(acc[i][2 * p][k]));
          o[p][4 + k] = bf2f(f2bf(acc[i][2 * p + 1][k]));
        }
      if (rot) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float c = __uint_as_float(cv[u][p][k >> 2][k & 3]), sn = __uint_as_float(sv[u][p][k >> 2][k & 3]);
            const float x1 = o[p][k], x2 = o[p + 2][k];
            o[p][k] = bf2f(f2bf(bf2f(f2bf(x1 * c)) + bf2f(f2bf(-x2 * sn))));
            o[p + 2][k] = bf2f(f2bf(bf2f(f2bf(x2 * c)) + bf2f(f2bf(x1 * sn))));
          }
      }
      if (FULL || gr < M) {
        bf16_t* crow = C + (size_t)gr * ldc + n0 + wc * 128 + d0;
#pragma unroll
        for (int p = 0; p < 4; ++p) *reinterpret_cast<u32x4*>(crow + 32 * p) = pack8(o[p]);
        const int sl = slot[i];
        if (!isq && sl >= 0) {
          bf16_t* dst = cache + (((size_t)(sl / rk.BS) * rk.Hkv + kvh) * rk.BS + (sl % rk.BS)) * 128 + d0;
#pragma unroll
          for (int p = 0; p < 4; ++p) *reinterpret_cast<u32x4*>(dst + 32 * p) = pack8(o[p]);
        }
      }
    }
  }
}

// Per-accumulator epilogue: fp32 outputs (full tiles: 16-B stores) and every edge tile (guarded, any
// output type). Lane (fr, fh) of acc[i][j] owns columns w4_perm(16j + 4fh) .. +3 of its wave tile.
// Nout = output columns (packed rows / 2 for SiLU*up).
template <int EPI, bool OUT_F32, bool FULL>
__device__ __forceinline__ void w4_epilogue_reg(const f32x4 (&acc)[8][8], int wr, int wc, int fr, int fh, int m0,
                                                int n0, void* C, int ldc, const bf16_t* __restrict__ bias,
                                                const bf16_t* resid, int ldr, int M, int Nout) {
  const int row0 = m0 + wr * 128 + fr;
  if constexpr (EPI == EPI_SILU_MUL) {
    const int colw = (n0 >> 1) + wc * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gr = row0 + 16 * i;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int gc = colw + w4_perm(16 * j + 4 * fh);
        if (FULL || (gr < M && gc < Nout)) {
          float o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = silu(acc[i][j][k]) * acc[i][j + 4][k];
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + gc) =
              make_uint2(pk2bf(o[0], o[1]), pk2bf(o[2], o[3]));
        }
      }
    }
  } else {
    constexpr bool RES = epi_res(EPI), BIAS = epi_bias(EPI);
    const int colw = n0 + wc * 128;
    uint2 bv[BIAS ? 8 : 1];
    if constexpr (BIAS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gc = colw + w4_perm(16 * j + 4 * fh);
        bv[j] = *reinterpret_cast<const uint2*>(bias + (FULL ? gc : min(gc, Nout - 4)));
      }
    }
    // residual row groups in flight: the whole tile (RD = 8, 128 registers) for the residual-only form;
    // one 16-row group at a time with a bias too (the whole tile there made this rarely taken path the
    // loop body's register peak: 22 -> 8 spilled values bf16, 38 -> 0 fp32; the residual-only form
    // spills more, 2 -> 4, when grouped)
    constexpr int RD = BIAS ? 1 : 8;
    uint2 rv[RES ? 8 * RD : 1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gr = row0 + 16 * i;
      if constexpr (RES) {
        if (i % RD == 0) {
#pragma unroll
          for (int g = 0; g < RD; ++g)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int grc = FULL ? gr + 16 * g : min(gr + 16 * g, M - 1);
              const int gc = colw + w4_perm(16 * j + 4 * fh);
              rv[8 * g + j] = *reinterpret_cast<const uint2*>(resid + (size_t)grc * ldr + (FULL ? gc : min(gc, Nout - 4)));
            }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gc = colw + w4_perm(16 * j + 4 * fh);
        if (FULL || (gr < M && gc < Nout)) {
          float o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = acc[i][j][k];
          if constexpr (BIAS) {
            float b[4];
            unpack4(bv[j], b);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] += b[k];
          }
          if constexpr (RES) {
            float r[4];
            unpack4(rv[8 * (i % RD) + j], r);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] += r[k];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = w4_act<EPI>(o[k]);
          if constexpr (OUT_F32) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + (size_t)gr * ldc + gc) =
                (f32x4){o[0], o[1], o[2], o[3]};
          } else {
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(C) + (size_t)gr * ldc + gc) =
                make_uint2(pk2bf(o[0], o[1]), pk2bf(o[2], o[3]));
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Three-barrier K-tile schedule. Per K-tile and wave, MFMA m = 8i + j per 32-deep sub-step (the
// activation fragment a[i] held for 8 MFMAs, the weight fragment b[j] cycling):
//   m  0..14 : 8 reads b1[j] (weights, sub-step 1 of tile t), one per 2 MFMAs
//   m 21/22  : lgkmcnt(0), barrier X        -> every wave is done with the weight half of buffer t&1
//   m 22..58 : 8 weight DMAs of tile t+2 into it; reads a1[i] at m 24..42 between them
//   m 51/52  : lgkmcnt(0), barrier Y        -> the activation half of buffer t&1 is free
//   m 61..125: 8 activation DMAs of tile t+2
//   m 92/93  : vmcnt(13) (the 13 DMAs of this tile are the youngest), barrier: tile t+1 landed
//   m 93..123: the 16 F0 reads of tile t+1 (8 weight, then 8 activation fragments, spread)
// and no drain at the end of the K-tile: the next iteration waits for exactly the F0 fragments each of
// its first MFMAs needs (lgkmcnt(7) before m 0 = b0[0..7] and a0[0] landed; 10 before m 8: a0[1]; 13
// before m 16: a0[2]; the m 21 drain covers the rest), so the last F0 reads of a K-tile get 20+ MFMAs
// instead of 4 to land (an lgkmcnt(0) before the last MFMA exposed their latency every K-tile).
// M0 is set once per DMA group and post-incremented after the next MFMA (no s_nop between M0 and DMA).
__device__ __forceinline__ void h_read(bf16x8& d, unsigned addr, int off_imm) {
  // off_imm is a compile-time constant at every call site (fully unrolled schedule)
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(off_imm) : "memory");
}
__device__ __forceinline__ void h_dma(i32x4 srd, int voff, int soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(srd), "s"(soff) : "memory");
}
__device__ __forceinline__ void h_m0_set(unsigned lds) { asm volatile("s_mov_b32 m0, %0" ::"s"(lds) : "memory"); }
__device__ __forceinline__ void h_m0_inc() { asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory"); }

// MFMA index after which each DMA piece / fragment read is issued
constexpr int H_DX[8] = {22, 25, 28, 31, 34, 52, 55, 58};              // weight pieces (operand B)
constexpr int H_DY[8] = {61, 64, 85, 87, 89, 96, 99, 125};             // activation pieces (operand A)
constexpr int H_RB1[8] = {0, 2, 4, 6, 8, 10, 12, 14};                  // b1[j]
constexpr int H_RA1[8] = {24, 27, 30, 33, 36, 38, 40, 42};             // a1[i]
constexpr int H_RB0[8] = {93, 94, 95, 97, 98, 100, 101, 102};          // b0[j] of tile t+1
constexpr int H_RA0[8] = {104, 107, 110, 113, 116, 119, 121, 123};     // a0[i] of tile t+1
constexpr int H_VM = 13;  // DMAs of this iteration issued before the m = 92 wait

constexpr int h_find(const int (&s)[8], int m) {
  for (int q = 0; q < 8; ++q)
    if (s[q] == m) return q;
  return -1;
}

// One K-tile. g = running K-tile index (ring slot g & 1); sa / sb = DMA source offsets at K-tile kst
// (this tile's t+2 or the next tile's 0 / 1); ZERO = the F0 MFMAs start the accumulators (srcC = 0);
// VMW = the m = 92 vmcnt bound (H_VM plus the vector-memory ops issued between the previous
// iteration's DMAs and this one's, i.e. an epilogue). F0 = issue the 16 F0 reads of K-tile t+1 (false:
// the caller issues them itself, w4_read_f0). rbA / rbB: this lane's read bases (sub-step s, buffer 0)
// of the activation / weight fragments; fragment i at + 2048 i (the swizzle of row 16 i + fr does not
// depend on i).
template <bool ZERO, int VMW, bool F0 = true>
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
    if constexpr (m == 0) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
    if constexpr (m == 8) asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
    if constexpr (m == 16) asm volatile("s_waitcnt lgkmcnt(13)" ::: "memory");
    if constexpr (m == 21 || m == 51) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (m == 22 || m == 52) w4_barrier();
    if constexpr (m == 92) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMW) : "memory");
    if constexpr (m == 93) w4_barrier();
    if constexpr (m < 64) {
      if constexpr (ZERO) w4_mfma0(acc, a0, b0, m);
      else w4_mfma(acc, a0, b0, m);
    } else {
      w4_mfma(acc, a1, b1, m - 64);
    }
    // post-increment M0 one MFMA after each piece; a group's M0 is set before its first piece
    if constexpr (h_find(H_DX, m - 1) >= 0 || h_find(H_DY, m - 1) >= 0) h_m0_inc();
    if constexpr (m == 21) h_m0_set(mX);
    if constexpr (m == 59) h_m0_set(mY);
    constexpr int qx = h_find(H_DX, m), qy = h_find(H_DY, m);
    if constexpr (qx >= 0) h_dma(srd_b, sb[qx], kb);
    if constexpr (qy >= 0) h_dma(srd_a, sa[qy], kb);
    constexpr int r1b = h_find(H_RB1, m), r1a = h_find(H_RA1, m), r0b = h_find(H_RB0, m), r0a = h_find(H_RA0, m);
    if constexpr (r1b >= 0) h_read(b1[r1b], rb1, r1b * 2048);
    if constexpr (r1a >= 0) h_read(a1[r1a], ra1, r1a * 2048);
    if constexpr (F0 && r0b >= 0) h_read(b0[r0b], rb0, r0b * 2048);
    if constexpr (F0 && r0a >= 0) h_read(a0[r0a], ra0, r0a * 2048);
  });
}

// The F0 reads of the K-tile in ring slot g & 1, in w4_iter_h's order (the 8 weight fragments, then the
// 8 activation fragments), left in flight for the next w4_iter_h's counted waits.
__device__ __forceinline__ void w4_read_f0(int g, const unsigned (&rbA)[2], const unsigned (&rbB)[2],
                                           bf16x8 (&a0)[8], bf16x8 (&b0)[8]) {
  const unsigned buf = (unsigned)(g & 1) * W_BUF;
  const unsigned rb0 = rbB[0] + buf, ra0 = rbA[0] + buf;
  static_for<8>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    h_read(b0[j], rb0, j * 2048);
  });
  static_for<8>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    h_read(a0[i], ra0, i * 2048);
  });
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

// Persistent kernel, requires K / 64 >= W4_MIN_KT. Block b computes work items b, b + G, ...
// KSPLIT: split-K over nsplit K-slabs of K columns each in ONE launch -- work item t = z * tiles + tile
// writes the fp32 partial tile of slab z to C + z * M * ldc (the consumer, e.g. add_partials_rmsnorm,
// sums the slabs). For prefill shapes whose tile count fills only ~1.3 waves of the CUs (o_proj / down
// at M ~ 5k: 336 tiles on 256 CUs), two slabs make 2.6 waves.
template <int EPI, bool OUT_F32, bool KSPLIT = false>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4_kernel(const bf16_t* __restrict__ A, int lda,
                                                                const bf16_t* __restrict__ B, int ldb, void* C,
                                                                int ldc, const bf16_t* __restrict__ bias,
                                                                const bf16_t* resid, int ldr, int M, int N, int K,
                                                                int nsplit, RopeKV rk) {
  __shared__ __attribute__((aligned(16))) char smem[W4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fh = lane >> 4;
  const int tiles_m = (M + WBM - 1) / WBM, tiles_n = (N + WBN - 1) / WBN;
  const int nwg = tiles_m * tiles_n;
  const int nwt = KSPLIT ? nwg * nsplit : nwg;  // work items
  const int nk = K / WBK;
  const int Nout = EPI == EPI_SILU_MUL ? N / 2 : N;
  // byte offsets are 32-bit: the launcher guarantees rows * ld * 2 < 2^31 for both operands
  const i32x4 srd_a = make_srd(A, (unsigned)M * (unsigned)lda * 2u);
  const i32x4 srd_b = make_srd(B, (unsigned)N * (unsigned)ldb * 2u);

  // epilogue vector-memory ops younger than the next tile's K-tile-1 DMA at its first vmcnt
  constexpr int EV = w4_epi_vmem<EPI, OUT_F32>();
  constexpr int VMH0 = H_VM + EV > 63 ? 63 : H_VM + EV;
  // The next tile's F0 fragments are read before the epilogue (in the last K-tile, hidden under its
  // MFMAs) only where the epilogue leaves room for their 64 registers: with the bias, GELU or fp32
  // residual epilogues the allocator spilled them to scratch straight after the asm read issued, i.e.
  // before the data landed (tools/isa_lds_hazard.py checks every instantiation for that). Those read
  // them after the epilogue instead.
  constexpr bool LATE_F0 = !(EPI == EPI_NONE || EPI == EPI_SILU_MUL || (EPI == EPI_RESID && !OUT_F32));
  static_assert(EPI != EPI_ROPE_KV || (!OUT_F32 && !KSPLIT), "rope epilogue: bf16 output, no split-K");

  int tile = blockIdx.x;
  int z = KSPLIT ? tile / nwg : 0;
  int m0, n0;
  w4_origin(tile - z * nwg, nwg, tiles_m, tiles_n, m0, n0);
  int off_a[8], off_b[8];
  w4_offsets<false>(lda, m0, M, wid, lane, off_a);
  w4_offsets<true>(ldb, n0, N, wid, lane, off_b);
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
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): K-tiles 0 and 1 (the first iteration's vmcnt then covers K-tile 2)
  w4_barrier();
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  w4_read(smem, 0, wr, wc, fr, fh, a0, b0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_sched_barrier(0);

  // read bases (buffer 0) of the activation / weight fragments of sub-step s
  unsigned rbA[2], rbB[2];
  {
    const unsigned l0 = (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)smem;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const unsigned cs = (unsigned)(((4 * s + fh) ^ ((fr >> 1) & 7)) * 16);
      rbA[s] = l0 + (unsigned)((wr * 128 + fr) * 128) + cs;
      rbB[s] = l0 + W_TILE_A + (unsigned)((wc * 128 + fr) * 128) + cs;
    }
  }

  f32x4 acc[8][8];
  int g = 0;
  for (;;) {
    const int next = tile + (int)gridDim.x;
    const bool has_next = next < nwt;
    w4_iter_h<true, VMH0>(smem, g, srd_a, srd_b, off_a, off_b, 2, wid, rbA, rbB, acc, a0, b0, a1, b1);
    ++g;
    for (int t = 1; t + 2 < nk; ++t, ++g)
      w4_iter_h<false, H_VM>(smem, g, srd_a, srd_b, off_a, off_b, t + 2, wid, rbA, rbB, acc, a0, b0, a1, b1);
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
      w4_offsets<false>(lda, nm0, M, wid, ln, off_a);
      w4_offsets<true>(ldb, nn0, N, wid, ln, off_b);
      if constexpr (KSPLIT) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          off_a[i] += nz * K * 2;
          off_b[i] += nz * K * 2;
        }
      }
    }
    w4_iter_h<false, H_VM>(smem, g, srd_a, srd_b, off_a, off_b, 0, wid, rbA, rbB, acc, a0, b0, a1, b1);
    ++g;
    w4_iter_h<false, H_VM, !LATE_F0>(smem, g, srd_a, srd_b, off_a, off_b, 1, wid, rbA, rbB, acc, a0, b0, a1, b1);
    ++g;
    // the epilogue is compiler-scheduled code: it may move any register, so no asm read is in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w4_pin_acc(acc);
    void* Cz = KSPLIT ? (void*)(reinterpret_cast<float*>(C) + (size_t)z * M * ldc) : C;
    if constexpr (EPI == EPI_ROPE_KV) {
      if (m0 + WBM <= M) {
        w4_epilogue_rope<true>(acc, wr, wc, fr, fh, m0, n0, reinterpret_cast<bf16_t*>(Cz), ldc, rk, M);
      } else {
        w4_epilogue_rope<false>(acc, wr, wc, fr, fh, m0, n0, reinterpret_cast<bf16_t*>(Cz), ldc, rk, M);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // guarded: count unknown, drain (the next K-tile 1 lands too)
      }
    } else if (m0 + WBM <= M && n0 + WBN <= N) {
      if constexpr (OUT_F32)
        w4_epilogue_reg<EPI, true, true>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr, M, Nout);
      else
        w4_epilogue_full_bf16<EPI>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr);
    } else {
      w4_epilogue_reg<EPI, OUT_F32, false>(acc, wr, wc, fr, fh, m0, n0, Cz, ldc, bias, resid, ldr, M, Nout);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // guarded: count unknown, drain (the next K-tile 1 lands too)
    }
    // epilogue accumulator reads -> the next tile's srcC = 0 MFMA writes
    asm volatile("s_nop 7" ::: "memory");
    if (!has_next) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // the re-staged K-tiles land before the block's LDS is released
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // and the last (unused) F0 reads
      break;
    }
    if constexpr (LATE_F0) w4_read_f0(g, rbA, rbB, a0, b0);
    tile = next;
    m0 = nm0;
    n0 = nn0;
    z = nz;
  }
}

// Persistent grid: one block per CU (the kernel holds 128 KiB of LDS and 4 waves x 512 registers,
// so a CU never runs two), rounded down to a multiple of 8 so a block keeps its XCD across tiles.
// ragk_gemm_w4_set_grid(n > 0) caps the grid at n (tests: many tiles per block), 0 = one block per tile.
static int g_w4_grid = -1;
static int w4_grid(int nwg) {
  if (g_w4_grid < 0) {
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    g_w4_grid = (cus / 8) * 8;
  }
  return (g_w4_grid == 0 || g_w4_grid >= nwg) ? nwg : g_w4_grid;
}

template <int EPI, bool F32>
int launch_w4(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias, const void* resid,
              int ldr, int M, int N, int K, hipStream_t st) {
  const int nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  hipLaunchKernelGGL((gemm_w4_kernel<EPI, F32>), dim3(w4_grid(nwg)), dim3(W4_THREADS), 0, st, (const bf16_t*)A, lda,
                     (const bf16_t*)B, ldb, C, ldc, (const bf16_t*)bias, (const bf16_t*)resid, ldr, M, N, K, 1,
                     RopeKV{});
  return (int)hipGetLastError();
}

}  // namespace

// Persistent-grid override (tests): 0 = one block per tile, g > 0 = at most g blocks (a multiple of 8
// keeps each block on one XCD), < 0 = back to the CU count.
RAGK_API int ragk_gemm_w4_set_grid(int g) {
  g_w4_grid = g < 0 ? -1 : g;
  return 0;
}

// N = output columns (for EPI_SILU_MUL the weight has 2N rows, N % 128 == 0). Requires K % 64 == 0 and
// K >= 192 (three K-tiles per tile for the continuous ring).
RAGK_API int ragk_gemm_w4(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                          const void* resid, int ldr, int M, int N, int K, int epi, int out_f32, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % WBK != 0 || K / WBK < W4_MIN_KT) return (int)hipErrorInvalidValue;
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
// Ks = K / nsplit, one persistent launch over nsplit x tiles work items (see KSPLIT).
RAGK_API int ragk_gemm_w4_splitk(const void* A, int lda, const void* B, int ldb, float* P, int M, int N, int K,
                                 int nsplit, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (nsplit < 1 || K % nsplit || (K / nsplit) % WBK || (K / nsplit) / WBK < W4_MIN_KT || N % 8 || !P)
    return (int)hipErrorInvalidValue;
  if ((long long)M * lda * 2 >= (1LL << 31) || (long long)N * ldb * 2 >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_NONE, true, true>), dim3(w4_grid(nwg * nsplit)), dim3(W4_THREADS), 0, st,
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, (void*)P, N, nullptr, nullptr, 0, M, N, K / nsplit,
                     nsplit, RopeKV{});
  return (int)hipGetLastError();
}

// qkv = A . B^T (B = [(Hq + 2 Hkv) * 128][K]) with rope_kv's work in the epilogue (EPI_ROPE_KV above): q and
// k rotated (positions pos[M], tables cos_t / sin_t [positions][64]), k and v rows also into the paged caches
// kc / vc [blocks][Hkv][BS][128] at slot[M] (slot < 0: not cached). Same conditions as ragk_gemm_w4.
RAGK_API int ragk_gemm_w4_rope_kv(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int K,
                                  const int* pos, const int* slot, const float* cos_t, const float* sin_t, void* kc,
                                  void* vc, int Hq, int Hkv, int BS, hipStream_t st) {
  if (M <= 0) return 0;
  const int N = (Hq + 2 * Hkv) * 128;
  if (K % WBK != 0 || K / WBK < W4_MIN_KT || Hq < 1 || Hkv < 1 || BS < 1 || N % WBN != 0) return (int)hipErrorInvalidValue;
  if (!pos || !slot || !cos_t || !sin_t || !kc || !vc || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  if ((long long)M * lda * 2 >= (1LL << 31) || (long long)N * ldb * 2 >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int nwg = ((M + WBM - 1) / WBM) * (N / WBN);
  const RopeKV rk{pos, slot, cos_t, sin_t, (bf16_t*)kc, (bf16_t*)vc, Hq, Hkv, BS};
  hipLaunchKernelGGL((gemm_w4_kernel<EPI_ROPE_KV, false>), dim3(w4_grid(nwg)), dim3(W4_THREADS), 0, st,
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, nullptr, nullptr, 0, M, N, K, 1, rk);
  return (int)hipGetLastError();
}
