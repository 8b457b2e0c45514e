// Flash attention for gfx950 (MFMA 16x16x32 bf16, 64-key tiles, online softmax).
//
// Layout trick ("swapped" products, so no P transpose is ever needed):
//   S^T = K . Q^T   A = K rows from LDS (ds_read_b128, XOR swizzled), B = Q^T
//                   fragments held in VGPRs. C-layout: col = query (lane&15),
//                   row = key (4*(lane>>4)+r)  -> the softmax over keys of one
//                   query is lane-local + 2 shuffles (xor 16, 32).
//   O^T = V^T . P^T A = V^T read with ds_read_b64_tr_b16 (hardware transpose) from
//                   a row-major LDS V tile, B = P^T taken directly from the S^T
//                   accumulators of the same lane (k-slot order permuted to match).
//
// Kernels
//  * attn_prefill<D, GB, CAUSAL, PAGED>: varlen packed queries. PAGED reads K/V
//    from the paged cache [nblocks][Hkv][64][D] through block tables (prefill with
//    any prior context: chunked prefill / prefix reuse); !PAGED reads K/V straight
//    from a packed qkv buffer (bidirectional encoders). One block = 4 waves =
//    GB query heads sharing one KV head x (4/GB) groups of 32 query rows.
//  * attn_decode<D, G>: one query token per sequence, split-K over the context
//    (flash-decoding). Each wave streams its own 64-key tiles (K straight to
//    VGPRs, V through a wave-private LDS tile for the transposed read); 4 waves
//    combine in LDS; partitions merged by attn_decode_reduce.
//
// Replaces reference ops K5/K6 (causal GQA attention in transformers' Llama SDPA path,
// [dep] modeling_llama.py:191-215) and E3 (XLM-R/BERT bidirectional attention).
#include "common.h"
#include <type_traits>
using namespace ragk;

namespace {

constexpr int KT = 64;  // keys per tile == KV-cache page size
constexpr int MAX_BT = 2048;  // prefill block-table row cached in LDS (128k tokens)
constexpr float RESCALE_LOG2 = 8.f;  // deferred-rescale threshold (log2 units)

// max with the xor-16 / xor-32 lane partner without an LDS round trip (gfx950
// v_permlane{16,32}_swap). With both operands = v the swap returns, per lane, {v, partner} in
// some order, so max(r0, r1) is the pairwise max on every lane.
__device__ __forceinline__ float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <int D>
struct Cfg {
  static constexpr int NC = D / 8;               // 16-B chunks per row
  static constexpr int ROWB = D * 2;             // bytes per row
  static constexpr int TILEB = KT * D * 2;       // bytes per K or V tile
  static constexpr int PIECES = TILEB / 1024;    // 1-KiB glds pieces per tile
  static constexpr int RPP = 1024 / ROWB;        // rows per piece
  static constexpr int KS = D / 32;              // k-steps of QK^T
  static constexpr int DT = D / 16;              // 16-wide d tiles of O
  static constexpr int GR = D / 16;              // 32-B granules per row
  static constexpr int RB = 8 / GR;              // rows per 256-B bank row
};

// K tile: swizzle for row reads (ds_read_b128)
template <int D>
__device__ __forceinline__ int kswz(int row) {
  constexpr int NC = Cfg<D>::NC;
  return (row / (16 / NC)) & (NC - 1);
}
// V tile: swizzle for transposed reads (keeps 32-B granules intact)
template <int D>
__device__ __forceinline__ int vswz(int row) {
  return 2 * ((row / Cfg<D>::RB) & (Cfg<D>::GR - 1));
}

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(p));
}

// Stage one 64-row tile (K or V) into LDS with glds; `pieces_per_wave` pieces per wave.
// row_src(row) returns the global row pointer for tile row `row`.
template <int D, bool IS_V, bool NT = false, int NW = 0, typename RowSrc>
__device__ __forceinline__ void stage_kv(char* lds_tile, int wid, int nwaves, int lane, RowSrc row_src) {
  constexpr int NC = Cfg<D>::NC, PIECES = Cfg<D>::PIECES, RPP = Cfg<D>::RPP;
  constexpr int PPW = NW > 0 ? PIECES / NW : PIECES;  // NW > 0: compile-time wave count, unrolled
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = NW > 0 ? wid + NW * i : wid + nwaves * i;
    if (NW == 0 && p >= PIECES) break;
    const int row = p * RPP + lane / NC;
    const int ph = lane % NC;
    const int c = ph ^ (IS_V ? vswz<D>(row) : kswz<D>(row));
    if constexpr (NT)  // once-read K/V stream (decode): non-temporal LDS-DMA
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(row_src(row) + c * 8),
                                       (__attribute__((address_space(3))) void*)(lds_tile + p * 1024), 16, 0, 2);
    else
      glds16(row_src(row) + c * 8, lds_tile + p * 1024);
  }
}

// V^T A-fragment for d-tile dt and key k-step ks (32 keys) from a V tile in LDS.
template <int D>
__device__ __forceinline__ bf16x8 load_vt(const char* sV, int dt, int ks, int lane) {
  const int h = lane >> 4, i = lane & 15;
  const int chunk = 2 * dt + ((i >> 1) & 1);
  const int r0 = 32 * ks + 4 * h + (i >> 2);
  const int r1 = r0 + 16;
  const bf16x4 a = tr_read(sV + r0 * Cfg<D>::ROWB + 16 * (chunk ^ vswz<D>(r0)) + 8 * (i & 1));
  const bf16x4 b = tr_read(sV + r1 * Cfg<D>::ROWB + 16 * (chunk ^ vswz<D>(r1)) + 8 * (i & 1));
  return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int D>
__device__ __forceinline__ bf16x8 load_k(const char* sK, int t, int s, int lane) {
  const int R = 16 * t + (lane & 15);
  const int c = 4 * s + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(sK + R * Cfg<D>::ROWB + 16 * (c ^ kswz<D>(R)));
}

__device__ __forceinline__ bf16x8 pack_p(const f32x4& a, const f32x4& b) {
  return (bf16x8){f2bf_s(a[0]), f2bf_s(a[1]), f2bf_s(a[2]), f2bf_s(a[3]),
                  f2bf_s(b[0]), f2bf_s(b[1]), f2bf_s(b[2]), f2bf_s(b[3])};
}

// ------------------------------------------------------------------------------------
// Prefill / encoder attention
// ------------------------------------------------------------------------------------
struct PrefillArgs {
  const bf16_t* q;  int q_stride;          // token row stride (elements); head h at +h*D
  const bf16_t* k;  const bf16_t* v;       // PAGED: caches; else packed K/V base pointers
  int kv_stride;                           // !PAGED: token row stride of k/v
  const int* block_tables; int bt_stride;  // PAGED
  const int* cu_q;                         // [S+1] query token offsets
  const int* cu_kv;                        // [S+1] kv token offsets (!PAGED)
  const int* kv_lens;                      // [S] total context length per sequence
  const int* tiles;                        // [n][2] = (seq, q_start)
  bf16_t* out; int out_stride;
  int Hq, Hkv;
  float scale_log2;
  unsigned kv_bytes;                       // PAGED: bytes of one cache (K or V) if < 4 GiB, else 0
  int n_hg;                                // > 0: 1-D grid of n_tiles x n_hg, head group fastest
};

// Prefill block -> (tile index, head group). 1-D grid, head group fastest (n_hg > 0, the default): the
// workgroups dispatch in the tile list's order -- heaviest causal tiles first -- across EVERY head (a 2-D
// grid dispatches head 0's whole list before head 1's, so the last heads' longest tiles start late and
// set the tail), and the round-robin XCD placement of consecutive workgroups keeps each head group on
// one XCD when n_hg is a multiple of 8 (its K/V tiles are re-read from that XCD's L2 by every query tile).
__device__ inline void prefill_block(const PrefillArgs& a, int& tile, int& hg) {
  if (a.n_hg > 0) {
    tile = (int)blockIdx.x / a.n_hg;
    hg = (int)blockIdx.x - tile * a.n_hg;
  } else {
    tile = blockIdx.x;
    hg = blockIdx.y;
  }
}

__device__ unsigned long long* g_attn_dbg = nullptr;  // stamp build only

// PRIO: wave priority around the MFMA clusters (0 none, 1 QK^T and PV, 2 PV only). Two waves share
// each SIMD (2 blocks per CU); raising the priority of the wave that is issuing MFMAs lets the
// other wave's softmax VALU fill around them instead of delaying them.
// BUF (PAGED only, cache < 4 GiB): K/V tiles staged by buffer_load ... lds with the per-lane byte
// offsets (row, swizzled chunk) computed once and the tile's cache offset in an SGPR, instead of
// 64-bit address math per piece per tile (the stamp build put the DMA issue at ~490 of ~4300 wave
// cycles per tile).
template <int D, int GB, bool CAUSAL, bool PAGED, bool STAMP = false, int NWV = 4, int PRIO = 0,
          bool BUF = false>
__global__ __launch_bounds__(NWV * 64, 8 / NWV) void attn_prefill_kernel(PrefillArgs a) {
  unsigned long long stp[6] = {0, 0, 0, 0, 0, 0};
  using C = Cfg<D>;
  constexpr int NTH = NWV * 64;
  constexpr int QT = 32 * (NWV / GB);  // query positions per block
  __shared__ __attribute__((aligned(16))) char smem[4 * C::TILEB];  // [buf][K|V]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  int tix, hg;
  prefill_block(a, tix, hg);
  const int seq = a.tiles[2 * tix], q_start = a.tiles[2 * tix + 1];
  const int G = a.Hq / a.Hkv;
  const int groups_per_kv = G / GB;
  const int kvh = hg / groups_per_kv;
  const int gsub = hg % groups_per_kv;
  const int hq = kvh * G + gsub * GB + (wid % GB);
  const int pbase = q_start + (wid / GB) * 32;

  const int q_off = a.cu_q[seq];
  const int q_len = a.cu_q[seq + 1] - q_off;
  const int kv_len = a.kv_lens[seq];
  const int ctx0 = kv_len - q_len;  // absolute position of query 0

  const int blk_qmax = min(q_start + QT, q_len) - 1;
  const int n_keys = CAUSAL ? min(kv_len, ctx0 + blk_qmax + 1) : kv_len;
  const int n_kt = (n_keys + KT - 1) / KT;
  const int wave_qmax = min(pbase + 31, q_len - 1);
  const int wave_pmax = ctx0 + wave_qmax;

  const int fr = lane & 15, fh = lane >> 4;

  // Q^T fragments (B operand), 2 query sub-tiles of 16
  bf16x8 qf[2][C::KS];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    int qi = pbase + 16 * qt + fr;
    qi = qi < q_len ? qi : q_len - 1;
    const bf16_t* qp = a.q + (size_t)(q_off + qi) * a.q_stride + hq * D + 8 * fh;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[qt][s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }

  f32x4 o[C::DT][2];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_i[2] = {-INFINITY, -INFINITY}, l_i[2] = {0.f, 0.f};

  const int kv_off = PAGED ? 0 : a.cu_kv[seq];
  const int* bt = PAGED ? a.block_tables + (size_t)seq * a.bt_stride : nullptr;

  // the sequence's block-table row, cached in LDS once (a global load per tile sat on the DMA
  // issue path: ~1.2k of ~5.7k wave cycles per tile in the stamp build, tools/attn_stamps.py)
  __shared__ int s_bt[PAGED ? MAX_BT : 1];
  if constexpr (PAGED) {
    for (int i = threadIdx.x; i < n_kt; i += NTH) s_bt[i] = bt[i];
    __syncthreads();
  }
  int bt_next = PAGED && n_kt > 0 ? s_bt[0] : 0;  // block of the tile staged next

  static_assert(!BUF || (PAGED && C::PIECES % NWV == 0), "buffer staging: paged caches, whole pieces per wave");
  constexpr int BPW = BUF ? C::PIECES / NWV : 1;
  int koff[BPW], voff[BPW];
  i32x4 srd_k, srd_v;
  if constexpr (BUF) {
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      const int p = wid_u + NWV * i;
      const int row = p * C::RPP + lane / C::NC, ph = lane % C::NC;
      koff[i] = row * C::ROWB + 16 * (ph ^ kswz<D>(row));
      voff[i] = row * C::ROWB + 16 * (ph ^ vswz<D>(row));
    }
    srd_k = make_srd(a.k, a.kv_bytes);
    srd_v = make_srd(a.v, a.kv_bytes);
  }
  auto stage = [&](int kt, int buf) {
    char* sK = smem + buf * 2 * C::TILEB;
    char* sV = sK + C::TILEB;
    if constexpr (BUF) {
      // unsigned: a cache of 2-4 GiB has tile offsets past INT_MAX (soffset is an unsigned 32-bit add)
      const int soff = __builtin_amdgcn_readfirstlane((int)((unsigned)(bt_next * a.Hkv + kvh) * (unsigned)(KT * D * 2)));
#pragma unroll
      for (int i = 0; i < BPW; ++i) {
        const int p = wid_u + NWV * i;
        blds16(srd_k, koff[i], soff, sK + p * 1024);
        blds16(srd_v, voff[i], soff, sV + p * 1024);
      }
    } else if constexpr (PAGED) {
      const size_t base = ((size_t)bt_next * a.Hkv + kvh) * KT * D;
      const bf16_t* kb = a.k + base;
      const bf16_t* vb = a.v + base;
      stage_kv<D, false, false, NWV>(sK, wid_u, NWV, lane, [&](int r) { return kb + (size_t)r * D; });
      stage_kv<D, true, false, NWV>(sV, wid_u, NWV, lane, [&](int r) { return vb + (size_t)r * D; });
    } else {
      const int k0 = kt * KT;
      auto rowp = [&](const bf16_t* base, int r) {
        int tok = k0 + r;
        tok = tok < kv_len ? tok : kv_len - 1;
        return base + (size_t)(kv_off + tok) * a.kv_stride + kvh * D;
      };
      stage_kv<D, false, false, NWV>(sK, wid_u, NWV, lane, [&](int r) { return rowp(a.k, r); });
      stage_kv<D, true, false, NWV>(sV, wid_u, NWV, lane, [&](int r) { return rowp(a.v, r); });
    }
  };

  if (n_kt > 0) stage(0, 0);
  if constexpr (PAGED) bt_next = n_kt > 1 ? s_bt[1] : 0;
  wait_vmcnt0();
  __syncthreads();

  for (int kt = 0; kt < n_kt; ++kt) {
    unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    const int cur = kt & 1;
    const char* sK = smem + cur * 2 * C::TILEB;
    const char* sV = sK + C::TILEB;
    const int k0 = kt * KT;
    const bool active = !CAUSAL || k0 <= wave_pmax;
    // ---- S^T = K Q^T ----
    f32x4 s[4][2];
    if (active) {
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
        s[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < C::KS; ++ks) {
          const bf16x8 kf = load_k<D>(sK, t, ks, lane);
          s[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][ks], s[t][0], 0, 0, 0);
          s[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][ks], s[t][1], 0, 0, 0);
        }
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
    // next tile's DMA issued behind the QK^T MFMAs (async-STAGE split: the issue overlaps the MFMA
    // pipe instead of delaying it); every wave stages its pieces, active or not
    if (kt + 1 < n_kt) stage(kt + 1, cur ^ 1);
    if constexpr (PAGED) bt_next = kt + 2 < n_kt ? s_bt[kt + 2] : 0;  // consumed next iteration
    if constexpr (STAMP) t2 = t3 = t4 = __builtin_amdgcn_s_memtime();
    if (active) {
      // ---- online softmax (per query column, lane-local + xor 16/32) ----
      // Max on the raw scores (scale > 0 keeps the order); the log2 scale is folded into one FMA
      // per element. Deferred rescale: the reference max m_i only moves when the tile max exceeds
      // it by more than RESCALE_LOG2 (p stays <= 2^RESCALE_LOG2, exact in fp32 / bf16 P), so the
      // O *= alpha pass (DT*2*4 multiplies per lane) runs on a few early tiles instead of every tile.
      const bool need_mask = CAUSAL ? (k0 + KT - 1 > ctx0 + pbase) || (k0 + KT > kv_len) : (k0 + KT > kv_len);
      const float c = a.scale_log2;
      float alpha[2];
      // one wave-uniform branch per tile (the masked body only runs on diagonal / ragged tiles)
      auto softmax = [&](auto mask_tag, const int qt) {
        constexpr bool MASK = decltype(mask_tag)::value;
        const int qpos = ctx0 + pbase + 16 * qt + fr;
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = s[t][qt][r];
            if constexpr (MASK) {
              const int kj = k0 + 16 * t + 4 * fh + r;
              const bool ok = kj < kv_len && (!CAUSAL || kj <= qpos);
              x = ok ? x : -INFINITY;
              s[t][qt][r] = x;
            }
            mx = fmaxf(mx, x);
          }
        mx = max_xor16(mx);
        mx = max_xor32(mx);
        const float mxs = mx * c;
        alpha[qt] = 1.f;
        if (mxs > m_i[qt] + RESCALE_LOG2) {
          alpha[qt] = m_i[qt] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_i[qt] - mxs);
          m_i[qt] = mxs;
        }
        const float mref = m_i[qt] == -INFINITY ? 0.f : m_i[qt];
        float ls = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[t][qt][r], c, -mref));
            s[t][qt][r] = p;
            ls += p;
          }
        l_i[qt] = l_i[qt] * alpha[qt] + ls;
      };
      if (need_mask) {
        softmax(std::true_type{}, 0);
        softmax(std::true_type{}, 1);
      } else {
        softmax(std::false_type{}, 0);
        softmax(std::false_type{}, 1);
      }
      if (__builtin_amdgcn_ballot_w64(alpha[0] != 1.f || alpha[1] != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) o[dt][qt] *= alpha[qt];
      }
      // ---- O^T += V^T P^T ----
      bf16x8 pb[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) pb[ks][qt] = pack_p(s[2 * ks][qt], s[2 * ks + 1][qt]);
      if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
      if constexpr (PRIO != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 vf = load_vt<D>(sV, dt, ks, lane);
          o[dt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[ks][0], o[dt][0], 0, 0, 0);
          o[dt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[ks][1], o[dt][1], 0, 0, 0);
        }
      if constexpr (PRIO != 0) __builtin_amdgcn_s_setprio(0);
      if constexpr (STAMP) t4 = __builtin_amdgcn_s_memtime();
    }
    wait_vmcnt0();
    __syncthreads();
    if constexpr (STAMP) {
      const unsigned long long t5 = __builtin_amdgcn_s_memtime();
      stp[0] += t2 - t1;  // DMA issue of the next tile
      stp[1] += t1 - t0;  // QK^T (K reads + 32 MFMA issue)
      stp[2] += t3 - t2;  // softmax (+ waiting for the QK^T results)
      stp[3] += t4 - t3;  // PV (V tr-reads + 32 MFMA issue)
      stp[4] += t5 - t4;  // vmcnt(0) + barrier
      stp[5] += 1;
    }
  }
  if constexpr (STAMP) {
    if (lane == 0 && g_attn_dbg) {
      unsigned long long* d = g_attn_dbg + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + wid) * 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = stp[i];
    }
  }

  // ---- finalize: O = O^T / l, store 4 consecutive d (8 B) per (dt, qt) ----
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = l_i[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qi = pbase + 16 * qt + fr;
    if (qi < q_len) {
      bf16_t* op = a.out + (size_t)(q_off + qi) * a.out_stride + hq * D + 4 * fh;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        const f32x4 v = o[dt][qt] * inv;
        const unsigned lo = pk2bf(v[0], v[1]);
        const unsigned hi = pk2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(op + 16 * dt) = make_uint2(lo, hi);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Ping-pong prefill attention (Llama config: D 128, 4 query heads per KV head, causal, paged
// cache < 4 GiB). One 8-wave block per CU: waves 0-3 (group A) and 4-7 (group B) each own 32 query
// rows of the same 4 heads, so wave w and its SIMD partner w + 4 run the same program one segment
// apart. A segment is the interval between two block barriers; in every segment one group is in
// its MFMA phase (PV of tile u-1 + QK^T of tile u: 64 MFMAs, LDS fragment reads) while the other
// is in its VALU phase (online softmax of its tile, the next K or V tile's LDS-DMA). The stamp
// build of attn_prefill_kernel put a wave at ~4.3k cycles per tile for 1024 cycles of its own
// MFMAs: the two co-resident waves of a SIMD (independent 4-wave blocks) reached their softmax
// at the same time and left the matrix pipe idle; here the barrier schedule makes the softmax of
// one wave and the MFMAs of its partner coincide (MI355X_MICROARCH.md "Two waves per SIMD").
//
// K/V ring of 3 slots (tile t in slot t % 3), segment s (A: MFMA phase when s is even, B when odd):
//   A (MFMA): seg 2u   PV(u-1) + QK(u)       A (VALU): seg 2u+1  softmax(u), DMA K(u+2)
//   B (MFMA): seg 2u+1 PV(u-1) + QK(u)       B (VALU): seg 2u+2  softmax(u), DMA V(u+2)
// K(t) is read in segments 2t / 2t+1 and rewritten (as K(t+3)) in 2t+3; V(t) read in 2t+2 / 2t+3,
// rewritten in 2t+4. The VALU phase ends with vmcnt(4) (only the DMAs it just issued may stay in
// flight), so every tile lands >= 2 segments after its DMA was issued, before the barrier that
// precedes its first reader. Prologue: K(0), V(0), K(1). 2n + 2 segments for n KV tiles.
// Same arithmetic as attn_prefill_kernel (bit-identical outputs).
constexpr int PP_NS = 3;

template <typename F, int... Is>
__device__ __forceinline__ void pp_static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void pp_static_for(F&& f) {
  pp_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// One MFMA phase: 16 PV steps (d-tile dt = i / 2, key step ks = i % 2; two tr-read pairs per
// fragment) or 16 QK^T steps (key sub-tile t = j / 4, d-step ks = j % 4; one b128 read). The LDS
// fragment of step i + PF is requested before the MFMAs of step i and a scheduling fence follows
// every step, so at most PF + 1 fragments are live. Fragment addresses are the load_vt / load_k
// images (D = 128: kswz(R) = R & 15, vswz(r) = 2 (r & 7)) rebuilt per phase from an opaque copy of
// the lane id: loop-invariant per-lane offsets hoisted out of the segment loop spilled (12 VGPRs).
template <bool PV, int PF>
__device__ __forceinline__ void pp_mfma_phase(const char* sV, const char* sK, int lane, const bf16x8 (&pb)[2][2],
                                              const bf16x8 (&qf)[2][Cfg<128>::KS], f32x4 (&o)[Cfg<128>::DT][2],
                                              f32x4 (&s)[4][2]) {
  constexpr int N = 16;
  int ln = lane;
  asm volatile("" : "+v"(ln));
  // V^T: rows r0 = 32 ks + 4 h + (i >> 2) and r0 + 16, chunk (2 dt + b) ^ 2 (r0 & 7), half i & 1
  const int vi = ln & 15, vr = 4 * (ln >> 4) + (vi >> 2);
  const int vx = vr & 7;
  const char* vb = sV + vr * 256 + 16 * ((vi >> 1) & 1) + 8 * (vi & 1);
  // K: row 16 t + fr, chunk (4 s + fh) ^ fr
  const int fr = ln & 15;
  const char* kb = sK + fr * 256 + 16 * ((ln >> 4) ^ (fr & 3));
  const int kx = fr >> 2;
  auto frag = [&](auto ic) -> bf16x8 {
    constexpr int i = decltype(ic)::value;
    if constexpr (PV) {
      constexpr int dt = i >> 1, ks = i & 1;
      const char* p = vb + ks * 32 * 256 + 32 * (dt ^ vx);
      const bf16x4 x0 = tr_read(p), x1 = tr_read(p + 16 * 256);
      return (bf16x8){x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    } else {
      constexpr int t = i >> 2, ks = i & 3;
      return *reinterpret_cast<const bf16x8*>(kb + t * 16 * 256 + 64 * (ks ^ kx));
    }
  };
  bf16x8 ring[PF + 1];
  pp_static_for<PF>([&](auto ic) { ring[decltype(ic)::value] = frag(ic); });
  pp_static_for<N>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if constexpr (i + PF < N) ring[(i + PF) % (PF + 1)] = frag(std::integral_constant<int, i + PF>{});
    const bf16x8 f = ring[i % (PF + 1)];
    if constexpr (PV) {
      constexpr int dt = i >> 1, ks = i & 1;
      o[dt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, pb[ks][0], o[dt][0], 0, 0, 0);
      o[dt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, pb[ks][1], o[dt][1], 0, 0, 0);
    } else {
      constexpr int t = i >> 2, ks = i & 3;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      s[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, qf[0][ks], ks == 0 ? z : s[t][0], 0, 0, 0);
      s[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, qf[1][ks], ks == 0 ? z : s[t][1], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <int PRIO_B, int PF = 2, bool STAMP = false>
__global__ __launch_bounds__(512, 2) void attn_prefill_pp_kernel(PrefillArgs a) {
  constexpr int D = 128;
  using C = Cfg<D>;
  constexpr bool CAUSAL = true;
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_NS * C::TILEB];  // [K slots][V slots]
  __shared__ int s_bt[MAX_BT];

  const int lane = threadIdx.x & 63;
  const int wid_u = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int grp = wid_u >> 2, hs = wid_u & 3;
  int tix, hg;
  prefill_block(a, tix, hg);
  const int seq = a.tiles[2 * tix], q_start = a.tiles[2 * tix + 1];
  const int G = a.Hq / a.Hkv;
  const int groups_per_kv = G / 4;
  const int kvh = hg / groups_per_kv;
  const int hq = kvh * G + (hg % groups_per_kv) * 4 + hs;
  const int pbase = q_start + grp * 32;

  const int q_off = a.cu_q[seq];
  const int q_len = a.cu_q[seq + 1] - q_off;
  const int kv_len = a.kv_lens[seq];
  const int ctx0 = kv_len - q_len;
  const int blk_qmax = min(q_start + 64, q_len) - 1;
  const int n_keys = min(kv_len, ctx0 + blk_qmax + 1);
  const int n_kt = (n_keys + KT - 1) / KT;
  const int wave_pmax = ctx0 + min(pbase + 31, q_len - 1);
  const int fr = lane & 15, fh = lane >> 4;

  bf16x8 qf[2][C::KS];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    int qi = pbase + 16 * qt + fr;
    qi = qi < q_len ? qi : q_len - 1;
    const bf16_t* qp = a.q + (size_t)(q_off + qi) * a.q_stride + hq * D + 8 * fh;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[qt][s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }
  f32x4 o[C::DT][2];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_i[2] = {-INFINITY, -INFINITY}, l_i[2] = {0.f, 0.f};
  f32x4 s[4][2];
  bf16x8 pb[2][2];

  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;
  for (int i = threadIdx.x; i < n_kt; i += 512) s_bt[i] = bt[i];

  // pieces hs, hs + 4, hs + 8, hs + 12 of a 16-piece K / V tile (the wave's share in its group)
  int koff[4], voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = hs + 4 * i;
    const int row = p * C::RPP + lane / C::NC, ph = lane % C::NC;
    koff[i] = row * C::ROWB + 16 * (ph ^ kswz<D>(row));
    voff[i] = row * C::ROWB + 16 * (ph ^ vswz<D>(row));
  }
  const i32x4 srd_k = make_srd(a.k, a.kv_bytes);
  const i32x4 srd_v = make_srd(a.v, a.kv_bytes);
  auto stage = [&](int kt, bool is_v) {
    const int soff = __builtin_amdgcn_readfirstlane(
        (int)((unsigned)(s_bt[kt] * a.Hkv + kvh) * (unsigned)(KT * D * 2)));
    char* base = smem + ((is_v ? PP_NS : 0) + kt % PP_NS) * C::TILEB;
#pragma unroll
    for (int i = 0; i < 4; ++i) blds16(is_v ? srd_v : srd_k, is_v ? voff[i] : koff[i], soff, base + (hs + 4 * i) * 1024);
  };
  __syncthreads();  // s_bt
  if (grp == 0) {
    stage(0, false);
    stage(0, true);
  } else if (n_kt > 1) {
    stage(1, false);
  }
  wait_vmcnt0();
  __syncthreads();
  if constexpr (PRIO_B) {
    if (grp == 1) __builtin_amdgcn_s_setprio(1);
  }

  const float c = a.scale_log2;
  // MFMA phase of tile u: PV(u-1) (V slot (u-1) % 3) and QK^T(u) (K slot u % 3)
  auto mfma_phase = [&](int u) {
    if (u >= 1 && u - 1 < n_kt && (u - 1) * KT <= wave_pmax)
      pp_mfma_phase<true, PF>(smem + (PP_NS + (u + PP_NS - 1) % PP_NS) * C::TILEB, nullptr, lane, pb, qf, o, s);
    if (u < n_kt && u * KT <= wave_pmax)
      pp_mfma_phase<false, PF>(nullptr, smem + (u % PP_NS) * C::TILEB, lane, pb, qf, o, s);
  };
  // VALU phase of tile u in segment seg: softmax(u) -> pb (O rescaled), then this segment's DMA
  // (odd seg: group A stages K((seg + 3) / 2); even: group B stages V(seg / 2 + 1))
  auto valu_phase = [&](int u, int seg) {
    const int k0 = u * KT;
    if (u >= 0 && u < n_kt && k0 <= wave_pmax) {
      const bool need_mask = (k0 + KT - 1 > ctx0 + pbase) || (k0 + KT > kv_len);
      float alpha[2];
      auto softmax = [&](auto mask_tag, const int qt) {
        constexpr bool MASK = decltype(mask_tag)::value;
        const int qpos = ctx0 + pbase + 16 * qt + fr;
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = s[t][qt][r];
            if constexpr (MASK) {
              const int kj = k0 + 16 * t + 4 * fh + r;
              const bool ok = kj < kv_len && kj <= qpos;
              x = ok ? x : -INFINITY;
              s[t][qt][r] = x;
            }
            mx = fmaxf(mx, x);
          }
        mx = max_xor16(mx);
        mx = max_xor32(mx);
        const float mxs = mx * c;
        alpha[qt] = 1.f;
        if (mxs > m_i[qt] + RESCALE_LOG2) {
          alpha[qt] = m_i[qt] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_i[qt] - mxs);
          m_i[qt] = mxs;
        }
        const float mref = m_i[qt] == -INFINITY ? 0.f : m_i[qt];
        float ls = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[t][qt][r], c, -mref));
            s[t][qt][r] = pv;
            ls += pv;
          }
        l_i[qt] = l_i[qt] * alpha[qt] + ls;
      };
      if (need_mask) {
        softmax(std::true_type{}, 0);
        softmax(std::true_type{}, 1);
      } else {
        softmax(std::false_type{}, 0);
        softmax(std::false_type{}, 1);
      }
      if (__builtin_amdgcn_ballot_w64(alpha[0] != 1.f || alpha[1] != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) o[dt][qt] *= alpha[qt];
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) pb[ks][qt] = pack_p(s[2 * ks][qt], s[2 * ks + 1][qt]);
    }
    const int item = (seg & 1) ? (seg + 3) >> 1 : (seg >> 1) + 1;
    if (item < n_kt) {
      stage(item, (seg & 1) == 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      wait_vmcnt0();
    }
  };
  // stamp build: per wave [MFMA phase, barrier after it, VALU phase, barrier after it, segments]
  unsigned long long stp[5] = {0, 0, 0, 0, 0};
  unsigned long long t0 = 0;
  auto stamp = [&](int i) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      stp[i] += t - t0;
      t0 = t;
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
  // 2 n_kt + 2 segments, two per iteration; group A: [MFMA(u) | VALU(u)], group B one segment
  // behind: [VALU(u-1) | MFMA(u)]
  if (grp == 0) {
    for (int u = 0; u <= n_kt; ++u) {
      mfma_phase(u);
      stamp(0);
      barrier();
      stamp(1);
      valu_phase(u, 2 * u + 1);
      stamp(2);
      barrier();
      stamp(3);
    }
  } else {
    for (int u = 0; u <= n_kt; ++u) {
      valu_phase(u - 1, 2 * u);
      stamp(2);
      barrier();
      stamp(3);
      mfma_phase(u);
      stamp(0);
      barrier();
      stamp(1);
    }
  }
  if constexpr (STAMP) {
    stp[4] = n_kt + 1;
    if (lane == 0 && g_attn_dbg) {
      unsigned long long* d = g_attn_dbg + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + wid_u) * 6;
#pragma unroll
      for (int i = 0; i < 5; ++i) d[i] = stp[i];
    }
  }
  if constexpr (PRIO_B) {
    if (grp == 1) __builtin_amdgcn_s_setprio(0);
  }

#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = l_i[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qi = pbase + 16 * qt + fr;
    if (qi < q_len) {
      bf16_t* op = a.out + (size_t)(q_off + qi) * a.out_stride + hq * D + 4 * fh;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        const f32x4 v = o[dt][qt] * inv;
        *reinterpret_cast<uint2*>(op + 16 * dt) = make_uint2(pk2bf(v[0], v[1]), pk2bf(v[2], v[3]));
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Software-pipelined prefill attention, one wave per SIMD (Llama config: D 128, 4 query heads per
// KV head, causal, paged cache < 4 GiB). attn_prefill_kernel runs two waves per SIMD, each in
// lockstep phases QK^T -> softmax -> PV: the stamps put a wave at ~4.3k cycles per 64-key tile for
// 1024 cycles of its own 16x16x32 MFMAs (~48 % matrix-pipe use), and a barrier-alternated 8-wave
// variant (attn_prefill_pp_kernel) was slower still -- the two waves of a SIMD share one vector
// issue port, and a 16x16x32 MFMA holds it 8 of its 16 cycles. Here:
//   * 32x32x16 MFMAs (the issue port is held 8 of 32 cycles per MFMA, MI355X_MICROARCH.md cycle
//     constants), 32 per tile per wave, and ONE wave per SIMD (4-wave block, one block per CU);
//   * iteration t issues PV(t-1) then QK^T(t+1) on the matrix pipe while the same wave's VALU runs the
//     online softmax of tile t between them: 32 slots, one MFMA each, the LDS fragment of slot i + 2
//     and a softmax chunk (max in slots 0..3, row statistics in 4, one element's fma / exp / add per
//     slot from 5 on: at most one transcendental per MFMA gap). Every MFMA is an ordered volatile asm
//     and each chunk's inputs / results are pinned, so neither the IR passes nor the scheduler can
//     regroup the stream; S is double-buffered (tile loop unrolled by two), P is single-buffered
//     (P(t-1)[ks] is dead before P(t)[ks] is packed);
//   * K / V ring of 4 slots, K staged 3 and V 2 tiles ahead, so iteration t's last two slots can read
//     the first PV fragments of iteration t + 1; LDS-DMA as inline asm (the intrinsic made the
//     waitcnt pass drain vmcnt(0) before every later ds_read); one vmcnt + barrier per tile.
// Diagonal / ragged tiles (masked softmax), the first tile (no PV) and the last (no QK) run the same
// MFMA stream with its halves guarded and the whole softmax after it.
// Layouts (v_mfma_f32_32x32x16_bf16, lane l, h = l >> 5): A[i = l & 31][k = 8h + j], B[k = 8h + j][n = l & 31],
// C[8b + 4h + r][l & 31] in acc[4b + r]. S^T = K Q^T: lane holds query pbase + (l & 31), keys
// 32 kb + 8b + 4h + r. P^T fragment of key step ks (16 keys) = acc S[ks / 2][8 (ks % 2) + j] (keys
// 16 ks + 8 (j / 4) + 4h + j % 4), so V^T is read with the same key order: ds_read_b64_tr_b16 of rows
// 16 ks + 4h + (i >> 2) and + 8 (i = l & 15) gives lane l the d column 32 db + 16 ((l >> 4) & 1) + i.
typedef __attribute__((ext_vector_type(16))) float f32x16;
constexpr int V3_NS = 4;
constexpr int V3_PF = 4, V3_RING = 8;  // ring size divides the 32 slots (continuity across iterations)

// MFMA through the builtin (the compiler's hazard recognizer then covers every MFMA-result read: as
// inline asm the compiler treated the results as ready and could copy an accumulator before the MFMA
// retired). The slot order is kept by a scheduling barrier after every slot. Callers never chain two
// on the same accumulator back to back (PV db-minor, QK^T alternating key blocks).
__device__ __forceinline__ void mfma32_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ void mfma32_v0(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  const f32x16 z = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, z, 0, 0, 0);
}
// Empty volatile asm on a value: the computation of x cannot move across the pin (inputs pinned at
// the start of a slot's VALU chunk, results at its end: the chunk stays between its two MFMAs).
template <typename T>
__device__ __forceinline__ void pin(T& x) {
  asm volatile("" : "+v"(x));
}
__device__ __forceinline__ void pin_s(int& x) { asm volatile("" : "+s"(x)); }
// The asm MFMAs are opaque to the compiler's hazard recognizer: a VALU read of an MFMA result needs
// the XDL-write -> VALU-read wait states (18 for a 16-pass op), and a VALU write read by an MFMA a few.
__device__ __forceinline__ void mfma_result_wait() {}
// LDS-DMA piece as inline asm: the compiler's waitcnt pass cannot tell which LDS bytes a
// buffer_load ... lds intrinsic writes, so it drained vmcnt(0) before the next ds_read of ANY slot
// (an HBM round trip per fragment read). The kernel orders its slots itself (vmcnt + barrier per
// iteration) and issues every LDS-DMA of the kernel through this, so M0 is never live for the compiler.
__device__ __forceinline__ void blds16_asm(i32x4 srd, int voff, int soff, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds_addr), "v"(voff), "s"(srd),
               "s"(soff));
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)p;
}

// NW = 8: two groups of 4 waves (query rows q_start + [0, 32) and + [32, 64)) share every K / V tile,
// so each SIMD runs two of these streams and one wave's dependency stalls are the other's issue slots.
// DIAG (stamp builds only, wrong results): 1 = no softmax chunks in the fast slots, 2 = no fragment reads
// PRIO_B: static s_setprio 1 for waves 4-7 over the tile loop (MI355X_MICROARCH.md "Two waves per SIMD"
// item 4: the second-dispatched half loses every arbitration otherwise).
// WIDE: the output tile goes through LDS and out as whole 256-B rows (16-B stores, 4 rows per wave
// instruction) instead of 16 8-B stores per lane into 32 different rows (MI355X_MICROARCH.md: the
// attention epilogue store tail is store-issue bound).
template <int NW = 4, bool STAMP = false, int DIAG = 0, int PRIO_B = 0, bool WIDE = false>
__global__ __launch_bounds__(NW * 64, NW / 4) void attn_prefill_v3_kernel(PrefillArgs a) {
  constexpr int D = 128;
  using C = Cfg<D>;
  __shared__ __attribute__((aligned(16))) char smem[2 * V3_NS * C::TILEB];  // [K slots][V slots] 128 KB
  __shared__ int s_bt[MAX_BT];

  constexpr int PPW = 16 / NW;  // DMA pieces per wave per K or V tile
  const int lane = threadIdx.x & 63;
  const int wid_u = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int tix, hg;
  prefill_block(a, tix, hg);
  const int seq = a.tiles[2 * tix], q_start = a.tiles[2 * tix + 1];
  const int G = a.Hq / a.Hkv;
  const int groups_per_kv = G / 4;
  const int kvh = hg / groups_per_kv;
  const int hq = kvh * G + (hg % groups_per_kv) * 4 + (wid_u & 3);
  const int pbase = q_start + 32 * (wid_u >> 2);

  const int q_off = a.cu_q[seq];
  const int q_len = a.cu_q[seq + 1] - q_off;
  const int kv_len = a.kv_lens[seq];
  const int ctx0 = kv_len - q_len;
  // block-uniform tile counts (every wave runs the same iterations and barriers)
  const int blk_qmax = min(q_start + 8 * NW, q_len) - 1;
  const int n_keys = min(kv_len, ctx0 + blk_qmax + 1);
  const int n_kt = (n_keys + KT - 1) / KT;
  const int h = lane >> 5, l32 = lane & 31;
  // tiles [0, n_fast) need no mask for any wave: every key <= the block's first query position and < kv_len
  const int n_fast = min((ctx0 + q_start + 1) / KT, kv_len / KT);

  // Q^T fragments (B operand): query pbase + l32, d = 16 s + 8 h + [0, 8)
  bf16x8 qf[8];
  {
    int qi = pbase + l32;
    qi = qi < q_len ? qi : q_len - 1;
    const bf16_t* qp = a.q + (size_t)(q_off + qi) * a.q_stride + hq * D + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
  }
  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;
  for (int i = threadIdx.x; i < n_kt; i += NW * 64) s_bt[i] = bt[i];

  // DMA: pieces PPW wid + i (i < PPW) of a 16-piece tile (rows 4 p .. 4 p + 3, one 16-B chunk per lane)
  int koff[PPW], voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = PPW * wid_u + i;
    const int row = p * C::RPP + lane / C::NC, ph = lane % C::NC;
    koff[i] = row * C::ROWB + 16 * (ph ^ kswz<D>(row));
    voff[i] = row * C::ROWB + 16 * (ph ^ vswz<D>(row));
  }
  const i32x4 srd_k = make_srd(a.k, a.kv_bytes);
  const i32x4 srd_v = make_srd(a.v, a.kv_bytes);
  const unsigned lds0 = lds_addr(smem);
  auto tile_soff = [&](int kt) {
    return __builtin_amdgcn_readfirstlane((int)((unsigned)(s_bt[kt] * a.Hkv + kvh) * (unsigned)(KT * D * 2)));
  };
  auto kslot_off = [&](int kt) { return (kt & (V3_NS - 1)) * C::TILEB; };
  auto vslot_off = [&](int kt) { return (V3_NS + (kt & (V3_NS - 1))) * C::TILEB; };
  auto stage_piece = [&](int kt, int soff, bool is_v, int i) {
    blds16_asm(is_v ? srd_v : srd_k, is_v ? voff[i] : koff[i], soff,
               lds0 + (is_v ? vslot_off(kt) : kslot_off(kt)) + (PPW * wid_u + i) * 1024);
  };
  auto stage = [&](int kt, bool is_v) {
    const int soff = tile_soff(kt);
#pragma unroll
    for (int i = 0; i < PPW; ++i) stage_piece(kt, soff, is_v, i);
  };

  // per-lane fragment offsets (bytes within a tile)
  // K (A of QK^T): row 32 kb + l32, chunk (2 s + h) ^ (l & 15) = 16 (h ^ (l & 1)) + 32 (s ^ ((l & 15) >> 1))
  const int kx = (lane & 15) >> 1;
  const int kbase = l32 * 256 + 16 * (h ^ (lane & 1));
  // V^T (A of PV): rows 16 ks + 4h + (i >> 2) [+ 8], chunk (2 (2 db + c16) + ((i >> 1) & 1)) ^ 2 (row & 7)
  const int vi = lane & 15, c16 = (lane >> 4) & 1;
  const int vrow = 4 * h + (vi >> 2);
  const int vbase = vrow * 256 + 16 * ((vi >> 1) & 1) + 8 * (vi & 1);
  const int vx = vrow & 7;
  auto kfrag = [&](int tile_off, int kb, int s) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + tile_off + kbase + kb * 32 * 256 + 32 * (s ^ kx));
  };
  auto vfrag = [&](int tile_off, int db, int ks) -> bf16x8 {
    const char* p = smem + tile_off + vbase + ks * 16 * 256 + 32 * ((2 * db + c16) ^ vx);
    const bf16x4 x0 = tr_read(p), x1 = tr_read(p + 8 * 256);
    return (bf16x8){x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  };

  f32x16 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;
  f32x16 S0[2], S1[2];
  bf16x8 P[4];
  // fragment of MFMA slot i in ring[i % V3_RING], read V3_PF slots ahead (LDS latency ~100+ cycles: at
  // 2 slots ahead every MFMA waited on its own ds_read)
  bf16x8 ring[V3_RING];
  const float c = a.scale_log2;

  __syncthreads();  // s_bt
#pragma unroll
  for (int kt = 0; kt < 3; ++kt)
    if (kt < n_kt) stage(kt, false);
  stage(0, true);
  if (n_kt > 1) stage(1, true);
  wait_vmcnt0();
  __syncthreads();

  auto pack_p32 = [&](const f32x16& A, int e0) -> bf16x8 {
    return (bf16x8){f2bf_s(A[e0]), f2bf_s(A[e0 + 1]), f2bf_s(A[e0 + 2]), f2bf_s(A[e0 + 3]),
                    f2bf_s(A[e0 + 4]), f2bf_s(A[e0 + 5]), f2bf_s(A[e0 + 6]), f2bf_s(A[e0 + 7])};
  };
  // simple (non-interleaved) pieces for the warm-up tile and the epilogue
  auto qk_simple = [&](int kt, f32x16 (&S)[2]) {
#pragma unroll
    for (int sd = 0; sd < 8; ++sd)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const bf16x8 f = kfrag(kslot_off(kt), kb, sd);
        if (sd == 0) mfma32_v0(S[kb], f, qf[sd]);
        else mfma32_v(S[kb], f, qf[sd]);
      }
  };
  auto pv_simple = [&](int kt) {
    const int vo = vslot_off(kt);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int db = 0; db < 4; ++db) mfma32_v(o[db], vfrag(vo, db, ks), P[ks]);
  };
  // whole-tile online softmax: this lane's query, 32 of the tile's 64 keys -> P; returns alpha
  auto softmax = [&](auto mask_tag, int k0, f32x16 (&S)[2]) -> float {
    constexpr bool MASK = decltype(mask_tag)::value;
    if constexpr (MASK) {
      const int qpos = ctx0 + pbase + l32;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int kj = k0 + 32 * kb + 8 * (e >> 2) + 4 * h + (e & 3);
          S[kb][e] = (kj < kv_len && kj <= qpos) ? S[kb][e] : -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) mx = fmaxf(mx, S[kb][e]);
    mx = max_xor32(mx);
    const float mxs = mx * c;
    const bool up = mxs > m_i + RESCALE_LOG2;
    const float alpha = up ? (m_i == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_i - mxs)) : 1.f;
    m_i = up ? mxs : m_i;
    const float mref = m_i == -INFINITY ? 0.f : m_i;
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float pe = __builtin_amdgcn_exp2f(__builtin_fmaf(S[kb][e], c, -mref));
        S[kb][e] = pe;
        ls += pe;
      }
    l_i = l_i * alpha + ls;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) P[ks] = pack_p32(S[ks >> 1], 8 * (ks & 1));
    return alpha;
  };
  auto rescale = [&](float alpha) {
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  unsigned long long stp[4] = {0, 0, 0, 0};
  // Fast iteration t (1 <= t < t_end: tile t unmasked, PV(t-1) and QK^T(t+1) exist). MFMA slots
  // 0..15: PV(t-1) (V slot t-1; ks = i / 4, db = i % 4), 16..31: QK^T(t+1) (K slot t+1; kb = i % 2,
  // d-step (i-16) / 2). Slot i reads the fragment of slot i + V3_PF; the last V3_PF slots read the
  // first PV(t) fragments of the next iteration. Softmax(t) of S_cur -> P in chunks. DMA: K(t+3) (slots 6..18),
  // V(t+2) (22..28). Then O *= alpha(t) (rare), vmcnt (this iteration's DMAs stay in flight), barrier.
  auto fast = [&](int t, f32x16 (&S_cur)[2], f32x16 (&S_next)[2]) {
    unsigned long long t0 = 0;
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    const int vo = vslot_off(t - 1), ko = kslot_off(t + 1), vno = vslot_off(t);
    const bool st_k = t + 3 < n_kt, st_v = t + 2 < n_kt;
    const int soff_k = tile_soff(st_k ? t + 3 : 0);
    const int soff_v = tile_soff(st_v ? t + 2 : 0);
    float alpha = 1.f, mx = -INFINITY, mref = 0.f, ls = 0.f, pend = 0.f;
    pp_static_for<32>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      // MFMA slot i
      if constexpr (i < 16) {
        mfma32_v(o[i % 4], ring[i % V3_RING], P[i / 4]);
      } else {
        constexpr int kb = i % 2, sd = (i - 16) / 2;
        if constexpr (sd == 0) mfma32_v0(S_next[kb], ring[i % V3_RING], qf[sd]);
        else mfma32_v(S_next[kb], ring[i % V3_RING], qf[sd]);
      }
      // fragment for slot i + V3_PF (the per-lane bases x tile offsets are CSE'd: 12 address adds per
      // iteration; the scheduling barrier at the end of the slot keeps each read in its slot)
      constexpr int j = i + V3_PF;
      if constexpr (DIAG != 2) {
        const int ao = j < 16 ? vo : (j < 32 ? ko : vno);
        if constexpr (j < 16) ring[j % V3_RING] = vfrag(ao, j % 4, j / 4);
        else if constexpr (j < 32) ring[j % V3_RING] = kfrag(ao, j % 2, (j - 16) / 2);
        else ring[j % V3_RING] = vfrag(ao, (j - 32) % 4, (j - 32) / 4);
      }
      // softmax chunk: max in slots 0..3, row statistics in 4, one element per slot from 5 on
      if constexpr (DIAG == 1) {
      } else if constexpr (i < 4) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = S_cur[i / 2][8 * (i % 2) + e];
          pin(v[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) mx = fmaxf(mx, v[e]);
        pin(mx);
      } else if constexpr (i == 4) {
        mx = max_xor32(mx);
        const float mxs = mx * c;
        const bool up = mxs > m_i + RESCALE_LOG2;
        alpha = up ? (m_i == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_i - mxs)) : 1.f;
        m_i = up ? mxs : m_i;
        mref = m_i == -INFINITY ? 0.f : m_i;
        pin(alpha);
        pin(m_i);
        pin(mref);
      } else {
        // elements x with 5 + (27 x) / 32 == i; each exp result is added to the row sum one element
        // later (no exp -> add dependency inside a slot: that was a wait state per element)
        pp_static_for<32>([&](auto xc) {
          constexpr int x = decltype(xc)::value;
          if constexpr (5 + (27 * x) / 32 == i) {
            float sv = S_cur[x >> 4][x & 15];
            pin(sv);
            ls += pend;
            const float pe = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -mref));
            S_cur[x >> 4][x & 15] = pe;
            pend = pe;
            if constexpr (x % 8 == 7) {
              P[x / 8] = pack_p32(S_cur[x / 16], 8 * ((x / 8) & 1));
              pin(P[x / 8]);
            }
            pin(ls);
            pin(pend);
          }
        });
      }
      // DMA pieces: K(t+3) in slots 6, 10, 14, 18; V(t+2) in slots 22, 24, 26, 28 (the first PPW of each)
      if constexpr (i >= 6 && i <= 18 && (i - 6) % 4 == 0 && (i - 6) / 4 < PPW) {
        if (st_k) stage_piece(t + 3, soff_k, false, (i - 6) / 4);
      }
      if constexpr (i >= 22 && i <= 28 && (i - 22) % 2 == 0 && (i - 22) / 2 < PPW) {
        if (st_v) stage_piece(t + 2, soff_v, true, (i - 22) / 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    l_i = l_i * alpha + (ls + pend);
    if constexpr (STAMP) {
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      stp[0] += t1 - t0;
      t0 = t1;
    }
    rescale(alpha);
    // this iteration's DMAs (PPW per issued tile) stay in flight, the previous iteration's have landed
    if constexpr (PPW == 4) {
      if (st_k && st_v) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (st_k || st_v) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else wait_vmcnt0();
    } else {
      if (st_k && st_v) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (st_k || st_v) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else wait_vmcnt0();
    }
    barrier();
    if constexpr (STAMP) stp[1] += __builtin_amdgcn_s_memtime() - t0;
  };

  unsigned long long te = 0;
  if constexpr (STAMP) te = __builtin_amdgcn_s_memtime();
  if constexpr (PRIO_B) {
    if (wid_u >= 4) __builtin_amdgcn_s_setprio(1);
  }
  qk_simple(0, S0);  // S(0)
  mfma_result_wait();
  // fast iterations: [1, t_end); warm-up tile 0 when there is at least one
  const int t_end = min(n_fast, n_kt - 1);
  int t = 0;
  if (t_end >= 1) {
    // tile 0 (unmasked, QK^T(1) exists): softmax(0), S(1), DMA K(3) / V(2), the first PV(0) fragments
    softmax(std::false_type{}, 0, S0);
    qk_simple(1, S1);
    mfma_result_wait();
    if (3 < n_kt) stage(3, false);
    if (2 < n_kt) stage(2, true);
#pragma unroll
    for (int j = 0; j < V3_PF; ++j) ring[j] = vfrag(vslot_off(0), j % 4, j / 4);
    barrier();  // (O is zero: no rescale; the prologue DMAs were drained)
    t = 1;
    for (; t + 1 < t_end; t += 2) {
      fast(t, S1, S0);
      fast(t + 1, S0, S1);
    }
    if (t < t_end) {
      fast(t, S1, S0);
      ++t;
    }
    if (t & 1) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) S0[kb] = S1[kb];
    }
  }
  if constexpr (STAMP) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    stp[2] += t1 - te - stp[0] - stp[1];
    te = t1;
  }
  // epilogue: tiles [t, n_kt) (masked diagonal / ragged ones and the last; at most 3), S(t) in S0, P(t-1)
  // pending. Every tile they touch is staged after V(t + 2) here (the ring holds it), then drained.
  if (t + 2 < n_kt) stage(t + 2, true);
  wait_vmcnt0();
  barrier();
  if (t >= 1) pv_simple(t - 1);
  for (; t < n_kt; ++t) {
    const int k0 = t * KT;
    const bool need_mask = (k0 + KT - 1 > ctx0 + pbase) || (k0 + KT > kv_len);
    mfma_result_wait();  // S(t) and O from the MFMAs just issued
    const float alpha = need_mask ? softmax(std::true_type{}, k0, S0) : softmax(std::false_type{}, k0, S0);
    rescale(alpha);
    pv_simple(t);
    if (t + 1 < n_kt) qk_simple(t + 1, S0);
  }
  if constexpr (STAMP) stp[3] += __builtin_amdgcn_s_memtime() - te;
  if constexpr (STAMP) {
    if (lane == 0 && g_attn_dbg) {
      unsigned long long* d = g_attn_dbg + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * NW + wid_u) * 6;
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = stp[i];
      d[4] = n_kt;
      d[5] = max(0, min(n_fast, n_kt - 1) - 1);  // fast iterations
    }
  }

  // finalize: O^T[32 db + 8 b + 4 h + r][query] = o[db][4 b + r] / l; {r0, r1} = {l_i, partner's l_i}
  const auto lr = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_i), __float_as_uint(l_i), false, false);
  const float l = __uint_as_float(lr[0]) + __uint_as_float(lr[1]);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  const int qi = pbase + l32;
  if constexpr (WIDE) {
    // every wave is past its last K / V slot read (the loop's barrier count is the same in both groups),
    // so the ring is free: each wave stages its 32 x 128 bf16 tile (8 KiB, rows of 256 B, 16-B chunk c of
    // row r at slot c ^ (r & 15)) and stores whole rows
    __syncthreads();
    char* so = smem + wid_u * 8192;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int e = 4 * b;
        const int d = 32 * db + 8 * b + 4 * h;  // 4 values: chunk d / 8, half (d / 4) & 1
        const int c = (d >> 3) ^ (l32 & 15);
        *reinterpret_cast<uint2*>(so + l32 * 256 + 16 * c + 8 * ((d >> 2) & 1)) =
            make_uint2(pk2bf(o[db][e] * inv, o[db][e + 1] * inv), pk2bf(o[db][e + 2] * inv, o[db][e + 3] * inv));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes, read back by itself
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 4 * i + (lane >> 4), c = lane & 15;
      const u32x4 v = *reinterpret_cast<const u32x4*>(so + r * 256 + 16 * (c ^ (r & 15)));
      if (pbase + r < q_len)
        *reinterpret_cast<u32x4*>(a.out + (size_t)(q_off + pbase + r) * a.out_stride + hq * D + 8 * c) = v;
    }
    return;
  }
  if (qi < q_len) {
    bf16_t* op = a.out + (size_t)(q_off + qi) * a.out_stride + hq * D + 4 * h;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int e = 4 * b;
        *reinterpret_cast<uint2*>(op + 32 * db + 8 * b) =
            make_uint2(pk2bf(o[db][e] * inv, o[db][e + 1] * inv), pk2bf(o[db][e + 2] * inv, o[db][e + 3] * inv));
      }
  }
}

// ------------------------------------------------------------------------------------
// Decode attention (one query token per sequence), split-K over context partitions.
// ------------------------------------------------------------------------------------
struct DecodeArgs {
  const bf16_t* q; int q_stride;           // [B] rows, head h at +h*D
  const bf16_t* kc; const bf16_t* vc;      // paged caches
  const int* block_tables; int bt_stride;
  const int* kv_lens;                      // [B]
  float* part_o;                           // [B][Hq][max_parts][D]
  float* part_ml;                          // [B][Hq][max_parts][2]
  bf16_t* out; int out_stride;
  int Hq, Hkv, part_tiles, max_parts;
  float scale_log2;
  int* counters;                           // [B][Hkv] zeroed tickets: fused split-K merge (null: separate
                                           // attn_decode_reduce_kernel launch)
  // Fused RoPE + KV append (null qkv_p: q is read from `q` and the cache already holds the new token).
  // The qkv projection arrives as fp32 split-K partial slabs P[S][B][ldp] (gemm_part.hip); every
  // block sums + rotates its G query heads itself, and the block owning the last KV tile also sums,
  // rotates and appends the new token's k / v before reading that tile.
  const float* qkv_p; long long p_slab; int ldp, S;
  const int* positions; const int* slots;
  const float* cos_t; const float* sin_t;
  int nb;                                  // batch (0: gridDim.z, the 3-D launch)
};

// Tiles per partition of one sequence: its KV tiles spread evenly over all max_parts partitions
// (never fewer than part_tiles per partition). The grid is sized once for max_parts (hipGraph
// capture), so sizing the split from the actual length keeps every launched block busy with the
// same amount of KV: splitting a 5.3k-token context by a fixed 32-tile partition left 1 of 4
// partitions idle and 8 vs 5 tiles per wave on the others.
__device__ __forceinline__ int decode_part_tiles(int n_kt, const DecodeArgs& a) {
  return max(a.part_tiles, (n_kt + a.max_parts - 1) / a.max_parts);
}

// LDS of one decode-attention block: one V tile per wave, then the block's rotated q (G x D bf16).
template <int D, int G, int NW = 4>
constexpr int decode_lds_bytes() { return NW * Cfg<D>::TILEB + G * D * 2; }

// Signal of a decode-attention block inside the fused attention + o_proj launch (attn_oproj_kernel):
// every storing wave has drained its write-through (sc1) stores, then one lane adds to the agent-scope
// counter the o_proj blocks poll (MI355X_MICROARCH.md "Valid forms": sc1 stores, vmcnt(0), barrier,
// agent atomic; the consumer polls with sc1 loads and reads the bytes with sc1 loads only).
// Stage hand-off of the fused launches: arrivals count on ONE counter; the block whose add returns
// total - 1 (every other producer's stores were drained before its add) raises a done flag in FL_REPL
// replicas, each on its own 128-B line, and consumers poll the replica of their block index with a long
// s_sleep -- hundreds of pollers on the counter itself (one line, hammered while it is being
// incremented) slowed the whole launch (MI355X_MICROARCH.md polling-cost / fanin).
// In-kernel stamps of the fused launches (diagnostic instantiation only, tools/fused_stamps.py): lane 0
// of a block writes s_memrealtime (100 MHz, device-wide) at stage boundaries into g_fused_stamps[block][k].
__device__ unsigned long long* g_fused_stamps;
template <bool ST>
__device__ __forceinline__ void fstamp(int k) {
  if constexpr (ST) {
    if (threadIdx.x == 0) g_fused_stamps[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
  }
}
constexpr int FL_REPL = 16;       // flag replicas
constexpr int FL_STRIDE = 32;     // ints between replicas (128 B)
constexpr int FL_A = 64;          // cnt offset of the attention-done flags
constexpr int FL_Q = FL_A + FL_REPL * FL_STRIDE;  // cnt offset of the qkv-done flags
constexpr int FL_P = FL_Q + FL_REPL * FL_STRIDE;           // v2: "attention KV prefetch issued" flags
constexpr int CNT_TICKETS = FL_P + FL_REPL * FL_STRIDE;  // MIA: per (sequence, KV head) merge tickets
constexpr int CNT_SS = CNT_TICKETS + 4 * 64;               // v2 o_proj: [4][<= 512] sum-of-squares partials
constexpr int CNT_INTS = CNT_SS + 4 * 512;
__device__ __forceinline__ void stage_arrive(int* cnt, int total, int* flags) {
  wait_vmcnt0();
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
#pragma unroll
      for (int k = 0; k < FL_REPL; ++k) __hip_atomic_store(flags + k * FL_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One split-K partition block of decode attention: partition `part` of KV head `kvh` of sequence `b`.
// FUSED (attn_oproj_kernel): the partition record is written write-through even for a single-partition
// sequence (the o_proj blocks merge records only), there is no merge here, and the block signals
// `fused_cnt` when its records are out -- also when it has no tiles (the counter counts every block).
// qkv slab sum of sum_partials8x2 with write-through (sc1) buffer loads: the slabs were produced by
// other blocks of the same launch (attn_oproj_kernel's qkv blocks). off1 / off2: byte offsets of the two
// 8-float runs in slab 0, slab_b: bytes per slab. Same summation order.
__device__ __forceinline__ void sum_partials8x2_sc1(__amdgpu_buffer_rsrc_t rs, int off1, int off2, int S, int slab_b,
                                                    float* a, float* b) {
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  for (int s0 = 0; s0 < S; s0 += PSU) {
    u32x4 p[PSU][4];
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      const int o = min(s0 + u, S - 1) * slab_b;
      p[u][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off1 + o, 0, 16));
      p[u][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off1 + o + 16, 0, 16));
      p[u][2] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off2 + o, 0, 16));
      p[u][3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off2 + o + 16, 0, 16));
    }
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      if (s0 + u < S) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] += __uint_as_float(p[u][0][e]);
          a[4 + e] += __uint_as_float(p[u][1][e]);
          b[e] += __uint_as_float(p[u][2][e]);
          b[4 + e] += __uint_as_float(p[u][3][e]);
        }
      }
    }
  }
}

// Bounded poll of an agent-scope counter by one lane (sc1 loads), then the block's barrier. Sets err[0]
// and gives up (the block computes garbage, never hangs) after `limit` s_memrealtime ticks.
__device__ __forceinline__ void wait_flag(const int* flags, int* err, unsigned limit) {
  if (threadIdx.x == 0) {
    const int* f = flags + (blockIdx.x % FL_REPL) * FL_STRIDE;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      __builtin_amdgcn_s_sleep(8);
      if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}


struct QWait {       // attention blocks waiting for the in-launch qkv blocks (QW mode)
  const int* flags;  // qkv-done flag replicas
  int* err;
  unsigned limit;
};

// bf16 pair (d, d + 1) of an attention output row, stored write-through for the o_proj blocks of the
// same launch (4 B per store: a 2-B write-through store costs ~2x per byte).
__device__ __forceinline__ void out_pair_sc1(const DecodeArgs& a, int b, int col, float x, float y) {
  const int nb = a.nb ? a.nb : (int)gridDim.z;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, nb * a.out_stride * 2, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(pk2bf(x, y), rs, (b * a.out_stride + col) * 2, 0, 16);
}

// MIA (FUSED only): the partitions of a (sequence, KV head) are merged by the last of its partition blocks
// (ticket counters a.counters) into the bf16 attention output, written through; the o_proj blocks then
// stage a plain bf16 activation slice instead of each merging the records of its K-slice.
// NW: waves per block (4; 8 for the batch-32 grid with one partition per sequence: one 8-wave block per
// CU keeps the same KV bytes in flight as two 4-wave blocks and needs no merge launch)
template <int D, int G, bool NT = false, bool FUSED = false, bool QW = false, bool MIA = false, bool ST = false,
          int NW = 4>
__device__ __forceinline__ void attn_decode_block(const DecodeArgs& a, int part, int kvh, int b, char* smem,
                                                  int* fused_cnt = nullptr, QWait qw = {}, int fused_total = 0) {
  static_assert(NW == 4 || (NW == 8 && !FUSED), "8-wave blocks: the plain decode kernel only");
  constexpr int NTH = NW * 64;
  fstamp<ST>(0);
  using C = Cfg<D>;
  static_assert(G <= 16, "at most 16 query heads per KV head");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int kv_len = a.kv_lens[b];
  const int n_kt = (kv_len + KT - 1) / KT;
  const int pt = decode_part_tiles(n_kt, a);
  const int kt0 = part * pt;
  if (kt0 >= n_kt) {  // block-uniform early exit (before any barrier)
    if constexpr (FUSED && MIA) {
      if (threadIdx.x == 0 &&
          __hip_atomic_fetch_add(fused_cnt + 5, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fused_total - 1) {
#pragma unroll
        for (int k = 0; k < FL_REPL; ++k)
          __hip_atomic_store(fused_cnt + FL_P + k * FL_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (FUSED) stage_arrive(fused_cnt, fused_total, fused_cnt + FL_A);
    return;
  }
  const int kt1 = min(kt0 + pt, n_kt);
  const int nparts = (n_kt + pt - 1) / pt;
  const int fr = lane & 15, fh = lane >> 4;
  const int* bt = a.block_tables + (size_t)b * a.bt_stride;

  bf16x8 qf[C::KS];
  // Fused-RoPE path: this wave's first KV tile is requested BEFORE the q prologue (K straight to
  // registers, V to the wave's LDS tile), so its HBM latency overlaps the qkv partial-slab loads instead
  // of following them -- at batch 1 a wave handles a single tile and the two latencies were in series.
  // Not for the sequence's last tile: the new token's k / v is appended into it during the prologue.
  char* sV = smem + wid * C::TILEB;
  const bool pre = a.qkv_p != nullptr && kt0 + wid_u < kt1 && kt0 + wid_u != n_kt - 1;  // wave-uniform
  bf16x8 kf0[4][C::KS];
  if (pre) {
    const size_t base = ((size_t)bt[kt0 + wid_u] * a.Hkv + kvh) * KT * D;
    const bf16_t* kb = a.kc + base;
    const bf16_t* vb = a.vc + base;
    stage_kv<D, true, NT, 1>(sV, 0, 1, lane, [&](int r) { return vb + (size_t)r * D; });
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < C::KS; ++s)
        kf0[t][s] = NT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D +
                                                                                   32 * s + 8 * fh))
                       : *reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D + 32 * s + 8 * fh);
  }
  fstamp<ST>(1);
  if constexpr (FUSED && MIA) {
    // tell the o_proj blocks this block's KV requests are out (their weight stream queues behind them;
    // nothing is handed off, so no drain): counter cnt[5], flags FL_P
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(fused_cnt + 5, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fused_total - 1) {
#pragma unroll
      for (int k = 0; k < FL_REPL; ++k)
        __hip_atomic_store(fused_cnt + FL_P + k * FL_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (QW) wait_flag(qw.flags, qw.err, qw.limit);  // the KV prefetch above is in flight
  fstamp<ST>(2);
  if (a.qkv_p != nullptr) {
    // q = RoPE(bf16(sum_s P[s][b])) for this KV head's G query heads, one (d, d + D/2) rotate_half
    // pair of 8-vectors per thread (G * D/16 threads, all slab loads of a thread in flight together),
    // staged through LDS; in the block owning the last KV tile, other threads append the new
    // token's k (rotated) and v meanwhile. One barrier covers both.
    bf16_t* s_q = reinterpret_cast<bf16_t*>(smem + NW * C::TILEB);
    constexpr int NV = D / 16;  // pairs per head
    const int pos = a.positions[b];
    const float* prow = a.qkv_p + (size_t)b * a.ldp;
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rs_qkv = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.qkv_p), (short)0, (int)(a.p_slab * a.S * 4), 0x00020000);
    const float* ct = a.cos_t + (size_t)pos * (D / 2);
    const float* st = a.sin_t + (size_t)pos * (D / 2);
    const int tid = threadIdx.x;
    const bool append = kt1 == n_kt;  // block-uniform
    constexpr int KV0 = (G * NV + 63) / 64 * 64;  // append threads start on a fresh wave
    if (tid < G * NV) {
      const int g = tid / NV, v = tid % NV;
      const float* ph = prow + (size_t)(kvh * G + g) * D + 8 * v;
      float x1[8], x2[8], o1[8], o2[8];
      if constexpr (QW) {
        const int o = (int)((ph - a.qkv_p) * 4);
        sum_partials8x2_sc1(rs_qkv, o, o + D * 2, a.S, (int)(a.p_slab * 4), x1, x2);
      } else {
        sum_partials8x2(ph, ph + D / 2, a.S, (size_t)a.p_slab, x1, x2);
      }
      rope8(x1, x2, ct + 8 * v, st + 8 * v, o1, o2);
      *reinterpret_cast<u32x4*>(s_q + g * D + 8 * v) = pack8(o1);
      *reinterpret_cast<u32x4*>(s_q + g * D + D / 2 + 8 * v) = pack8(o2);
    } else if (append && tid >= KV0 && tid < KV0 + 2 * NV) {  // [KV0, KV0+NV): k, [KV0+NV, KV0+2NV): v
      const int isv = tid - KV0 >= NV, v = (tid - KV0) % NV;
      const int slot = a.slots[b];
      const size_t kvo = (((size_t)(slot / KT) * a.Hkv + kvh) * KT + (slot % KT)) * D;
      const float* ph = prow + (size_t)(a.Hq + (isv ? a.Hkv : 0) + kvh) * D + 8 * v;
      float x1[8], x2[8];
      if constexpr (QW) {
        const int o = (int)((ph - a.qkv_p) * 4);
        sum_partials8x2_sc1(rs_qkv, o, o + D * 2, a.S, (int)(a.p_slab * 4), x1, x2);
      } else {
        sum_partials8x2(ph, ph + D / 2, a.S, (size_t)a.p_slab, x1, x2);
      }
      bf16_t* dst = (isv ? const_cast<bf16_t*>(a.vc) : const_cast<bf16_t*>(a.kc)) + kvo;
      if (isv) {
        *reinterpret_cast<u32x4*>(dst + 8 * v) = pack8(x1);
        *reinterpret_cast<u32x4*>(dst + D / 2 + 8 * v) = pack8(x2);
      } else {
        float o1[8], o2[8];
        rope8(x1, x2, ct + 8 * v, st + 8 * v, o1, o2);
        *reinterpret_cast<u32x4*>(dst + 8 * v) = pack8(o1);
        *reinterpret_cast<u32x4*>(dst + D / 2 + 8 * v) = pack8(o2);
      }
    }
    __syncthreads();  // q in LDS; the appended row visible to every wave of this block (same CU)
#pragma unroll
    for (int s = 0; s < C::KS; ++s)
      qf[s] = fr < G ? *reinterpret_cast<const bf16x8*>(s_q + fr * D + 32 * s + 8 * fh)
                     : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  } else {
    const int g = fr < G ? fr : 0;
    const bf16_t* qp = a.q + (size_t)b * a.q_stride + (kvh * G + g) * D + 8 * fh;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
      qf[s] = fr < G ? v : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  f32x4 o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_i = -INFINITY, l_i = 0.f;

  for (int kt = kt0 + wid_u; kt < kt1; kt += NW) {
    bf16x8 kf[4][C::KS];
    if (pre && kt == kt0 + wid_u) {  // requested before the prologue
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s) kf[t][s] = kf0[t][s];
    } else {
      const size_t base = ((size_t)bt[kt] * a.Hkv + kvh) * KT * D;
      const bf16_t* kb = a.kc + base;
      const bf16_t* vb = a.vc + base;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous tile's V reads retired
      // V tile -> wave-private LDS (transposed reads later)
      stage_kv<D, true, NT, 1>(sV, 0, 1, lane, [&](int r) { return vb + (size_t)r * D; });
      // K fragments straight to VGPRs
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s)
          kf[t][s] = NT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D +
                                                                                    32 * s + 8 * fh))
                        : *reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D + 32 * s + 8 * fh);
    }
    f32x4 s4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s4[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) s4[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][s], qf[s], s4[t], 0, 0, 0);
    }
    const int k0 = kt * KT;
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = k0 + 16 * t + 4 * fh + r;
        const float x = kj < kv_len ? s4[t][r] * a.scale_log2 : -INFINITY;
        s4[t][r] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_i, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m_i - m_use);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s4[t][r] - m_use);
        s4[t][r] = p;
        ls += p;
      }
    l_i = l_i * alpha + ls;
    m_i = m_new;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) o[dt] *= alpha;
    const bf16x8 pb0 = pack_p(s4[0], s4[1]);
    const bf16x8 pb1 = pack_p(s4[2], s4[3]);
    wait_vmcnt0();  // V tile landed in this wave's LDS
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_vt<D>(sV, dt, 0, lane), pb0, o[dt], 0, 0, 0);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_vt<D>(sV, dt, 1, lane), pb1, o[dt], 0, 0, 0);
    }
  }

  fstamp<ST>(3);
  // partition-statistics buffers as write-through (sc1) buffer resources for the fused merge
  const unsigned pbytes = (unsigned)((size_t)(a.nb ? a.nb : (int)gridDim.z) * a.Hq * a.max_parts * 4);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(a.part_o, (short)0, (int)(pbytes * D), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_ml = __builtin_amdgcn_make_buffer_rsrc(a.part_ml, (short)0, (int)(pbytes * 2), 0x00020000);

  // ---- combine the 4 waves in LDS ----
  __syncthreads();
  float* sm = reinterpret_cast<float*>(smem);    // [4][16] max
  float* sl = sm + NW * 16;                      // [NW][64] partial l (per lane)
  float* so = sl + NW * 64;                      // [NW][16][D] O
  if (fh == 0) sm[wid * 16 + fr] = m_i;
  sl[wid * 64 + lane] = l_i;
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) so[(wid * 16 + fr) * D + 16 * dt + 4 * fh + r] = o[dt][r];
  __syncthreads();
  if constexpr (FUSED && MIA) {
    if (nparts == 1) {  // the block's output is final: bf16 pairs, written through
      for (int e2 = threadIdx.x; e2 < G * D / 2; e2 += NTH) {
        const int g = (2 * e2) / D, d = (2 * e2) % D;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w * 16 + g]);
        const float Mu = M == -INFINITY ? 0.f : M;
        float L = 0.f, O0 = 0.f, O1 = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const float sc = exp2f(sm[w * 16 + g] - Mu);
          L += (sl[w * 64 + g] + sl[w * 64 + g + 16] + sl[w * 64 + g + 32] + sl[w * 64 + g + 48]) * sc;
          O0 += so[(w * 16 + g) * D + d] * sc;
          O1 += so[(w * 16 + g) * D + d + 1] * sc;
        }
        out_pair_sc1(a, b, (kvh * G + g) * D + d, L > 0.f ? O0 / L : 0.f, L > 0.f ? O1 / L : 0.f);
      }
      fstamp<ST>(4);
      stage_arrive(fused_cnt, fused_total, fused_cnt + FL_A);
      fstamp<ST>(5);
      return;
    }
  }
  // thread -> (g, d) pairs
  for (int e = threadIdx.x; e < G * D; e += NTH) {
    const int g = e / D, d = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w * 16 + g]);
    const float Mu = M == -INFINITY ? 0.f : M;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float sc = exp2f(sm[w * 16 + g] - Mu);
      L += (sl[w * 64 + g] + sl[w * 64 + g + 16] + sl[w * 64 + g + 32] + sl[w * 64 + g + 48]) * sc;
      O += so[(w * 16 + g) * D + d] * sc;
    }
    const int hq = kvh * G + g;
    if (nparts == 1 && !FUSED) {
      a.out[(size_t)b * a.out_stride + hq * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const size_t pi = ((size_t)b * a.Hq + hq) * a.max_parts + part;
      if (FUSED || a.counters) {  // write-through (sc1) stores, read back by another CU
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(O), rs_o, (int)((pi * D + d) * 4), 0, 16);
        if (d == 0) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), rs_ml, (int)(pi * 8), 0, 16);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), rs_ml, (int)(pi * 8 + 4), 0, 16);
        }
      } else {
        a.part_o[pi * D + d] = O;
        if (d == 0) {
          a.part_ml[pi * 2] = M;
          a.part_ml[pi * 2 + 1] = L;
        }
      }
    }
  }
  if constexpr (FUSED && !MIA) {
    stage_arrive(fused_cnt, fused_total, fused_cnt + FL_A);
    return;
  }
  if (!FUSED && (nparts == 1 || a.counters == nullptr)) return;

  // ---- fused split-K merge: the last of this (b, kvh)'s nparts partition blocks to finish merges
  // them (same math as attn_decode_reduce_kernel), so the merge costs no extra launch. The partials
  // were stored write-through (sc1) and are read back with sc1 loads, so no agent-scope release or
  // acquire fence is needed for any block -> XCD placement (an L2 write-back per block cost more than
  // the merge launch it saved).
  __shared__ int s_last;
  wait_vmcnt0();  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(a.counters + b * a.Hkv + kvh, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old == nparts - 1);
  }
  __syncthreads();
  if (!s_last) {
    fstamp<ST>(4);
    if constexpr (FUSED) stage_arrive(fused_cnt, fused_total, fused_cnt + FL_A);
    fstamp<ST>(5);
    return;
  }
  asm volatile("" ::: "memory");  // the sc1 loads below stay after the ticket
  const size_t hb = (size_t)b * a.Hq + kvh * G;  // first query head of this KV head
  if constexpr (FUSED) {
    // Merge on the critical path of the fused launch: each thread's partial-output records of its (head,
    // d pair)s for the first MCH partitions are requested first, then the (max, sum) statistics (into LDS),
    // so both are in flight together -- one memory round trip for <= MCH partitions -- and merged in
    // registers once the per-partition scales are known.
    constexpr int MCH = 16;
    constexpr int NPR = (G * D / 2 + NTH - 1) / NTH;  // (head, pair) items per thread
    float* s_m = reinterpret_cast<float*>(smem);  // [G][nparts] max -> scale
    float* s_l = s_m + G * nparts;
    float* s_L = s_l + G * nparts;
    f32x2 v[NPR][MCH];
#pragma unroll
    for (int k = 0; k < NPR; ++k) {
      const int e2 = min((int)threadIdx.x + NTH * k, G * D / 2 - 1);
      const int g = (2 * e2) / D, d = (2 * e2) % D;
      const int po = (int)(((hb + g) * a.max_parts * D + d) * 4);
#pragma unroll
      for (int i = 0; i < MCH; ++i)
        v[k][i] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_o, po + min(i, nparts - 1) * D * 4, 0, 16));
    }
    for (int e = threadIdx.x; e < G * nparts; e += NTH) {
      const int g = e / nparts, p = e % nparts;
      const f32x2 ml = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_ml, (int)(((hb + g) * a.max_parts + p) * 8), 0, 16));
      s_m[e] = ml[0];
      s_l[e] = ml[1];
    }
    __syncthreads();
    if (threadIdx.x < G) {
      const int g = threadIdx.x;
      float Mx = -INFINITY;
      for (int p = 0; p < nparts; ++p) Mx = fmaxf(Mx, s_m[g * nparts + p]);
      const float Mu = Mx == -INFINITY ? 0.f : Mx;
      float L = 0.f;
      for (int p = 0; p < nparts; ++p) {
        const float sc = exp2f(s_m[g * nparts + p] - Mu);
        s_m[g * nparts + p] = sc;
        L += s_l[g * nparts + p] * sc;
      }
      s_L[g] = L;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPR; ++k) {
      const int e2 = threadIdx.x + NTH * k;
      if (e2 >= G * D / 2) break;
      const int g = (2 * e2) / D, d = (2 * e2) % D;
      const float* sc = s_m + g * nparts;
      float O0 = 0.f, O1 = 0.f;
#pragma unroll
      for (int i = 0; i < MCH; ++i) {
        const float f = i < nparts ? sc[i] : 0.f;
        O0 += v[k][i][0] * f;
        O1 += v[k][i][1] * f;
      }
      const int po = (int)(((hb + g) * a.max_parts * D + d) * 4);
      for (int p0 = MCH; p0 < nparts; p0 += MCH) {  // long contexts: further rounds of MCH records
        f32x2 w[MCH];
#pragma unroll
        for (int i = 0; i < MCH; ++i)
          w[i] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_o, po + min(p0 + i, nparts - 1) * D * 4, 0, 16));
#pragma unroll
        for (int i = 0; i < MCH; ++i) {
          const float f = p0 + i < nparts ? sc[p0 + i] : 0.f;
          O0 += w[i][0] * f;
          O1 += w[i][1] * f;
        }
      }
      const float L = s_L[g];
      out_pair_sc1(a, b, (kvh * G + g) * D + d, L > 0.f ? O0 / L : 0.f, L > 0.f ? O1 / L : 0.f);
    }
    if (threadIdx.x == 0) __hip_atomic_store(a.counters + b * a.Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fstamp<ST>(6);
    stage_arrive(fused_cnt, fused_total, fused_cnt + FL_A);
    fstamp<ST>(5);
    return;
  }
  float* s_m = reinterpret_cast<float*>(smem);  // [G][nparts] partition max, then its scale
  float* s_l = s_m + G * nparts;                 // [G][nparts] partition sum
  float* s_L = s_l + G * nparts;                 // [G] merged sum
  for (int e = threadIdx.x; e < G * nparts; e += NTH) {
    const int g = e / nparts, p = e % nparts;
    const size_t pi = (hb + g) * a.max_parts + p;
    s_m[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_ml, (int)(pi * 8), 0, 16));
    s_l[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_ml, (int)(pi * 8 + 4), 0, 16));
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    float Mx = -INFINITY;
    for (int p = 0; p < nparts; ++p) Mx = fmaxf(Mx, s_m[g * nparts + p]);
    const float Mu = Mx == -INFINITY ? 0.f : Mx;
    float L = 0.f;
    for (int p = 0; p < nparts; ++p) {
      const float sc = exp2f(s_m[g * nparts + p] - Mu);
      s_m[g * nparts + p] = sc;
      L += s_l[g * nparts + p] * sc;
    }
    s_L[g] = L;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * D; e += NTH) {
    const int g = e / D, d = e % D;
    const int po = (int)(((hb + g) * a.max_parts * D + d) * 4);  // byte offset of partition 0
    const float* sc = s_m + g * nparts;
    float O = 0.f;
    int p = 0;
    for (; p + 8 <= nparts; p += 8) {  // 8 independent loads in flight
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_o, po + (p + i) * D * 4, 0, 16));
#pragma unroll
      for (int i = 0; i < 8; ++i) O += v[i] * sc[p + i];
    }
    for (; p < nparts; ++p) O += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_o, po + p * D * 4, 0, 16)) * sc[p];
    const float L = s_L[g];
    a.out[(size_t)b * a.out_stride + (kvh * G + g) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
  if (threadIdx.x == 0) __hip_atomic_store(a.counters + b * a.Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D, int G, bool NT = false, int NW = 4>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void attn_decode_kernel(DecodeArgs a, PfArgs pf) {
  __shared__ __attribute__((aligned(16))) char smem[decode_lds_bytes<D, G, NW>()];
  if ((int)blockIdx.x >= a.max_parts) {  // MALL prefetch rider (block-uniform): x beyond the partitions
    const int ex = gridDim.x - a.max_parts;
    pf_rider(pf, (blockIdx.x - a.max_parts) + ex * (blockIdx.y + gridDim.y * blockIdx.z), ex * gridDim.y * gridDim.z);
    return;
  }
  attn_decode_block<D, G, NT, false, false, false, false, NW>(a, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// ------------------------------------------------------------------------------------
// Fused decode attention + o_proj (batch <= 4): one launch instead of attention -> o_proj.
// ------------------------------------------------------------------------------------
// Blocks [0, na) are attention partition blocks (attn_decode_block<FUSED>); blocks [na, na + nob) are
// o_proj split-K blocks. An o_proj block issues its whole weight slice (64 output columns x KS, straight
// to VGPRs, non-temporal) as soon as it is dispatched -- while the attention blocks still stream the KV
// cache -- then polls the attention-done counter, merges the split-K partitions of the heads of its
// K-slice into an LDS activation slice and runs the MFMAs; its fp32 partial slab goes to the
// add_partials_rmsnorm consumer as gemm_part_merge's does. The o_proj weight stream (33.5 MB per layer
// at 8B) overlaps the attention instead of following it. Deadlock-free by construction: only o_proj
// blocks wait, and only on attention blocks, which have lower indices (dispatched first) and never
// wait; the wait is bounded anyway (error word, never a hang). Counters: cnt[0] attention blocks done,
// cnt[1] o_proj blocks past their wait (the last one re-arms both for the next layer / replay),
// cnt[2] error.
struct OprojArgs {
  const bf16_t* W; int ldw;  // o_proj weight [N][K] bf16
  float* P;                  // [K / KS][M][N] fp32 partial slabs
  int M, N, K;
  int na, nob;               // attention blocks, o_proj blocks
  int* cnt;
  unsigned spin_limit;       // s_memrealtime ticks (100 MHz)
  // optional residual + RMSNorm tail (add_partials_rmsnorm's math, done by the last o_proj block):
  // h[M][ldh] += bf16(sum of the slabs) (bf16), xn[M][ldx] = rmsnorm(h) * gamma. h == nullptr: none.
  bf16_t* h; int ldh;
  const bf16_t* gamma;
  bf16_t* xn; int ldx;
  float eps;
  float* ss;                 // v2 tail: [4][nob] per-block sum-of-squares partials
};
constexpr int OP_MAXP = 64;  // partitions per (row, head) merged in LDS

template <int D, int NLD, bool MIA = false, bool ST = false>
__device__ __forceinline__ void oproj_merge_block(const DecodeArgs& a, const OprojArgs& o, int ob, char* smem) {
  fstamp<ST>(0);
  constexpr int KS = 32 * NLD;          // K-slice (NLD 32-k MFMA steps, one 16-B load each per lane)
  constexpr int ROWB = KS * 2;          // bytes per row of the LDS activation slice
  constexpr int HPB = KS / D;           // attention heads in the slice
  static_assert(KS % D == 0, "slice = whole heads");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int ncb = (o.N + 63) / 64;
  const int cb = ob % ncb, s = ob / ncb;
  const int n0 = cb * 64, kbase = s * KS, h0 = kbase / D;
  const int M = o.M;

  // 1) the weight slice, all loads in flight before anything else (wave w: columns n0 + 16w + fr)
  const int wrow = min(n0 + 16 * wid + fr, o.N - 1);
  const bf16_t* wp = o.W + (size_t)wrow * o.ldw + kbase + 8 * fh;
  bf16x8 wf[NLD];
#pragma unroll
  for (int ks = 0; ks < NLD; ++ks) wf[ks] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + 32 * ks));

  // 2) wait for every attention block (one lane polls a done-flag replica; the others wait at the barrier;
  //    a bounded wait: on timeout the error word is set and the block computes garbage, never hangs)
  fstamp<ST>(1);
  wait_flag(o.cnt + FL_A, o.cnt + 2, o.spin_limit);
  fstamp<ST>(2);
  if constexpr (MIA) {
    // the attention blocks merged the partitions: stage the bf16 rows of this K-slice (write-through loads)
    const __amdgpu_buffer_rsrc_t rs_x =
        __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, M * a.out_stride * 2, 0x00020000);
    constexpr int CPR = KS / 8;  // 16-B chunks per slice row
    u32x4 xv[(4 * CPR + 255) / 256];
#pragma unroll
    for (int i = 0; i < (4 * CPR + 255) / 256; ++i) {
      const int e = min(tid + 256 * i, M * CPR - 1);
      const int r = e / CPR, c = e % CPR;
      xv[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, (r * a.out_stride + kbase + 8 * c) * 2, 0, 16));
    }
#pragma unroll
    for (int i = 0; i < (4 * CPR + 255) / 256; ++i) {
      const int e = tid + 256 * i;
      if (e < M * CPR) {
        const int r = e / CPR, c = e % CPR;
        *reinterpret_cast<u32x4*>(smem + r * ROWB + 16 * ((c & ~15) | ((c & 15) ^ (r & 15)))) = xv[i];
      }
    }
  } else {

  // 3) merge the partitions of (row r, head h0 + j): pass 1 the statistics -> per-partition scales and
  //    the merged sum in LDS, pass 2 the partial outputs (all loads of a thread in flight: the scales are
  //    known, so there is no running rescale chain). Records are read write-through (sc1), as written.
  const unsigned pbytes = (unsigned)((size_t)M * a.Hq * a.max_parts * 4);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(a.part_o, (short)0, (int)(pbytes * D), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_ml = __builtin_amdgcn_make_buffer_rsrc(a.part_ml, (short)0, (int)(pbytes * 2), 0x00020000);
  float* s_sc = reinterpret_cast<float*>(smem + 16 * ROWB);  // [M][HPB][OP_MAXP] max, then scale
  float* s_l = s_sc + 4 * HPB * OP_MAXP;                      // [M][HPB][OP_MAXP] partition sums
  float* s_il = s_l + 4 * HPB * OP_MAXP;                      // [M][HPB] 1 / merged sum (0 if empty)
  int* s_np = reinterpret_cast<int*>(s_il + 4 * HPB);         // [M] partitions of row r
  if (tid < M) {
    const int n_kt = (a.kv_lens[tid] + KT - 1) / KT;
    const int pt = decode_part_tiles(n_kt, a);
    s_np[tid] = (n_kt + pt - 1) / pt;
  }
  __syncthreads();
  const int MP = a.max_parts;
  {
    // every (max, sum) load of the thread issued before any is used (indices clamped, masked after):
    // at most 4 x 4 heads x 64 partitions = 4 per thread
    constexpr int PER = (4 * HPB * OP_MAXP + 255) / 256;
    f32x2 ml[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = min(tid + 256 * k, M * HPB * MP - 1);
      const int p = e % MP, j = (e / MP) % HPB, r = e / (MP * HPB);
      const int pi = ((r * a.Hq + h0 + j) * MP + p) * 8;
      ml[k] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_ml, pi, 0, 16));
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k;
      if (e < M * HPB * MP) {
        const int p = e % MP, j = (e / MP) % HPB, r = e / (MP * HPB);
        const bool ok = p < s_np[r];
        s_sc[(r * HPB + j) * OP_MAXP + p] = ok ? ml[k][0] : -INFINITY;
        s_l[(r * HPB + j) * OP_MAXP + p] = ok ? ml[k][1] : 0.f;
      }
    }
  }
  __syncthreads();
  if (tid < M * HPB) {
    float* sc = s_sc + tid * OP_MAXP;
    const float* sl = s_l + tid * OP_MAXP;
    float mx = -INFINITY;
    for (int p = 0; p < MP; ++p) mx = fmaxf(mx, sc[p]);
    const float mu = mx == -INFINITY ? 0.f : mx;
    float L = 0.f;
    for (int p = 0; p < MP; ++p) {
      const float f = sc[p] == -INFINITY ? 0.f : exp2f(sc[p] - mu);
      sc[p] = f;
      L += sl[p] * f;
    }
    s_il[tid] = L > 0.f ? 1.f / L : 0.f;
  }
  __syncthreads();
  // pass 2: task = (row r, head j, 4 dims d4); npg adjacent lanes split a task's partitions
  const int ntask = M * HPB * (D / 4);
  int npg = 1;
  while (npg < 8 && ntask * npg * 2 <= 256) npg *= 2;
  for (int t0 = 0; t0 < ntask * npg; t0 += 256) {
    const int tt = t0 + tid;
    const bool act = tt < ntask * npg;
    const int task = (act ? tt : 0) / npg, pg = tt % npg;
    const int d4 = task % (D / 4), j = (task / (D / 4)) % HPB, r = task / ((D / 4) * HPB);
    const int np = s_np[r];
    const float* sc = s_sc + (r * HPB + j) * OP_MAXP;
    const int base = ((r * a.Hq + h0 + j) * MP) * D * 4 + d4 * 16;
    f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
    for (int p0 = pg; p0 < np; p0 += 8 * npg) {  // 8 records per thread in flight
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int p = min(p0 + i * npg, np - 1);
        v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_o, base + p * D * 4, 0, 16));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f = p0 + i * npg < np ? sc[p0 + i * npg] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc4[e] += __uint_as_float(v[i][e]) * f;
      }
    }
    for (int off = 1; off < npg; off <<= 1)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc4[e] += __shfl_xor(acc4[e], off, 64);
    if (act && pg == 0) {
      const float il = s_il[r * HPB + j];
      uint2 w;
      w.x = pk2bf(acc4[0] * il, acc4[1] * il);
      w.y = pk2bf(acc4[2] * il, acc4[3] * il);
      const int cc = j * (D / 8) + d4 / 2;  // 16-B chunk of the slice row; 8-B half d4 & 1
      const int c = (cc & ~15) | ((cc & 15) ^ (r & 15));
      *reinterpret_cast<uint2*>(smem + r * ROWB + 16 * c + 8 * (d4 & 1)) = w;
    }
  }
  }  // !MIA
  __syncthreads();

  fstamp<ST>(3);
  // 4) MFMA over the slice: A = activation rows (fr), B = this wave's weight columns
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NLD; ++ks) {
    const int chunk = 4 * ks + fh;
    const bf16x8 xf = *reinterpret_cast<const bf16x8*>(smem + fr * ROWB + 16 * ((chunk & ~15) | ((chunk & 15) ^ (fr & 15))));
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wf[ks], acc, 0, 0, 0);
  }
  const int col = n0 + 16 * wid + fr;
  const int nslab = o.K / KS;
  const __amdgpu_buffer_rsrc_t rs_p =
      __builtin_amdgcn_make_buffer_rsrc(o.P, (short)0, (int)((size_t)nslab * M * o.N * 4), 0x00020000);
  if (fh == 0 && col < o.N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r < M) {
        const int off = (int)((((size_t)s * M + r) * o.N + col) * 4);
        if (o.h)  // read back by the last block below: write-through
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r]), rs_p, off, 0, 16);
        else
          o.P[off / 4] = acc[r];
      }
    }
  }
  // 5) arrival ticket (after this block's slab stores have drained): the last o_proj block re-arms both
  //    counters -- every attention block is done and every o_proj block has read cnt[0] by then; the next
  //    launch is stream-ordered after this one -- and, with the norm tail, reduces the slabs.
  int* s_last = reinterpret_cast<int*>(smem);  // the activation slice is dead
  wait_vmcnt0();
  __syncthreads();
  fstamp<ST>(4);
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(o.cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == o.nob - 1;
    if (last) {  // (cnt[4] + the qkv flags: the 3-role launch's; every attention block is past its wait)
      __hip_atomic_store(o.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 4, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 5, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < FL_REPL; ++k) {
        __hip_atomic_store(o.cnt + FL_A + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o.cnt + FL_Q + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o.cnt + FL_P + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    *s_last = last;
  }
  __syncthreads();
  if (!o.h || !*s_last) {
    fstamp<ST>(5);
    return;
  }
  // 6) residual + RMSNorm of every row (add_partials_rmsnorm_kernel's math; slab order kept)
  float* red = reinterpret_cast<float*>(smem) + 16;
  const int nvec = o.N >> 3;
  for (int r = 0; r < M; ++r) {
    float v[2][8];  // this thread's two row vectors (H <= 4096; longer rows are re-read from h below)
    float ss = 0.f;
    for (int i0 = 0; i0 < nvec; i0 += 512) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vi = i0 + tid + 256 * i;
        if (vi >= nvec) continue;
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        u32x4 pv[16][2];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int su = min(u, nslab - 1);
          const int off = (int)((((size_t)su * M + r) * o.N + vi * 8) * 4);
          pv[u][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_p, off, 0, 16));
          pv[u][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_p, off + 16, 0, 16));
        }
        const u32x4 hv = *reinterpret_cast<const u32x4*>(o.h + (size_t)r * o.ldh + vi * 8);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (u < nslab) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              a[e] += __uint_as_float(pv[u][0][e]);
              a[4 + e] += __uint_as_float(pv[u][1][e]);
            }
          }
        }
        float hf[8];
        unpack8(hv, hf);
        float* vv = v[i];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = bf2f(f2bf(hf[e] + bf2f(f2bf(a[e]))));
        *reinterpret_cast<u32x4*>(o.h + (size_t)r * o.ldh + vi * 8) = pack8(vv);
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += vv[e] * vv[e];
      }
    }
    ss = block_sum(ss, red);
    const float inv = rsqrtf(ss / (float)o.N + o.eps);
    for (int i0 = 0; i0 < nvec; i0 += 512) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vi = i0 + tid + 256 * i;
        if (vi >= nvec) continue;
        float hv8[8], wv[8], out8[8];
        if (nvec <= 512) {
#pragma unroll
          for (int e = 0; e < 8; ++e) hv8[e] = v[i][e];
        } else {
          unpack8(*reinterpret_cast<const u32x4*>(o.h + (size_t)r * o.ldh + vi * 8), hv8);
        }
        unpack8(*reinterpret_cast<const u32x4*>(o.gamma + vi * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) out8[e] = wv[e] * bf2f(f2bf(hv8[e] * inv));
        *reinterpret_cast<u32x4*>(o.xn + (size_t)r * o.ldx + vi * 8) = pack8(out8);
      }
    }
    __syncthreads();  // red[] reuse by the next row
  }
  fstamp<ST>(6);
}

// qkv projection blocks of the 3-role launch (attn_oproj_kernel<..., QNLD > 0>): split-K partial slabs
// P[s][M][N] of rmsnorm(h) . Wqkv^T (gemm_part_norm's math and reduction order: threads sum their row
// vectors, the 4 wave partials are added in order), 64 output columns x KS per 4-wave block, written
// through (sc1) for the attention blocks of the same launch, then signalled on cnt[4].
struct QkvArgs {
  const bf16_t* W; int ldw;    // [N][K] bf16 (packed q | k | v rows)
  const bf16_t* h; int ldh;    // [M][K] residual rows (un-normalised)
  const bf16_t* gamma;         // [K]
  float eps;
  float* P;                    // [K / KS][M][N] fp32
  int M, N, K;
  int nqb;                     // qkv blocks
};

template <int NLD, bool ST = false>
__device__ __forceinline__ void qkv_norm_block(const QkvArgs& q, int qb, char* smem, int* cnt) {
  fstamp<ST>(0);
  constexpr int KS = 32 * NLD;
  constexpr int ROWB = KS * 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int ncb = (q.N + 63) / 64;
  const int cb = qb % ncb, s = qb / ncb;
  const int n0 = cb * 64, kbase = s * KS;
  const int M = q.M;
  const int nvec = q.K >> 3;  // 16-B vectors per row (K <= 4096: two per thread)
  // 1) row vectors + the slice's norm weights first (a counted wait retires them before the weights)
  u32x4 hv[4][2], gv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int vi = min(tid + 256 * i, nvec - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) hv[r][i] = *reinterpret_cast<const u32x4*>(q.h + (size_t)min(r, M - 1) * q.ldh + vi * 8);
    gv[i] = *reinterpret_cast<const u32x4*>((q.gamma ? q.gamma : q.h) + min(max(vi * 8, kbase), kbase + KS - 8));
  }
  __builtin_amdgcn_sched_barrier(0);
  const int wrow = min(n0 + 16 * wid + fr, q.N - 1);
  const bf16_t* wp = q.W + (size_t)wrow * q.ldw + kbase + 8 * fh;
  bf16x8 wf[NLD];
#pragma unroll
  for (int ks = 0; ks < NLD; ++ks) wf[ks] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + 32 * ks));
  __builtin_amdgcn_s_waitcnt((NLD & 15) | (((NLD >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));  // vmcnt(NLD)
  __builtin_amdgcn_sched_barrier(0);
  // 2) RMSNorm statistics (rmsnorm_kernel's order), normalised slice -> LDS (swizzled as the O role's);
  //    gamma == nullptr: the rows are already normalised (tensor-parallel decode), staged as they are
  float* s_red = reinterpret_cast<float*>(smem + 16 * ROWB);  // [4 rows][4 waves]
  if (q.gamma == nullptr) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= M) break;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vi = tid + 256 * i;
        if (vi < nvec && vi * 8 >= kbase && vi * 8 < kbase + KS) {
          const int c = vi - kbase / 8;
          *reinterpret_cast<u32x4*>(smem + r * ROWB + 16 * ((c & ~15) | ((c & 15) ^ (r & 15)))) = hv[r][i];
        }
      }
    }
  }
  float ss[4];
  const u32x4 z = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ss[r] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const u32x4 v = tid + 256 * i < nvec ? hv[r][i] : z;
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss[r] += f[e] * f[e];
    }
    ss[r] = wave_sum(ss[r]);
    if (lane == 0) s_red[r * 4 + wid] = ss[r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r >= M || q.gamma == nullptr) break;
    const float t = ((s_red[r * 4] + s_red[r * 4 + 1]) + s_red[r * 4 + 2]) + s_red[r * 4 + 3];
    const float inv = rsqrtf(t / (float)q.K + q.eps);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int vi = tid + 256 * i;
      if (vi < nvec && vi * 8 >= kbase && vi * 8 < kbase + KS) {
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
  __builtin_amdgcn_s_barrier();  // raw: __syncthreads() would drain the weight loads (vmcnt(0))
  __builtin_amdgcn_sched_barrier(0);
  // 3) MFMA, write-through slab, signal
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NLD; ++ks) {
    const int chunk = 4 * ks + fh;
    const bf16x8 xf = *reinterpret_cast<const bf16x8*>(smem + fr * ROWB + 16 * ((chunk & ~15) | ((chunk & 15) ^ (fr & 15))));
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wf[ks], acc, 0, 0, 0);
  }
  const int col = n0 + 16 * wid + fr;
  const int nslab = q.K / KS;
  const __amdgpu_buffer_rsrc_t rs_p =
      __builtin_amdgcn_make_buffer_rsrc(q.P, (short)0, (int)((size_t)nslab * M * q.N * 4), 0x00020000);
  if (fh == 0 && col < q.N) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < M)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r]), rs_p, (int)((((size_t)s * M + r) * q.N + col) * 4),
                                              0, 16);
  }
  fstamp<ST>(3);
  stage_arrive(cnt + 4, q.nqb, cnt + FL_Q);
  fstamp<ST>(5);
}

// o_proj block of the fused launch, v2 (MIA only): 16 output columns x the FULL K per block, the 4 waves
// splitting K in quarters (NLQ 16-B weight loads per lane each, all in flight from the block's start), so
// N / 16 blocks (256 at N = 4096) are resident next to the attention blocks from the first cycle and no
// split-K slab exists: the block reduces its waves in LDS and finishes its columns itself --
//   tail (o.h set): h[r][cols] = bf16(h + bf16(o_proj)) written through, per-row sum-of-squares partial
//     to o.ss[r][block]; the last block (arrival ticket) sums the partials in block order and writes
//     xn = rmsnorm(h) * gamma;
//   no tail (tensor parallel): the fp32 partial row o.P[0][r][cols] for the cross-rank reduction.
template <int D, int NLQ, bool ST = false>
__device__ __forceinline__ void oproj_full_block(const DecodeArgs& a, const OprojArgs& o, int ob, char* smem) {
  constexpr int KQ = 32 * NLQ;  // K quarter of one wave
  constexpr int K = 4 * KQ;
  constexpr int ROWB = K * 2;   // LDS bytes per activation row (4 rows: M <= 4)
  fstamp<ST>(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int n0 = ob * 16;
  const int M = o.M;
  const int col = n0 + fr;
  // 0) the residual values this block adds to (wave 0, rows 0..3 of column n0 + fr), requested first
  float hres[4] = {0.f, 0.f, 0.f, 0.f};
  if (o.h && wid == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) hres[r] = bf2f(o.h[(size_t)min(r, M - 1) * o.ldh + min(col, o.N - 1)]);
  }
  // 1) this wave's quarter of the block's 16 weight rows, every load in flight -- issued once every
  //    attention block has its KV requests out (the weight stream then queues behind them instead of
  //    delaying the attention's dependent loads)
  if (o.na > 0) wait_flag(o.cnt + FL_P, o.cnt + 2, o.spin_limit);
  const bf16_t* wp = o.W + (size_t)min(n0 + fr, o.N - 1) * o.ldw + wid * KQ + 8 * fh;
  bf16x8 wf[NLQ];
#pragma unroll
  for (int ks = 0; ks < NLQ; ++ks) wf[ks] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + 32 * ks));
  fstamp<ST>(1);
  // 2) the attention blocks have merged every head into a.out
  wait_flag(o.cnt + FL_A, o.cnt + 2, o.spin_limit);
  fstamp<ST>(2);
  // 3) the M attention rows -> LDS (write-through loads), 16-B chunk c of row r at slot c ^ (r & 15)
  {
    const __amdgpu_buffer_rsrc_t rs_x =
        __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, M * a.out_stride * 2, 0x00020000);
    constexpr int CPR = K / 8;
    constexpr int PER = (4 * CPR + 255) / 256;
    u32x4 xv[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = min(tid + 256 * i, M * CPR - 1);
      xv[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, ((e / CPR) * a.out_stride + 8 * (e % CPR)) * 2, 0, 16));
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + 256 * i;
      if (e < M * CPR) {
        const int r = e / CPR, c = e % CPR;
        *reinterpret_cast<u32x4*>(smem + r * ROWB + 16 * ((c & ~15) | ((c & 15) ^ (r & 15)))) = xv[i];
      }
    }
  }
  __syncthreads();
  fstamp<ST>(3);
  // 4) MFMA over the wave's K quarter (activation rows >= M alias row fr & 3: their outputs are dropped)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int xr = fr & 3;
#pragma unroll
  for (int ks = 0; ks < NLQ; ++ks) {
    const int chunk = (wid * KQ) / 8 + 4 * ks + fh;
    const bf16x8 xf = *reinterpret_cast<const bf16x8*>(smem + xr * ROWB + 16 * ((chunk & ~15) | ((chunk & 15) ^ xr)));
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wf[ks], acc, 0, 0, 0);
  }
  // 5) the 4 K quarters summed in wave order (LDS after the activation rows)
  f32x4* red = reinterpret_cast<f32x4*>(smem + 4 * ROWB);
  red[wid * 64 + lane] = acc;
  __syncthreads();
  int* s_last = reinterpret_cast<int*>(smem + 4 * ROWB + 4 * 64 * 16);
  float* s_red = reinterpret_cast<float*>(s_last + 4);
  const __amdgpu_buffer_rsrc_t rs_h =
      __builtin_amdgcn_make_buffer_rsrc(o.h ? o.h : a.out, (short)0, o.h ? M * o.ldh * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_ss = __builtin_amdgcn_make_buffer_rsrc(o.ss, (short)0, o.ss ? 4 * o.nob * 4 : 0, 0x00020000);
  if (wid == 0) {
    f32x4 c = red[lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) c += red[w * 64 + lane];
    // lane (fr, fh): column n0 + fr, rows 4 fh + r -- rows 0..3 live in the fh == 0 lanes
    if (!o.h) {
      if (fh == 0 && col < o.N) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (r < M) o.P[(size_t)r * o.N + col] = c[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = bf2f(f2bf(hres[r] + bf2f(f2bf(c[r]))));
        const float vn = __shfl_xor(v, 1, 64);
        float sq = fh == 0 && col < o.N ? v * v : 0.f;
        if (r < M && fh == 0 && (fr & 1) == 0 && col < o.N)
          __builtin_amdgcn_raw_buffer_store_b32(pk2bf(v, vn), rs_h, (r * o.ldh + col) * 2, 0, 16);
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) sq += __shfl_xor(sq, off, 64);
        if (r < M && lane == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sq), rs_ss, (r * o.nob + ob) * 4, 0, 16);
      }
    }
  }
  fstamp<ST>(4);
  // 6) arrival ticket; the last block re-arms the counters and finishes the norm
  wait_vmcnt0();
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(o.cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == o.nob - 1;
    if (last) {
      __hip_atomic_store(o.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 4, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.cnt + 5, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < FL_REPL; ++k) {
        __hip_atomic_store(o.cnt + FL_A + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o.cnt + FL_Q + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o.cnt + FL_P + k * FL_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    *s_last = last;
  }
  __syncthreads();
  if (!o.h || !*s_last) {
    fstamp<ST>(5);
    return;
  }
  // per row: sum of squares = the blocks' partials in block order (tree fixed by thread index), then
  // xn = gamma * bf16(h * rsqrt(mean + eps)); h is re-read write-through (other blocks wrote it). The
  // row's h vectors and gamma are requested together with the partials (one round trip per row, H <= 4096).
  const int nvec = o.N >> 3;
  for (int r = 0; r < M; ++r) {
    u32x4 hv[2], gv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int vi = min(tid + 256 * i, nvec - 1);
      hv[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_h, (r * o.ldh + vi * 8) * 2, 0, 16));
      gv[i] = *reinterpret_cast<const u32x4*>(o.gamma + vi * 8);
    }
    float ss = 0.f;
    for (int b2 = tid; b2 < o.nob; b2 += 256)
      ss += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_ss, (r * o.nob + b2) * 4, 0, 16));
    ss = block_sum(ss, s_red);
    const float inv = rsqrtf(ss / (float)o.N + o.eps);
    for (int vi = tid; vi < nvec; vi += 256) {
      const int i = (vi - tid) / 256;
      u32x4 hvv, gvv;
      if (i < 2) {
        hvv = i == 0 ? hv[0] : hv[1];
        gvv = i == 0 ? gv[0] : gv[1];
      } else {
        hvv = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_h, (r * o.ldh + vi * 8) * 2, 0, 16));
        gvv = *reinterpret_cast<const u32x4*>(o.gamma + vi * 8);
      }
      float hf[8], wv[8], out8[8];
      unpack8(hvv, hf);
      unpack8(gvv, wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) out8[e] = wv[e] * bf2f(f2bf(hf[e] * inv));
      *reinterpret_cast<u32x4*>(o.xn + (size_t)r * o.ldx + vi * 8) = pack8(out8);
    }
    __syncthreads();  // s_red reuse by the next row
  }
  fstamp<ST>(6);
}

template <int D, int G, int NLD>
constexpr int attn_oproj_lds() {
  constexpr int a = decode_lds_bytes<D, G>();
  constexpr int o = 16 * 64 * NLD + (2 * 4 * (32 * NLD / D) * OP_MAXP + 4 * (32 * NLD / D) + 4) * 4;
  return a > o ? a : o;
}

// QNLD > 0: the 3-role launch -- blocks [0, nqb) are qkv blocks (qkv_norm_block<QNLD>), then the
// attention blocks (they prefetch their first KV tile, then wait for every qkv block), then the o_proj
// blocks. Every wait is on lower-indexed blocks only.
template <int D, int G, int NLD, int QNLD = 0, bool MIA = false, bool ST = false, bool OV2 = false>
__global__ __launch_bounds__(256, 2) void attn_oproj_kernel(DecodeArgs a, OprojArgs o, QkvArgs q) {
  constexpr int lds_q = QNLD > 0 ? 16 * 64 * QNLD + 64 : 0;
  constexpr int lds_o = OV2 ? 4 * 4 * 32 * NLD * 2 + 4 * 64 * 16 + 64 : attn_oproj_lds<D, G, NLD>();
  constexpr int lds_a = decode_lds_bytes<D, G>();
  constexpr int lds_ao = lds_o > lds_a ? lds_o : lds_a;
  constexpr int lds = lds_ao > lds_q ? lds_ao : lds_q;
  __shared__ __attribute__((aligned(16))) char smem[lds];
  int bid = blockIdx.x;
  if constexpr (QNLD > 0) {
    if (bid < q.nqb) {
      qkv_norm_block<QNLD, ST>(q, bid, smem, o.cnt);
      return;
    }
    bid -= q.nqb;
  }
  if (bid < o.na) {
    const int mp = a.max_parts;
    attn_decode_block<D, G, false, true, (QNLD > 0), MIA, ST>(a, bid % mp, (bid / mp) % a.Hkv, bid / (mp * a.Hkv),
                                                              smem, o.cnt, QWait{o.cnt + FL_Q, o.cnt + 2, o.spin_limit},
                                                              o.na);
    return;
  }
  if constexpr (OV2)
    oproj_full_block<D, NLD, ST>(a, o, bid - o.na, smem);
  else
    oproj_merge_block<D, NLD, MIA, ST>(a, o, bid - o.na, smem);
}

// merge split-K partitions: grid (Hq, B), block D threads. The partition statistics are loaded by
// all threads at once (thread t: partitions t, t + D, ...) and reduced in LDS, and each output
// element's partial sums are loaded 8 partitions per batch of independent loads: the previous
// version walked the partitions in two dependent load chains per thread (~9 us at batch 1 with 32
// partitions, pure load latency; the decode attention itself took 9.4 us).
constexpr int RED_MAXP = 256;  // partitions held in LDS (launcher guarantees max_parts <= this)
__global__ void attn_decode_reduce_kernel(DecodeArgs a, int D) {
  __shared__ float s_sc[RED_MAXP];
  __shared__ float s_red[8];
  __shared__ float s_M, s_L;
  const int hq = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int nw = (blockDim.x + 63) >> 6, lane = t & 63, wid = t >> 6;
  const int n_kt = (a.kv_lens[b] + KT - 1) / KT;
  const int pt = decode_part_tiles(n_kt, a);
  const int nparts = (n_kt + pt - 1) / pt;
  if (nparts <= 1) return;  // block-uniform: the partition kernel wrote the output itself
  const size_t p0 = ((size_t)b * a.Hq + hq) * a.max_parts;
  float m = -INFINITY;
  for (int p = t; p < nparts; p += blockDim.x) {
    const float mp = a.part_ml[(p0 + p) * 2];
    s_sc[p] = mp;
    m = fmaxf(m, mp);
  }
  m = wave_max(m);
  if (lane == 0) s_red[wid] = m;
  __syncthreads();
  if (t == 0) {
    float M = -INFINITY;
    for (int w = 0; w < nw; ++w) M = fmaxf(M, s_red[w]);
    s_M = M == -INFINITY ? 0.f : M;
  }
  __syncthreads();
  const float Mu = s_M;
  float l = 0.f;
  for (int p = t; p < nparts; p += blockDim.x) {
    const float sc = exp2f(s_sc[p] - Mu);
    s_sc[p] = sc;
    l += a.part_ml[(p0 + p) * 2 + 1] * sc;
  }
  l = wave_sum(l);
  __syncthreads();
  if (lane == 0) s_red[wid] = l;
  __syncthreads();
  if (t == 0) {
    float L = 0.f;
    for (int w = 0; w < nw; ++w) L += s_red[w];
    s_L = L;
  }
  __syncthreads();
  if (t >= D) return;
  const float* po = a.part_o + p0 * D + t;
  float O = 0.f;
  int p = 0;
  for (; p + 8 <= nparts; p += 8) {  // 8 independent loads in flight per thread
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = po[(size_t)(p + i) * D];
#pragma unroll
    for (int i = 0; i < 8; ++i) O += v[i] * s_sc[p + i];
  }
  for (; p < nparts; ++p) O += po[(size_t)p * D] * s_sc[p];
  const float L = s_L;
  a.out[(size_t)b * a.out_stride + hq * D + t] = f2bf(L > 0.f ? O / L : 0.f);
}

// Waves per block when 4 query heads share a KV head (Llama GQA): 8 = two 32-row groups share each
// K/V tile (half the DMA issue and K/V traffic per wave).
int g_prefill_waves = 4;
int g_prefill_prio = 1;  // PRIO variant of the Llama config (D 128, 4 heads per block, causal, paged)
int g_prefill_buf = 1;   // BUF staging for that config when the cache is < 4 GiB
// Ping-pong 8-wave kernel for the Llama config (0 off, 1 on, 2 on + static priority for waves 4-7);
// when on, every 4-heads-per-block config uses 64-query tiles (the 8-wave kernel where the cache
// is too large for buffer staging).
int g_prefill_pp = 0;

// Block order (prefill_block): 1 = 1-D grid, head group fastest (default); 0 = 2-D (tile, head group).
int g_prefill_order = 1;

template <int D, int GB, bool CAUSAL, bool PAGED>
hipError_t launch_prefill(PrefillArgs a, int n_tiles, hipStream_t st) {
  const int G = a.Hq / a.Hkv;
  const int n_hg = a.Hkv * (G / GB);
  a.n_hg = g_prefill_order ? n_hg : 0;
  const dim3 grid = a.n_hg ? dim3(n_tiles * n_hg) : dim3(n_tiles, n_hg);
  if constexpr (D == 128 && GB == 4 && CAUSAL && PAGED) {
    if (g_prefill_pp && a.kv_bytes) {
      switch (g_prefill_pp) {
        case 1: hipLaunchKernelGGL((attn_prefill_pp_kernel<0, 2>), grid, dim3(512), 0, st, a); break;
        case 2: hipLaunchKernelGGL((attn_prefill_pp_kernel<1, 2>), grid, dim3(512), 0, st, a); break;
        case 3: hipLaunchKernelGGL((attn_prefill_pp_kernel<1, 4>), grid, dim3(512), 0, st, a); break;
        case 4: hipLaunchKernelGGL((attn_prefill_pp_kernel<1, 8>), grid, dim3(512), 0, st, a); break;
        case 5: hipLaunchKernelGGL((attn_prefill_pp_kernel<1, 8, true>), grid, dim3(512), 0, st, a); break;
        case 6: hipLaunchKernelGGL((attn_prefill_v3_kernel<4>), grid, dim3(256), 0, st, a); break;
        case 7: hipLaunchKernelGGL((attn_prefill_v3_kernel<4, true>), grid, dim3(256), 0, st, a); break;
        case 8: hipLaunchKernelGGL((attn_prefill_v3_kernel<4, true, 1>), grid, dim3(256), 0, st, a); break;
        case 9: hipLaunchKernelGGL((attn_prefill_v3_kernel<4, true, 2>), grid, dim3(256), 0, st, a); break;
        case 10: hipLaunchKernelGGL((attn_prefill_v3_kernel<8>), grid, dim3(512), 0, st, a); break;
        case 11: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, true>), grid, dim3(512), 0, st, a); break;
        case 12: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, true, 1>), grid, dim3(512), 0, st, a); break;
        case 14: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, false, 0, 1>), grid, dim3(512), 0, st, a); break;
        case 15: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, false, 0, 0, true>), grid, dim3(512), 0, st, a); break;
        case 16: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, false, 0, 1, true>), grid, dim3(512), 0, st, a); break;
        case 13: hipLaunchKernelGGL((attn_prefill_v3_kernel<8, true, 2>), grid, dim3(512), 0, st, a); break;
        default: hipLaunchKernelGGL((attn_prefill_v3_kernel<8>), grid, dim3(512), 0, st, a); break;
      }
      return hipGetLastError();
    }
    if (!g_prefill_pp && g_prefill_waves == 4 && g_prefill_prio == 1 && g_prefill_buf && a.kv_bytes) {
      hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED, false, 4, 1, true>), grid, dim3(256), 0, st, a);
      return hipGetLastError();
    }
  }
  if (GB == 4 && (g_prefill_waves == 8 || (g_prefill_pp >= 1 && g_prefill_pp <= 5) || g_prefill_pp >= 10))
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED, false, 8>), grid, dim3(512), 0, st, a);
  else if (D == 128 && GB == 4 && CAUSAL && PAGED && g_prefill_prio == 1)
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED, false, 4, 1>), grid, dim3(256), 0, st, a);
  else if (D == 128 && GB == 4 && CAUSAL && PAGED && g_prefill_prio == 2)
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED, false, 4, 2>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace

// Stamp build of the Llama prefill config (D 128, 4 heads per block, causal, paged): per wave
// [DMA issue, QK^T, softmax, PV, wait+barrier, tiles] s_memtime sums into dbg[grid][4 waves][6].
RAGK_API int ragk_attn_prefill_stamp(const void* q, int q_stride, const void* k, const void* v,
                                     const int* block_tables, int bt_stride, const int* cu_q, const int* kv_lens,
                                     const int* tiles, int n_tiles, void* out, int out_stride, int Hq, int Hkv,
                                     float scale, unsigned long long* dbg, hipStream_t st) {
  if (n_tiles <= 0 || Hq % Hkv || (Hq / Hkv) % 4) return (int)hipErrorInvalidValue;
  hipMemcpyToSymbolAsync(HIP_SYMBOL(g_attn_dbg), &dbg, sizeof(dbg), 0, hipMemcpyHostToDevice, st);
  PrefillArgs a{(const bf16_t*)q, q_stride, (const bf16_t*)k, (const bf16_t*)v, 0, block_tables, bt_stride,
                cu_q, nullptr, kv_lens, tiles, (bf16_t*)out, out_stride, Hq, Hkv, scale * 1.4426950408889634f};
  const int G = Hq / Hkv;
  dim3 grid(n_tiles, Hkv * (G / 4));
  hipLaunchKernelGGL((attn_prefill_kernel<128, 4, true, true, true>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

RAGK_API int ragk_attn_set_dbg(unsigned long long* dbg) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_dbg), &dbg, sizeof(dbg), 0, hipMemcpyHostToDevice);
}

RAGK_API int ragk_attn_prefill_set_prio(int v) {
  if (v < 0 || v > 2) return (int)hipErrorInvalidValue;
  g_prefill_prio = v;
  return 0;
}

RAGK_API int ragk_attn_prefill_set_buf(int v) {
  g_prefill_buf = v ? 1 : 0;
  return 0;
}

// Returns the query positions per block (the host builds `tiles` with this step).
RAGK_API int ragk_attn_prefill_set_waves(int w) {
  if (w != 4 && w != 8) return (int)hipErrorInvalidValue;
  g_prefill_waves = w;
  return 0;
}

// (every GB == 4 config follows g_prefill_waves; the host builds tiles with this value)
RAGK_API int ragk_attn_prefill_qtile(int Hq, int Hkv) {
  const int G = Hq / Hkv;
  const int GB = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
  const bool pp64 = (g_prefill_pp >= 1 && g_prefill_pp <= 5) || g_prefill_pp >= 10;
  return 32 * ((GB == 4 ? (pp64 ? 8 : g_prefill_waves) : 4) / GB);
}

// 0 off; 1..4 variants (1: fragment prefetch 2 steps; 2: + priority for waves 4-7; 3 / 4: + prefetch
// 4 / 8 steps); 5: the stamp build of variant 4 (g_attn_dbg set by ragk_attn_set_dbg); 6: the
// software-pipelined one-wave-per-SIMD kernel (attn_prefill_v3_kernel, 32-query tiles); 7: its stamps
RAGK_API int ragk_attn_prefill_set_pp(int v) {
  if (v < 0 || v > 16) return (int)hipErrorInvalidValue;
  g_prefill_pp = v;
  return 0;
}

RAGK_API int ragk_attn_prefill(const void* q, int q_stride, const void* k, const void* v, int kv_stride,
                               const int* block_tables, int bt_stride, const int* cu_q, const int* cu_kv,
                               const int* kv_lens, const int* tiles, int n_tiles, void* out, int out_stride,
                               int Hq, int Hkv, int D, int causal, int paged, float scale, hipStream_t st) {
  if (n_tiles <= 0) return 0;
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  // paged: kv_stride = number of cache blocks (sizes the buffer descriptors of the BUF staging)
  const unsigned long long cache_bytes = paged ? (unsigned long long)kv_stride * Hkv * KT * D * 2 : 0ull;
  PrefillArgs a{(const bf16_t*)q, q_stride, (const bf16_t*)k, (const bf16_t*)v, kv_stride, block_tables, bt_stride,
                cu_q, cu_kv, kv_lens, tiles, (bf16_t*)out, out_stride, Hq, Hkv, scale * 1.4426950408889634f,
                cache_bytes < (1ull << 32) ? (unsigned)cache_bytes : 0u, 0};
  const int G = Hq / Hkv;
  const int GB = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
#define RAGK_PF(DD, GG, CC, PP)                                                          \
  if (D == DD && GB == GG && (bool)causal == CC && (bool)paged == PP)                      \
    return (int)launch_prefill<DD, GG, CC, PP>(a, n_tiles, st);
  RAGK_PF(128, 4, true, true)
  RAGK_PF(128, 1, true, true)
  RAGK_PF(128, 2, true, true)
  RAGK_PF(64, 1, true, true)
  RAGK_PF(64, 4, true, true)
  RAGK_PF(128, 4, true, false)
  RAGK_PF(64, 1, false, false)
  RAGK_PF(32, 1, false, false)
  RAGK_PF(128, 1, false, false)
  RAGK_PF(64, 1, true, false)
#undef RAGK_PF
  return (int)hipErrorInvalidValue;
}

RAGK_API int ragk_attn_prefill_set_order(int order) {
  g_prefill_order = order ? 1 : 0;
  return 0;
}

// K/V cache-policy switch for decode (0 = default, 1 = non-temporal loads; the KV stream is read
// once per step). A/B in tools/bench_kernels.py --quick.
static int g_decode_nt = 0;
// 8-wave single-partition decode attention once batch x KV heads reaches this (0 = never)
static int g_decode_nw8_min = 0;
RAGK_API int ragk_attn_decode_set_nw8(int min_pairs) {
  g_decode_nw8_min = min_pairs > 0 ? min_pairs : 0;
  return 0;
}
RAGK_API int ragk_attn_decode_set_nt(int nt) {
  g_decode_nt = nt ? 1 : 0;
  return 0;
}

static int launch_attn_decode(DecodeArgs a, int B, int D, int max_parts, int* counters, hipStream_t st);

// Deferred merge: the next decode-attention launches leave the split-K partitions unmerged (no
// attn_decode_reduce launch) for a consumer that merges them itself (gemm_part.hip MergeArgs: the
// o_proj GEMM). The host sets it around one launch.
static int g_decode_defer = 0;
RAGK_API int ragk_attn_decode_set_defer(int on) {
  g_decode_defer = on ? 1 : 0;
  return 0;
}

RAGK_API int ragk_attn_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                              int bt_stride, const int* kv_lens, float* part_o, float* part_ml, void* out,
                              int out_stride, int B, int Hq, int Hkv, int D, int part_tiles, int max_parts,
                              float scale, int* counters, hipStream_t st) {
  if (B <= 0) return 0;
  if (Hq % Hkv || part_tiles < 1 || max_parts < 1 || max_parts > RED_MAXP) return (int)hipErrorInvalidValue;
  // fused merge: LDS holds 2 x G x max_parts + G floats of partition statistics (< the 64 KiB V tiles)
  if (counters && 2 * (Hq / Hkv) * max_parts + 16 > 4 * KT * D * 2 / 4) return (int)hipErrorInvalidValue;
  DecodeArgs a{(const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, (bf16_t*)out, out_stride, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f, counters};
  return launch_attn_decode(a, B, D, max_parts, counters, st);
}

// Decode attention fed by the qkv projection's split-K partial slabs P[S][B][ldp] (gemm_part.hip):
// RoPE of q and k, the KV append at slots[b] and the attention in one launch (replaces
// rope_kv_partials + attn_decode). Cache blocks hold KT tokens.
RAGK_API int ragk_attn_decode_rope(const float* P, int S, int ldp, const int* positions, const int* slots,
                                   const float* cos_t, const float* sin_t, void* kc, void* vc,
                                   const int* block_tables, int bt_stride, const int* kv_lens, float* part_o,
                                   float* part_ml, void* out, int out_stride, int B, int Hq, int Hkv, int D,
                                   int part_tiles, int max_parts, float scale, int* counters, hipStream_t st) {
  if (B <= 0) return 0;
  if (Hq % Hkv || part_tiles < 1 || max_parts < 1 || max_parts > RED_MAXP || S < 1 || D % 64 ||
      ldp < (Hq + 2 * Hkv) * D || !P || !positions || !slots || !cos_t || !sin_t)
    return (int)hipErrorInvalidValue;
  if (counters && 2 * (Hq / Hkv) * max_parts + 16 > 4 * KT * D * 2 / 4) return (int)hipErrorInvalidValue;
  DecodeArgs a{nullptr, 0, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, (bf16_t*)out, out_stride, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f, counters, P, (long long)B * ldp, ldp, S, positions, slots, cos_t, sin_t};
  return launch_attn_decode(a, B, D, max_parts, counters, st);
}

static int launch_attn_decode(DecodeArgs a, int B, int D, int max_parts, int* counters, hipStream_t st) {
  const int Hq = a.Hq, Hkv = a.Hkv;
  const int G = Hq / Hkv;
  const PfArgs pf = pf_take();
  const int ex = (pf.blocks + Hkv * B - 1) / (Hkv * B);  // rider columns (x beyond max_parts)
  dim3 grid(max_parts + ex, Hkv, B);
  if (D == 128 && G == 4 && max_parts == 1 && !counters && g_decode_nw8_min > 0 && B * Hkv >= g_decode_nw8_min) {
    // one partition per sequence over >= 1 block per CU: 8-wave blocks, no merge launch
    if (g_decode_nt)
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, true, 8>), grid, dim3(512), 0, st, a, pf);
    else
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, false, 8>), grid, dim3(512), 0, st, a, pf);
    return (int)hipGetLastError();
  }
#define RAGK_DC(DD, GG)                                                            \
  if (D == DD && G == GG) {                                                          \
    if (g_decode_nt)                                                                 \
      hipLaunchKernelGGL((attn_decode_kernel<DD, GG, true>), grid, dim3(256), 0, st, a, pf); \
    else                                                                             \
      hipLaunchKernelGGL((attn_decode_kernel<DD, GG, false>), grid, dim3(256), 0, st, a, pf); \
    if (max_parts > 1 && !counters && !g_decode_defer)                               \
      hipLaunchKernelGGL(attn_decode_reduce_kernel, dim3(Hq, B), dim3(DD), 0, st, a, DD); \
    return (int)hipGetLastError();                                                   \
  }
  RAGK_DC(128, 4)
  RAGK_DC(128, 8)
  RAGK_DC(128, 1)
  RAGK_DC(64, 1)
  RAGK_DC(64, 4)
  RAGK_DC(128, 2)
#undef RAGK_DC
  return (int)hipErrorInvalidValue;
}

// Diagnostic: the next fused launches (G = 4, ks_steps 8, MIA, q_ks 16 or none) run the stamp build,
// writing 8 s_memrealtime stamps per block into `stamps` (u64 [grid][8]); nullptr = production build.
static unsigned long long* g_fused_stamps_host = nullptr;
// v2 o_proj role (oproj_full_block): 16-column full-K blocks, no split-K slabs (MIA launches only)
static int g_ao_v2 = 1;
RAGK_API int ragk_attn_oproj_set_v2(int on) {
  g_ao_v2 = on ? 1 : 0;
  return 0;
}

// Fused decode attention (RoPE + KV append from the qkv split-K slabs, as ragk_attn_decode_rope) and
// o_proj split-K partials (as ragk_gemm_part_merge) in ONE launch: attn_oproj_kernel. B <= 4, D = 128,
// G in {4, 8}; Wo bf16 [N][Hq * D] (ldw elements); Pout fp32 [K / KS][B][N], KS = 64 * ks_steps
// (ks_steps 4, 8 or 16). cnt: ragk_attn_oproj_cnt_ints() zeroed ints owned by the caller (re-armed by
// the kernel itself).
// h != nullptr: the residual + RMSNorm tail (h += bf16(sum of slabs), xn = rmsnorm(h) * gamma; the
// add_partials_rmsnorm consumer) runs in the last o_proj block.
// part_o / part_ml: the partition workspace (required, also for one partition).
RAGK_API int ragk_attn_oproj_fused(const float* P, int S, int ldp, const int* positions, const int* slots,
                                   const float* cos_t, const float* sin_t, void* kc, void* vc,
                                   const int* block_tables, int bt_stride, const int* kv_lens, float* part_o,
                                   float* part_ml, int B, int Hq, int Hkv, int D, int part_tiles, int max_parts,
                                   float scale, const void* Wo, int ldw, float* Pout, int N, int ks_steps, int* cnt,
                                   unsigned spin_us, void* h, int ldh, const void* gamma, void* xn, int ldx,
                                   float eps, void* attn_out, hipStream_t st) {
  if (B <= 0) return 0;
  const int G = Hq / (Hkv > 0 ? Hkv : 1);
  const int K = Hq * D;
  const int KS = 64 * ks_steps;
  if (B > 4 || D != 128 || Hq % Hkv || (G != 4 && G != 8) || (ks_steps != 4 && ks_steps != 8 && ks_steps != 16) || K % KS ||
      part_tiles < 1 || max_parts < 1 || max_parts > OP_MAXP || S < 1 || ldp < (Hq + 2 * Hkv) * D || !P ||
      !positions || !slots || !cos_t || !sin_t || !part_o || !part_ml || !Wo || !Pout || !cnt || N <= 0 ||
      ldw < K)
    return (int)hipErrorInvalidValue;
  // norm tail: the last o_proj block sums <= 16 slabs per row vector (h, gamma, xn: bf16, 16-B rows)
  if (h && (!gamma || !xn || K / KS > 16 || N % 8 || ldh % 8 || ldx % 8 || ((uintptr_t)h & 15) ||
            ((uintptr_t)xn & 15) || ((uintptr_t)gamma & 15)))
    return (int)hipErrorInvalidValue;
  DecodeArgs a{nullptr, 0, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, nullptr, 0, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f, nullptr, P, (long long)B * ldp, ldp, S, positions, slots, cos_t, sin_t, B};
  const unsigned long long ticks = (unsigned long long)(spin_us ? spin_us : 1000000u) * 100ull;
  OprojArgs o{(const bf16_t*)Wo, ldw, Pout, B, N, K, max_parts * Hkv * B, ((N + 63) / 64) * (K / KS), cnt,
              (unsigned)(ticks > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : ticks), (bf16_t*)h, ldh, (const bf16_t*)gamma,
              (bf16_t*)xn, ldx, eps};
  const dim3 grid(o.na + o.nob);
  const QkvArgs q{};
  const bool mia = attn_out != nullptr;  // partitions merged by the attention blocks into attn_out
  if (mia) {
    a.out = (bf16_t*)attn_out;
    a.out_stride = K;
    a.counters = cnt + CNT_TICKETS;
    if (B * Hkv > 4 * 64) return (int)hipErrorInvalidValue;
  }
  const int nlq = K / 128;  // v2: 16-B loads per lane of one wave's K quarter
  if (mia && g_ao_v2 && (nlq == 4 || nlq == 8 || nlq == 16 || nlq == 32) && (N + 15) / 16 <= 512) {
    o.nob = (N + 15) / 16;
    o.ss = reinterpret_cast<float*>(cnt + CNT_SS);
    const dim3 grid2(o.na + o.nob);
    if (g_fused_stamps_host && G == 4 && nlq == 32) {
      hipLaunchKernelGGL((attn_oproj_kernel<128, 4, 32, 0, true, true, true>), grid2, dim3(256), 0, st, a, o, q);
      return (int)hipGetLastError();
    }
#define RAGK_AO2(GG, NQ)                                                                                 \
    if (G == GG && nlq == NQ) {                                                                          \
      hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NQ, 0, true, false, true>), grid2, dim3(256), 0, st, a, o, q); \
      return (int)hipGetLastError();                                                                     \
    }
    RAGK_AO2(4, 4) RAGK_AO2(4, 8) RAGK_AO2(4, 16) RAGK_AO2(4, 32)
    RAGK_AO2(8, 4) RAGK_AO2(8, 8) RAGK_AO2(8, 16) RAGK_AO2(8, 32)
#undef RAGK_AO2
  }
  if (g_fused_stamps_host && mia && G == 4 && ks_steps == 8) {
    hipLaunchKernelGGL((attn_oproj_kernel<128, 4, 16, 0, true, true>), grid, dim3(256), 0, st, a, o, q);
    return (int)hipGetLastError();
  }
#define RAGK_AO(GG, NL)                                                                                \
  if (G == GG && 2 * ks_steps == NL) {                                                                 \
    if (mia) hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NL, 0, true>), grid, dim3(256), 0, st, a, o, q); \
    else hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NL>), grid, dim3(256), 0, st, a, o, q);         \
    return (int)hipGetLastError();                                                                     \
  }
  RAGK_AO(4, 8)
  RAGK_AO(4, 16)
  RAGK_AO(4, 32)
  RAGK_AO(8, 8)
  RAGK_AO(8, 16)
  RAGK_AO(8, 32)
#undef RAGK_AO
  return (int)hipErrorInvalidValue;
}

// The 3-role launch: the qkv projection with the input RMSNorm (gemm_part_norm's math) as well --
// qkv + attention + o_proj (+ the residual / post-attention norm tail) in ONE launch per layer.
// h [B][ldh] bf16 is the layer input (un-normalised residual), gin its norm weight, Wqkv [Nq][K] bf16
// (K = 4096), Pq the qkv slab workspace [K / (64 q_ks)][B][Nq] fp32 (q_ks 8 or 16). gin == nullptr: h is
// already normalised (tensor-parallel decode: the output of the fused cross-rank reduction). The
// post-attention tail (h2 != nullptr) updates h2 (the same residual buffer) in place and writes xn;
// without it the o_proj slabs Pout go to the caller's consumer (the cross-rank reduction under TP).
RAGK_API int ragk_qkv_attn_oproj_fused(const void* h, int ldh, const void* gin, float eps_in, const void* Wqkv,
                                       int ldwq, int Nq, int K, float* Pq, int q_ks, const int* positions,
                                       const int* slots, const float* cos_t, const float* sin_t, void* kc, void* vc,
                                       const int* block_tables, int bt_stride, const int* kv_lens, float* part_o,
                                       float* part_ml, int B, int Hq, int Hkv, int D, int part_tiles, int max_parts,
                                       float scale, const void* Wo, int ldw, float* Pout, int N, int ks_steps,
                                       int* cnt, unsigned spin_us, void* h2, int ldh2, const void* gamma, void* xn,
                                       int ldx, float eps, void* attn_out, hipStream_t st) {
  if (B <= 0) return 0;
  const int G = Hq / (Hkv > 0 ? Hkv : 1);
  const int Ko = Hq * D;
  const int KS = 64 * ks_steps, QKS = 64 * q_ks;
  if (B > 4 || D != 128 || Hq % Hkv || (G != 4 && G != 8) || (ks_steps != 4 && ks_steps != 8 && ks_steps != 16) ||
      Ko % KS || (q_ks != 8 && q_ks != 16) || K > 4096 || K % QKS || Nq != (Hq + 2 * Hkv) * D || ldwq < K ||
      ldh % 8 || ((uintptr_t)h & 15) || ((uintptr_t)gin & 15) || part_tiles < 1 || max_parts < 1 ||
      max_parts > OP_MAXP || !h || !Wqkv || !Pq || !positions || !slots || !cos_t || !sin_t || !part_o ||
      !part_ml || !Wo || !Pout || !cnt || N <= 0 || ldw < Ko)
    return (int)hipErrorInvalidValue;
  if (h2 && (!gamma || !xn || Ko / KS > 16 || N % 8 || ldh2 % 8 || ldx % 8 || ((uintptr_t)h2 & 15) ||
             ((uintptr_t)xn & 15) || ((uintptr_t)gamma & 15)))
    return (int)hipErrorInvalidValue;
  const int S = K / QKS;
  DecodeArgs a{nullptr, 0, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, nullptr, 0, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f, nullptr, Pq, (long long)B * Nq, Nq, S, positions, slots, cos_t, sin_t, B};
  const unsigned long long ticks = (unsigned long long)(spin_us ? spin_us : 1000000u) * 100ull;
  OprojArgs o{(const bf16_t*)Wo, ldw, Pout, B, N, Ko, max_parts * Hkv * B, ((N + 63) / 64) * (Ko / KS), cnt,
              (unsigned)(ticks > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : ticks), (bf16_t*)h2, ldh2, (const bf16_t*)gamma,
              (bf16_t*)xn, ldx, eps};
  const QkvArgs q{(const bf16_t*)Wqkv, ldwq, (const bf16_t*)h, ldh, (const bf16_t*)gin, eps_in, Pq, B, Nq, K,
                  ((Nq + 63) / 64) * S};
  const dim3 grid(q.nqb + o.na + o.nob);
  const bool mia = attn_out != nullptr;
  if (mia) {
    a.out = (bf16_t*)attn_out;
    a.out_stride = Ko;
    a.counters = cnt + CNT_TICKETS;
    if (B * Hkv > 4 * 64) return (int)hipErrorInvalidValue;
  }
  const int nlq = Ko / 128;
  if (mia && g_ao_v2 && (nlq == 4 || nlq == 8 || nlq == 16 || nlq == 32) && (N + 15) / 16 <= 512) {
    o.nob = (N + 15) / 16;
    o.ss = reinterpret_cast<float*>(cnt + CNT_SS);
    const dim3 grid2(q.nqb + o.na + o.nob);
    if (g_fused_stamps_host && G == 4 && nlq == 32 && q_ks == 16) {
      hipLaunchKernelGGL((attn_oproj_kernel<128, 4, 32, 32, true, true, true>), grid2, dim3(256), 0, st, a, o, q);
      return (int)hipGetLastError();
    }
#define RAGK_QAO2(GG, NQ, QN)                                                                                \
    if (G == GG && nlq == NQ && 2 * q_ks == QN) {                                                          \
      hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NQ, QN, true, false, true>), grid2, dim3(256), 0, st, a, o, q); \
      return (int)hipGetLastError();                                                                       \
    }
    RAGK_QAO2(4, 32, 16) RAGK_QAO2(4, 32, 32) RAGK_QAO2(4, 4, 32) RAGK_QAO2(8, 32, 32) RAGK_QAO2(8, 8, 32)
#undef RAGK_QAO2
  }
  if (g_fused_stamps_host && mia && G == 4 && ks_steps == 8 && q_ks == 16) {
    hipLaunchKernelGGL((attn_oproj_kernel<128, 4, 16, 32, true, true>), grid, dim3(256), 0, st, a, o, q);
    return (int)hipGetLastError();
  }
#define RAGK_QAO(GG, NL, QN)                                                                                 \
  if (G == GG && 2 * ks_steps == NL && 2 * q_ks == QN) {                                                     \
    if (mia) hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NL, QN, true>), grid, dim3(256), 0, st, a, o, q); \
    else hipLaunchKernelGGL((attn_oproj_kernel<128, GG, NL, QN>), grid, dim3(256), 0, st, a, o, q);          \
    return (int)hipGetLastError();                                                                           \
  }
  RAGK_QAO(4, 16, 16)
  RAGK_QAO(4, 16, 32)
  RAGK_QAO(8, 16, 16)
  RAGK_QAO(8, 16, 32)
#undef RAGK_QAO
  return (int)hipErrorInvalidValue;
}

RAGK_API int ragk_attn_oproj_cnt_ints() { return CNT_INTS; }

RAGK_API int ragk_fused_set_stamps(unsigned long long* stamps, hipStream_t st) {
  g_fused_stamps_host = stamps;
  return (int)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fused_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice, st);
}
