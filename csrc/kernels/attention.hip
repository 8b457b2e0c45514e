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

template <typename F, int... Is>
__device__ __forceinline__ void pp_static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, i>) for i = 0..N-1 (compile-time slot indices of a fully unrolled loop)
template <int N, typename F>
__device__ __forceinline__ void pp_static_for(F&& f) {
  pp_static_for_impl(f, std::make_integer_sequence<int, N>{});
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
  // PH = t & 3, a compile-time constant (the loop below is unrolled by the ring's 4 slots): with the slot
  // offsets constant every fragment read folds its tile offset into the ds_read immediate (one v_add per
  // fragment read with runtime offsets; unrolled: 6 x 5.4k 1328 -> 1279 us, one 5.2k prompt 250 -> 229,
  // profiles/attn_prefill_unroll4_ab_r5.log)
  auto fast = [&](auto ph_tag, int t, f32x16 (&S_cur)[2], f32x16 (&S_next)[2]) {
    constexpr int PH = decltype(ph_tag)::value;
    unsigned long long t0 = 0;
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    static_assert(V3_NS == 4 && PH >= 0 && PH < 4, "slot phase");
    constexpr int vo = (V3_NS + ((PH + 3) & 3)) * C::TILEB;  // V(t - 1)
    constexpr int ko = ((PH + 1) & 3) * C::TILEB;            // K(t + 1)
    constexpr int vno = (V3_NS + PH) * C::TILEB;             // V(t)
    const bool st_k = t + 3 < n_kt, st_v = t + 2 < n_kt;
    const int soff_k = tile_soff(st_k ? t + 3 : 0);
    const int soff_v = tile_soff(st_v ? t + 2 : 0);
    float alpha = 1.f, mx = -INFINITY, mref = 0.f, ls = 0.f, pend = 0.f;
    float pv[32];  // the probabilities of this tile (P is packed from here, S_cur is not rewritten)
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
        // no input pins: a pinned copy of each element cost a v_mov (the sched barrier keeps the slot)
#pragma unroll
        for (int e = 0; e < 8; ++e) mx = fmaxf(mx, S_cur[i / 2][8 * (i % 2) + e]);
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
        // elements x with 5 + (27 x) / 32 == i: the probability straight from the accumulator, pinned
        // (results only: a pinned copy of an input element cost a v_mov); each is added to the row sum
        // one element later (no exp -> add dependency inside a slot)
        pp_static_for<32>([&](auto xc) {
          constexpr int x = decltype(xc)::value;
          if constexpr (5 + (27 * x) / 32 == i) {
            float pe = __builtin_amdgcn_exp2f(__builtin_fmaf(S_cur[x >> 4][x & 15], c, -mref));
            pin(pe);
            ls += pend;  // the previous element's value: no exp -> add dependency inside a slot
            pend = pe;
            pv[x] = pe;
            if constexpr (x % 8 == 7) {
              P[x / 8] = (bf16x8){f2bf_s(pv[x - 7]), f2bf_s(pv[x - 6]), f2bf_s(pv[x - 5]), f2bf_s(pv[x - 4]),
                                  f2bf_s(pv[x - 3]), f2bf_s(pv[x - 2]), f2bf_s(pv[x - 1]), f2bf_s(pv[x])};
              pin(P[x / 8]);
            }
            pin(ls);
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
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    for (; t + 3 < t_end; t += 4) {  // t = 1 (mod 4) at every trip
      fast(P1{}, t, S1, S0);
      fast(P2{}, t + 1, S0, S1);
      fast(P3{}, t + 2, S1, S0);
      fast(P0{}, t + 3, S0, S1);
    }
    if (t < t_end) {
      fast(P1{}, t, S1, S0);
      ++t;
    }
    if (t < t_end) {
      fast(P2{}, t, S0, S1);
      ++t;
    }
    if (t < t_end) {
      fast(P3{}, t, S1, S0);
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
  // Fused RoPE + KV append (null qkv_p: q is read from `q` and the cache already holds the new token).
  // The qkv projection arrives as fp32 split-K partial slabs P[S][B][ldp] (gemm_part.hip); every
  // block sums + rotates its G query heads itself, and the block owning the last KV tile also sums,
  // rotates and appends the new token's k / v before reading that tile.
  const float* qkv_p; long long p_slab; int ldp, S;
  const int* positions; const int* slots;
  const float* cos_t; const float* sin_t;
};

// Tiles per partition of one sequence: its KV tiles spread evenly over all max_parts partitions
// (never fewer than part_tiles per partition). The grid is sized once for max_parts (hipGraph
// capture), so sizing the split from the actual length keeps every launched block busy with the
// same amount of KV: splitting a 5.3k-token context by a fixed 32-tile partition left 1 of 4
// partitions idle and 8 vs 5 tiles per wave on the others.
__device__ __forceinline__ int decode_part_tiles(int n_kt, const DecodeArgs& a) {
  return max(a.part_tiles, (n_kt + a.max_parts - 1) / a.max_parts);
}

// LDS of one decode-attention block: one V tile per wave (KL: and one K tile per wave after them), then the
// block's rotated q (G x D bf16).
template <int D, int G, int NW = 4, bool KL = false>
constexpr int decode_lds_bytes() { return NW * Cfg<D>::TILEB * (KL ? 2 : 1) + G * D * 2; }

// One split-K partition block of decode attention: partition `part` of KV head `kvh` of sequence `b`.
// NW: waves per block (4; 8 for the batch-32 grid with one partition per sequence: one 8-wave block per
// CU keeps the same KV bytes in flight as two 4-wave blocks and needs no merge launch). A multi-partition
// sequence writes its partition records; attn_decode_reduce_kernel (or, deferred, the o_proj GEMM's
// gemm_part_merge) merges them.
// DG = 1 (diagnostic build, tools/attn_decode_probe.py): the same K / V loads and waits, no QK^T / softmax / PV
// -- how much of the kernel's time the KV access pattern alone takes. DG = 2: as 1, but K also arrives by
// LDS-DMA (1 KiB per instruction, into the V buffer: results meaningless) instead of 64-B row pieces.
// KL: K tiles arrive by LDS-DMA too (whole 1 KiB pieces instead of 64-B row pieces per lane: the pure access
// pattern streams 4-5 % faster, tools/attn_decode_probe.py) and the QK^T fragments are read from LDS; a
// wave then holds 32 KB of LDS, so the single-partition grid uses 4-wave blocks (one per CU).
template <int D, int G, bool NT = false, int NW = 4, int DG = 0, bool KL = false>
__device__ __forceinline__ void attn_decode_block(const DecodeArgs& a, int part, int kvh, int b, char* smem) {
  constexpr int NTH = NW * 64;
  using C = Cfg<D>;
  static_assert(G <= 16, "at most 16 query heads per KV head");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int kv_len = a.kv_lens[b];
  const int n_kt = (kv_len + KT - 1) / KT;
  const int pt = decode_part_tiles(n_kt, a);
  const int kt0 = part * pt;
  if (kt0 >= n_kt) return;  // block-uniform early exit (before any barrier)
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
  char* sK = smem + (NW + wid) * C::TILEB;  // KL only
  const bool pre = a.qkv_p != nullptr && kt0 + wid_u < kt1 && kt0 + wid_u != n_kt - 1;  // wave-uniform
  bf16x8 kf0[4][C::KS];
  if (pre) {
    const size_t base = ((size_t)bt[kt0 + wid_u] * a.Hkv + kvh) * KT * D;
    const bf16_t* kb = a.kc + base;
    const bf16_t* vb = a.vc + base;
    if constexpr (KL) stage_kv<D, false, NT, 1>(sK, 0, 1, lane, [&](int r) { return kb + (size_t)r * D; });
    stage_kv<D, true, NT, 1>(sV, 0, 1, lane, [&](int r) { return vb + (size_t)r * D; });
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < C::KS; ++s)
        if constexpr (!KL)
          kf0[t][s] = NT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D +
                                                                                     32 * s + 8 * fh))
                         : *reinterpret_cast<const bf16x8*>(kb + (size_t)(16 * t + fr) * D + 32 * s + 8 * fh);
  }
  if (a.qkv_p != nullptr) {
    // q = RoPE(bf16(sum_s P[s][b])) for this KV head's G query heads, one (d, d + D/2) rotate_half
    // pair of 8-vectors per thread (G * D/16 threads, all slab loads of a thread in flight together),
    // staged through LDS; in the block owning the last KV tile, other threads append the new
    // token's k (rotated) and v meanwhile. One barrier covers both.
    bf16_t* s_q = reinterpret_cast<bf16_t*>(smem + NW * C::TILEB * (KL ? 2 : 1));
    constexpr int NV = D / 16;  // pairs per head
    const int pos = a.positions[b];
    const float* prow = a.qkv_p + (size_t)b * a.ldp;
    const float* ct = a.cos_t + (size_t)pos * (D / 2);
    const float* st = a.sin_t + (size_t)pos * (D / 2);
    const int tid = threadIdx.x;
    const bool append = kt1 == n_kt;  // block-uniform
    constexpr int KV0 = (G * NV + 63) / 64 * 64;  // append threads start on a fresh wave
    if (tid < G * NV) {
      const int g = tid / NV, v = tid % NV;
      const float* ph = prow + (size_t)(kvh * G + g) * D + 8 * v;
      float x1[8], x2[8], o1[8], o2[8];
      sum_partials8x2(ph, ph + D / 2, a.S, (size_t)a.p_slab, x1, x2);
      rope8(x1, x2, ct + 8 * v, st + 8 * v, o1, o2);
      *reinterpret_cast<u32x4*>(s_q + g * D + 8 * v) = pack8(o1);
      *reinterpret_cast<u32x4*>(s_q + g * D + D / 2 + 8 * v) = pack8(o2);
    } else if (append && tid >= KV0 && tid < KV0 + 2 * NV) {  // [KV0, KV0+NV): k, [KV0+NV, KV0+2NV): v
      const int isv = tid - KV0 >= NV, v = (tid - KV0) % NV;
      const int slot = a.slots[b];
      const size_t kvo = (((size_t)(slot / KT) * a.Hkv + kvh) * KT + (slot % KT)) * D;
      const float* ph = prow + (size_t)(a.Hq + (isv ? a.Hkv : 0) + kvh) * D + 8 * v;
      float x1[8], x2[8];
      sum_partials8x2(ph, ph + D / 2, a.S, (size_t)a.p_slab, x1, x2);
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
  unsigned dsink = 0;

  for (int kt = kt0 + wid_u; kt < kt1; kt += NW) {
    bf16x8 kf[4][C::KS];
    if constexpr (KL) {
      if (!(pre && kt == kt0 + wid_u)) {  // else staged before the prologue
        const size_t base = ((size_t)bt[kt] * a.Hkv + kvh) * KT * D;
        const bf16_t* kb = a.kc + base;
        const bf16_t* vb = a.vc + base;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous tile's K / V reads retired
        stage_kv<D, false, NT, 1>(sK, 0, 1, lane, [&](int r) { return kb + (size_t)r * D; });
        stage_kv<D, true, NT, 1>(sV, 0, 1, lane, [&](int r) { return vb + (size_t)r * D; });
      }
      // K first: QK^T and the softmax run while the V tile (the 16 youngest LDS-DMAs) is still landing. The
      // builtin wait (not inline asm) updates the compiler's own counter model, so it adds no vmcnt(0) of its own.
      static_assert(Cfg<D>::PIECES < 64, "vmcnt range");
      __builtin_amdgcn_s_waitcnt((Cfg<D>::PIECES & 15) | (((Cfg<D>::PIECES >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s) kf[t][s] = load_k<D>(sK, t, s, lane);
    } else if (pre && kt == kt0 + wid_u) {  // requested before the prologue
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s) kf[t][s] = kf0[t][s];
    } else if (DG == 2) {
      const size_t base = ((size_t)bt[kt] * a.Hkv + kvh) * KT * D;
      const bf16_t* kb = a.kc + base;
      const bf16_t* vb = a.vc + base;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stage_kv<D, true, NT, 1>(sV, 0, 1, lane, [&](int r) { return vb + (size_t)r * D; });
      stage_kv<D, false, NT, 1>(sV, 0, 1, lane, [&](int r) { return kb + (size_t)r * D; });
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s) kf[t][s] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
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
    if constexpr (DG != 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < C::KS; ++s) dsink ^= __builtin_bit_cast(u32x4, kf[t][s])[0];
      wait_vmcnt0();
      dsink ^= *reinterpret_cast<const unsigned*>(sV + 4 * lane);
      continue;
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
    // raw v_exp_f32 (the libm exp2f adds a denormal-range fixup per call: ~4 VALU; softmax terms below
    // 2^-126 do not change any fp32 sum here)
    const float alpha = __builtin_amdgcn_exp2f(m_i - m_use);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(s4[t][r] - m_use);
        s4[t][r] = p;
        ls += p;
      }
    l_i = l_i * alpha + ls;
    m_i = m_new;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) o[dt] *= alpha;
    const bf16x8 pb0 = pack_p(s4[0], s4[1]);
    const bf16x8 pb1 = pack_p(s4[2], s4[3]);
    if constexpr (KL)
      __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));  // V tile landed (vmcnt(0), seen by the compiler)
    else
      wait_vmcnt0();  // V tile landed in this wave's LDS
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_vt<D>(sV, dt, 0, lane), pb0, o[dt], 0, 0, 0);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_vt<D>(sV, dt, 1, lane), pb1, o[dt], 0, 0, 0);
    }
  }

  if constexpr (DG != 0) {
    if (dsink == 0x9e3779b9u) a.out[(size_t)b * a.out_stride + lane] = 0;  // keeps the loads alive
    return;
  }
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
    if (nparts == 1) {
      a.out[(size_t)b * a.out_stride + hq * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const size_t pi = ((size_t)b * a.Hq + hq) * a.max_parts + part;
      a.part_o[pi * D + d] = O;
      if (d == 0) {
        a.part_ml[pi * 2] = M;
        a.part_ml[pi * 2 + 1] = L;
      }
    }
  }
}

template <int D, int G, bool NT = false, int NW = 4, int DG = 0, bool KL = false>
__global__ __launch_bounds__(NW * 64, (NW == 4 && !KL) ? 2 : 1) void attn_decode_kernel(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[decode_lds_bytes<D, G, NW, KL>()];
  attn_decode_block<D, G, NT, NW, DG, KL>(a, blockIdx.x, blockIdx.y, blockIdx.z, smem);
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

// Block order (prefill_block): a 1-D grid, head group fastest, so the heaviest causal tiles of every head
// start first and consecutive blocks (round-robin over the XCDs) put one KV head on each XCD.
// Kernel per config:
//   * Llama (D 128, 4 query heads per KV head, causal, paged cache < 4 GiB): the software-pipelined
//     8-wave kernel with the whole-row LDS epilogue (attn_prefill_v3_kernel<8, ..., WIDE>; 64-query
//     tiles), tools/attn_pp_ab.py;
//   * every other 4-heads-per-block config: attn_prefill_kernel with 8 waves (64-query tiles, two 32-row
//     groups sharing each K/V tile);
//   * 1 or 2 heads per block (encoders, GPT-2, odd GQA ratios): the 4-wave attn_prefill_kernel.
template <int D, int GB, bool CAUSAL, bool PAGED>
hipError_t launch_prefill(PrefillArgs a, int n_tiles, hipStream_t st) {
  const int G = a.Hq / a.Hkv;
  const int n_hg = a.Hkv * (G / GB);
  a.n_hg = n_hg;
  const dim3 grid(n_tiles * n_hg);
  if constexpr (D == 128 && GB == 4 && CAUSAL && PAGED) {
    if (a.kv_bytes) {
      hipLaunchKernelGGL((attn_prefill_v3_kernel<8, false, 0, 1, true>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
  }
  if constexpr (GB == 4)
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED, false, 8>), grid, dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((attn_prefill_kernel<D, GB, CAUSAL, PAGED>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace

// Query rows per block (the host builds `tiles` with this step): 64 for 4 heads per block, else 128 / GB.
RAGK_API int ragk_attn_prefill_qtile(int Hq, int Hkv) {
  const int G = Hq / Hkv;
  const int GB = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
  return 32 * ((GB == 4 ? 8 : 4) / GB);
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


// K/V cache-policy switch for decode (0 = default, 1 = non-temporal loads; the KV stream is read
// once per step). A/B in tools/bench_kernels.py --quick.
static int g_decode_nt = 0;
// 8-wave single-partition decode attention once batch x KV heads reaches this (0 = never)
static int g_decode_nw8_min = 0;
// diagnostic instantiation of the 8-wave kernel (DG above; A/B tooling only, 0 = off)
static int g_decode_diag = 0;
// single-partition grid on 4-wave blocks with K tiles by LDS-DMA (KL above; 0 = the 8-wave kernel)
static int g_decode_kl = 0;
RAGK_API int ragk_attn_decode_set_kl(int on) {
  g_decode_kl = on ? 1 : 0;
  return 0;
}
RAGK_API int ragk_attn_decode_set_diag(int dg) {
  g_decode_diag = (dg == 1 || dg == 2) ? dg : 0;
  return 0;
}
RAGK_API int ragk_attn_decode_set_nw8(int min_pairs) {
  g_decode_nw8_min = min_pairs > 0 ? min_pairs : 0;
  return 0;
}
RAGK_API int ragk_attn_decode_set_nt(int nt) {
  g_decode_nt = nt ? 1 : 0;
  return 0;
}

static int launch_attn_decode(DecodeArgs a, int B, int D, int max_parts, hipStream_t st);

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
                              float scale, hipStream_t st) {
  if (B <= 0) return 0;
  if (Hq % Hkv || part_tiles < 1 || max_parts < 1 || max_parts > RED_MAXP) return (int)hipErrorInvalidValue;
  DecodeArgs a{(const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, (bf16_t*)out, out_stride, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f};
  return launch_attn_decode(a, B, D, max_parts, st);
}

// Decode attention fed by the qkv projection's split-K partial slabs P[S][B][ldp] (gemm_part.hip):
// RoPE of q and k, the KV append at slots[b] and the attention in one launch (replaces
// rope_kv_partials + attn_decode). Cache blocks hold KT tokens.
RAGK_API int ragk_attn_decode_rope(const float* P, int S, int ldp, const int* positions, const int* slots,
                                   const float* cos_t, const float* sin_t, void* kc, void* vc,
                                   const int* block_tables, int bt_stride, const int* kv_lens, float* part_o,
                                   float* part_ml, void* out, int out_stride, int B, int Hq, int Hkv, int D,
                                   int part_tiles, int max_parts, float scale, hipStream_t st) {
  if (B <= 0) return 0;
  if (Hq % Hkv || part_tiles < 1 || max_parts < 1 || max_parts > RED_MAXP || S < 1 || D % 64 ||
      ldp < (Hq + 2 * Hkv) * D || !P || !positions || !slots || !cos_t || !sin_t)
    return (int)hipErrorInvalidValue;
  DecodeArgs a{nullptr, 0, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, bt_stride, kv_lens,
               part_o, part_ml, (bf16_t*)out, out_stride, Hq, Hkv, part_tiles, max_parts,
               scale * 1.4426950408889634f, P, (long long)B * ldp, ldp, S, positions, slots, cos_t, sin_t};
  return launch_attn_decode(a, B, D, max_parts, st);
}

static int launch_attn_decode(DecodeArgs a, int B, int D, int max_parts, hipStream_t st) {
  const int Hq = a.Hq, Hkv = a.Hkv;
  const int G = Hq / Hkv;
  dim3 grid(max_parts, Hkv, B);
  if (D == 128 && G == 4 && max_parts == 1 && g_decode_nw8_min > 0 && B * Hkv >= g_decode_nw8_min) {
    // one partition per sequence over >= 1 block per CU: 8-wave blocks, no merge launch
    if (g_decode_kl && !g_decode_diag)
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, true, 4, 0, true>), grid, dim3(256), 0, st, a);
    else if (g_decode_diag == 1)
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, true, 8, 1>), grid, dim3(512), 0, st, a);
    else if (g_decode_diag == 2)
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, true, 8, 2>), grid, dim3(512), 0, st, a);
    else if (g_decode_nt)
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, true, 8>), grid, dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL((attn_decode_kernel<128, 4, false, 8>), grid, dim3(512), 0, st, a);
    return (int)hipGetLastError();
  }
#define RAGK_DC(DD, GG)                                                            \
  if (D == DD && G == GG) {                                                          \
    if (g_decode_nt)                                                                 \
      hipLaunchKernelGGL((attn_decode_kernel<DD, GG, true>), grid, dim3(256), 0, st, a); \
    else                                                                             \
      hipLaunchKernelGGL((attn_decode_kernel<DD, GG, false>), grid, dim3(256), 0, st, a); \
    if (max_parts > 1 && !g_decode_defer)                                            \
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

