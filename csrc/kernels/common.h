// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Every kernel in csrc/kernels/*.hip is written for 64-lane wavefronts, MFMA
// matrix cores and the 160 KiB LDS of gfx950. No CUDA / dual-path code: this
// library only targets --offload-arch=gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RAGK_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

namespace ragk {

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(((unsigned)x) << 16);
}
__device__ __forceinline__ float bf2f_s(short x) {
  return __uint_as_float(((unsigned)(unsigned short)x) << 16);
}
// Round-to-nearest-even f32 -> bf16; hipcc lowers the __bf16 cast to
// v_cvt_pk_bf16_f32 on gfx950 (keeps NaNs NaN).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}
__device__ __forceinline__ short f2bf_s(float f) { return (short)f2bf(f); }
// two floats -> packed bf16x2 (lo = a) in ONE v_cvt_pk_bf16_f32 (two scalar f2bf + shift/or is 3-4)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk2bf(float a, float b) {
  const bf16x2_t h = __builtin_convertvector((f32x2){a, b}, bf16x2_t);
  return __builtin_bit_cast(unsigned, h);
}

// 16-byte vector of 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = pk2bf(f[2 * i], f[2 * i + 1]);
  return v;
}

// Sum of S fp32 slabs of 8 consecutive floats (slab stride in floats), added in slab order 0..S-1.
// Loads go out in unrolled groups of PSU slabs (index clamped, the excess not added), so a thread
// has 2 x PSU loads in flight instead of one slab's pair per memory latency (a runtime-S loop made
// hipcc wait on every slab: 7.7 us for the qkv slabs at S = 8).
constexpr int PSU = 8;
__device__ __forceinline__ void sum_slabs8(const float* P, int S, size_t slab, float* a) {
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  for (int s0 = 0; s0 < S; s0 += PSU) {
    f32x4 p[PSU][2];
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      const f32x4* ps = reinterpret_cast<const f32x4*>(P + (size_t)min(s0 + u, S - 1) * slab);
      p[u][0] = ps[0];
      p[u][1] = ps[1];
    }
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      if (s0 + u < S) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] += p[u][0][e];
          a[4 + e] += p[u][1][e];
        }
      }
    }
  }
}

// sum_slabs8 split in two, so a kernel can put other independent loads (residual row, norm weights)
// in flight with the first PSU slabs' loads: load_slabs8 issues them (index clamped), add_slabs8 sums
// them in slab order and streams any slabs beyond PSU serially.
__device__ __forceinline__ void load_slabs8(const float* P, int S, size_t slab, f32x4 (&p)[PSU][2]) {
#pragma unroll
  for (int u = 0; u < PSU; ++u) {
    const f32x4* ps = reinterpret_cast<const f32x4*>(P + (size_t)min(u, S - 1) * slab);
    p[u][0] = ps[0];
    p[u][1] = ps[1];
  }
}
__device__ __forceinline__ void add_slabs8(const f32x4 (&p)[PSU][2], const float* P, int S, size_t slab, float* a) {
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
#pragma unroll
  for (int u = 0; u < PSU; ++u) {
    if (u < S) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] += p[u][0][e];
        a[4 + e] += p[u][1][e];
      }
    }
  }
  for (int s0 = PSU; s0 < S; s0 += PSU) {  // same order as sum_slabs8: one accumulator, slab by slab
    f32x4 q[PSU][2];
    load_slabs8(P + (size_t)s0 * slab, S - s0, slab, q);
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      if (s0 + u < S) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] += q[u][0][e];
          a[4 + e] += q[u][1][e];
        }
      }
    }
  }
}

__device__ __forceinline__ void sum_partials8(const float* P, int S, size_t slab, float* a) {
  sum_slabs8(P, S, slab, a);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = bf2f(f2bf(a[e]));
}

// sum_partials8 of two 8-float vectors at once (their 4 x PSU slab loads in flight together; each
// element summed in slab order 0..S-1, so the results equal two sum_partials8 calls)
__device__ __forceinline__ void sum_partials8x2(const float* P1, const float* P2, int S, size_t slab, float* a,
                                                float* b) {
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  for (int s0 = 0; s0 < S; s0 += PSU) {
    f32x4 p[PSU][4];
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      const size_t o = (size_t)min(s0 + u, S - 1) * slab;
      p[u][0] = reinterpret_cast<const f32x4*>(P1 + o)[0];
      p[u][1] = reinterpret_cast<const f32x4*>(P1 + o)[1];
      p[u][2] = reinterpret_cast<const f32x4*>(P2 + o)[0];
      p[u][3] = reinterpret_cast<const f32x4*>(P2 + o)[1];
    }
#pragma unroll
    for (int u = 0; u < PSU; ++u) {
      if (s0 + u < S) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] += p[u][0][e];
          a[4 + e] += p[u][1][e];
          b[e] += p[u][2][e];
          b[4 + e] += p[u][3][e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = bf2f(f2bf(a[e]));
    b[e] = bf2f(f2bf(b[e]));
  }
}

// HF rotate_half RoPE on one pair of 8-element half-vectors (x1 = d in [0, D/2), x2 = d + D/2) with
// the bf16 rounding of every torch op (q*cos, rotate_half(q)*sin, their sum).
__device__ __forceinline__ void rope8(const float* x1, const float* x2, const float* ct, const float* st, float* o1,
                                      float* o2) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float c = ct[e], sn = st[e];
    o1[e] = bf2f(f2bf(bf2f(f2bf(x1[e] * c)) + bf2f(f2bf(-x2[e] * sn))));
    o2[e] = bf2f(f2bf(bf2f(f2bf(x2[e] * c)) + bf2f(f2bf(x1[e] * sn))));
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `red` needs
// blockDim.x/64 floats of LDS. Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Bijective XCD-aware block remap (MI355X: 8 XCDs, blocks dealt round-robin).
// Blocks b, b+8, b+16... share an XCD; remap so each XCD gets a contiguous range
// of logical tile ids (neighbouring tiles share operand panels in its L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// x * sigmoid(x) with the hardware reciprocal (1 ulp) instead of an IEEE division: the division's
// scale / fma / fixup sequence was ~10 VALU per element in the gate/up GEMM epilogues
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// async global -> LDS copy, 16 B per lane; LDS destination = wave-uniform base + lane*16.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base,
                                   16, 0, 0);
}
__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): the per-lane source is a 32-bit byte
// offset (one VGPR, reusable across K-steps) + a wave-uniform SGPR offset, no 64-bit VALU address
// math per load. The LDS destination is M0 (wave-uniform base) + lane*16, as for glds16.
typedef __attribute__((ext_vector_type(4))) int i32x4;
__device__ void ragk_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) unsigned* lds, int size,
                                         int voffset, int soffset, int offset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

// Raw buffer descriptor (stride 0, bounds = `bytes`); dword3 = gfx9 data-format bits.
__device__ __forceinline__ i32x4 make_srd(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

__device__ __forceinline__ void blds16(i32x4 srd, int voff, int soff, void* lds_wave_base) {
  ragk_raw_buffer_load_lds(srd, (__attribute__((address_space(3))) unsigned*)lds_wave_base, 16, voff, soff, 0, 0);
}



// ---- lane-level bitonic networks over (value, id) pairs held one per lane of a wave (ascending by
// value, ties -> lower id as unsigned): the wave-resident top-64 lists of the L2 search and the
// small-batch sampler top-k. Every lane exchange stays on the VALU.
// Branch-free (bitwise | and &, selects): the short-circuit forms compiled to exec-mask branches around
// every compare-exchange, ~15 scalar / branch instructions per network step on a one-wave-per-SIMD
// dependent chain.
__device__ __forceinline__ bool cand_lt(float av, int ai, float bv, int bi) {
  return (av < bv) | ((av == bv) & ((unsigned)ai < (unsigned)bi));
}

// value of lane (lane ^ j), j a power of two that is a compile-time constant after unrolling: every
// exchange stays on the VALU -- DPP quad permutes / mirrors (one or two moves) for j <= 8,
// v_permlane16_swap / v_permlane32_swap for 16 / 32 -- instead of the LDS-pipe ds_bpermute (or
// ds_swizzle) whose round trip bounded every step of the networks below.
__device__ __forceinline__ int xor_lane(int v, int j, int lane) {
  if (j == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  if (j == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  if (j == 4)  // (i ^ 3) then the 8-lane mirror (i ^ 7): i ^ 4
    return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x1B, 0xF, 0xF, false), 0x141, 0xF, 0xF, false);
  if (j == 8)  // 8-lane mirror (i ^ 7) then the row mirror (i ^ 15): i ^ 8
    return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false), 0x140, 0xF, 0xF, false);
  if (j == 16) {  // odd rows of vdst <-> even rows of vsrc
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((lane >> 4) & 1) ? (int)p[0] : (int)p[1];
  }
  if (j == 32) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return lane < 32 ? (int)p[1] : (int)p[0];
  }
  return __shfl_xor(v, j, 64);
}

// value of lane 63 - lane (= lane ^ 63): DPP row mirror (lane ^ 15), then xor 16 and xor 32
__device__ __forceinline__ int rev_lane(int v, int lane) {
  return xor_lane(xor_lane(__builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false), 16, lane), 32, lane);
}
__device__ __forceinline__ float rev_lane(float v, int lane) { return __int_as_float(rev_lane(__float_as_int(v), lane)); }

// one compare-exchange step of a lane-level bitonic network (partner = lane ^ j)
__device__ __forceinline__ void cx(float& v, int& i, int lane, int j, bool asc) {
  const float ov = __int_as_float(xor_lane(__float_as_int(v), j, lane));
  const int oi = xor_lane(i, j, lane);
  const bool keep_min = ((lane & j) == 0) == asc;
  // keep_min: take the partner iff it precedes; keep_max: iff it does not (equal pairs: either)
  const bool take = keep_min == cand_lt(ov, oi, v, i);
  v = take ? ov : v;
  i = take ? oi : i;
}

// ascending sort of the 64 (v, i) pairs held one per lane
__device__ __forceinline__ void wave_sort64(float& v, int& i, int lane) {
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) cx(v, i, lane, j, (lane & kk) == 0);
}

// (bv, bi) sorted ascending, (nv, ni) sorted ascending -> (bv, bi) = the 64 smallest of both, sorted
__device__ __forceinline__ void wave_merge64(float& bv, int& bi, float nv, int ni, int lane) {
  const float rv = rev_lane(nv, lane);
  const int ri = rev_lane(ni, lane);
  const bool take = cand_lt(rv, ri, bv, bi);
  bv = take ? rv : bv;
  bi = take ? ri : bi;
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) cx(bv, bi, lane, j, true);
}

// feed 64 unsorted candidates (one per lane) into the running top list; k-th best = threshold
__device__ __forceinline__ void wave_offer(float& bv, int& bi, float v, int id, int k, int lane) {
  const float tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv), k - 1));  // k uniform
  const int ti = __builtin_amdgcn_readlane(bi, k - 1);
  if (!__any(cand_lt(v, id, tv, ti))) return;  // wave-uniform
  wave_sort64(v, id, lane);
  wave_merge64(bv, bi, v, id, lane);
}

}  // namespace ragk

// Epilogue selector shared by the GEMM family.
enum RagkEpilogue : int {
  EPI_NONE = 0,      // C = acc
  EPI_BIAS = 1,      // C = acc + bias[n]
  EPI_RESID = 2,     // C = resid + acc            (resid may alias C)
  EPI_BIAS_RESID = 3,// C = resid + acc + bias[n]
  EPI_BIAS_GELU = 4, // C = gelu_erf(acc + bias[n])
  EPI_SILU_MUL = 5,  // paired columns: C[:, j] = silu(gate_j) * up_j
  EPI_GELU = 6,      // C = gelu_erf(acc)
  EPI_BIAS_GELU_TANH = 7,  // GPT-2 MLP
  EPI_ROPE_KV = 8,   // qkv projection (D = 128 heads): RoPE on q / k, k and v rows also into the paged KV cache
};
