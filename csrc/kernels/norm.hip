// Memory-bound row kernels for gfx950: RMSNorm, LayerNorm, embedding gathers,
// fused RoPE + paged-KV write, pooling + L2 normalise, standalone SiLU*up.
//
// All loads/stores are 16-byte vectors (8 x bf16) -- hipcc does not vectorise
// bf16 on its own. Rows map to blocks of 256 threads (4 waves); reductions are
// wave shuffles + one LDS exchange.
//
// Reference semantics reproduced here:
//   K1 embed_tokens gather, K2 LlamaRMSNorm (fp32 variance, cast back, *weight),
//   K4 llama3-scaled RoPE in rotate_half layout, K13 KV-cache append,
//   E1 BERT/XLM-R embeddings (+LayerNorm), E4/E6 post-LN LayerNorm,
//   E7 CLS / masked-mean pooling + L2 normalise (sentence-transformers
//   Normalize(), /root/reference/llm/rag.py:55 normalize_embeddings=True).
#include <algorithm>

#include "common.h"
using namespace ragk;

namespace {

constexpr int NT = 256;

// out = bf16( w * bf16( x * rsqrt(mean(x^2) + eps) ) )      (HF LlamaRMSNorm exactly)
// If resid != nullptr: x = bf16(x + resid) is computed first and written back to resid
// (fused residual add: resid holds the new residual stream).
__global__ __launch_bounds__(NT) void rmsnorm_kernel(const bf16_t* x, int ldx, bf16_t* resid, int ldr,
                                                     const bf16_t* __restrict__ w, bf16_t* out, int ldo,
                                                     int H, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (size_t)row * ldx;
  bf16_t* rr = resid ? resid + (size_t)row * ldr : nullptr;
  bf16_t* orow = out + (size_t)row * ldo;
  constexpr int MAXV = 4;  // up to 4 x 8 x 256 = 8192 columns held in registers
  float v[MAXV][8];
  const int nvec = H >> 3;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      unpack8(*reinterpret_cast<const u32x4*>(xr + vi * 8), v[i]);
      if (rr) {
        float r8[8];
        unpack8(*reinterpret_cast<const u32x4*>(rr + vi * 8), r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = bf2f(f2bf(v[i][e] + r8[e]));
        *reinterpret_cast<u32x4*>(rr + vi * 8) = pack8(v[i]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      float wv[8], o[8];
      unpack8(*reinterpret_cast<const u32x4*>(w + vi * 8), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = wv[e] * bf2f(f2bf(v[i][e] * inv));
      *reinterpret_cast<u32x4*>(orow + vi * 8) = pack8(o);
    }
  }
}

// LayerNorm over the last dim (fp32 statistics, two-pass in registers), optional
// fused residual: y = LN(x + resid) * g + b.
__global__ __launch_bounds__(NT) void layernorm_kernel(const bf16_t* x, int ldx, const bf16_t* resid, int ldr,
                                                       const bf16_t* __restrict__ g, const bf16_t* __restrict__ b,
                                                       bf16_t* out, int ldo, int H, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (size_t)row * ldx;
  constexpr int MAXV = 4;
  float v[MAXV][8];
  const int nvec = H >> 3;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      unpack8(*reinterpret_cast<const u32x4*>(xr + vi * 8), v[i]);
      if (resid) {
        float r8[8];
        unpack8(*reinterpret_cast<const u32x4*>(resid + (size_t)row * ldr + vi * 8), r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += r8[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  const float mean = block_sum(s, red) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[i][e] - mean;
        sq += d * d;
      }
  }
  const float inv = rsqrtf(block_sum(sq, red) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      float gv[8], bv[8], o[8];
      unpack8(*reinterpret_cast<const u32x4*>(g + vi * 8), gv);
      unpack8(*reinterpret_cast<const u32x4*>(b + vi * 8), bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * inv * gv[e] + bv[e];
      *reinterpret_cast<u32x4*>(out + (size_t)row * ldo + vi * 8) = pack8(o);
    }
  }
}

// token embedding gather: out[t] = table[ids[t]]
// carry (optional, asynchronous decode): carry[t] >= 0 takes the token id from prev[carry[t]] (the
// previous decode step's sampled tokens, still on the device) instead of ids[t]; the resolved id is
// written back to ids[t] so the step's inputs stay self-describing.
__global__ __launch_bounds__(NT) void embed_kernel(int* __restrict__ ids, const bf16_t* __restrict__ table,
                                                   bf16_t* out, int H, int vocab, const int* __restrict__ carry,
                                                   const int* __restrict__ prev) {
  const int t = blockIdx.x;
  int id = ids[t];
  if (carry != nullptr) {
    const int c = carry[t];
    if (c >= 0) {
      id = prev[c];
      __syncthreads();  // every lane has read ids[t] before lane 0 overwrites it
      if (threadIdx.x == 0) ids[t] = id;
    }
  }
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const u32x4* src = reinterpret_cast<const u32x4*>(table + (size_t)id * H);
  u32x4* dst = reinterpret_cast<u32x4*>(out + (size_t)t * H);
  for (int i = threadIdx.x; i < (H >> 3); i += NT) dst[i] = src[i];
}

// BERT / XLM-R embeddings: LN(word[id] + pos[pos_id] + type[type_id]) (+ optional GPT-2 style no-LN)
__global__ __launch_bounds__(NT) void embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ pos_ids,
                                                      const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                      const bf16_t* __restrict__ type, const bf16_t* __restrict__ g,
                                                      const bf16_t* __restrict__ b, bf16_t* out, int H, float eps,
                                                      int do_ln) {
  __shared__ float red[NT / 64];
  const int t = blockIdx.x;
  const bf16_t* wr = word + (size_t)ids[t] * H;
  const bf16_t* pr = pos + (size_t)pos_ids[t] * H;
  constexpr int MAXV = 4;
  float v[MAXV][8];
  const int nvec = H >> 3;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      float a[8], p[8];
      unpack8(*reinterpret_cast<const u32x4*>(wr + vi * 8), a);
      unpack8(*reinterpret_cast<const u32x4*>(pr + vi * 8), p);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = a[e] + p[e];
      if (type) {
        float ty[8];
        unpack8(*reinterpret_cast<const u32x4*>(type + vi * 8), ty);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += ty[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  if (!do_ln) {
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int vi = threadIdx.x + i * NT;
      if (vi < nvec) *reinterpret_cast<u32x4*>(out + (size_t)t * H + vi * 8) = pack8(v[i]);
    }
    return;
  }
  const float mean = block_sum(s, red) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[i][e] - mean;
        sq += d * d;
      }
  }
  const float inv = rsqrtf(block_sum(sq, red) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      float gv[8], bv[8], o[8];
      unpack8(*reinterpret_cast<const u32x4*>(g + vi * 8), gv);
      unpack8(*reinterpret_cast<const u32x4*>(b + vi * 8), bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * inv * gv[e] + bv[e];
      *reinterpret_cast<u32x4*>(out + (size_t)t * H + vi * 8) = pack8(o);
    }
  }
}

// Fused RoPE (rotate_half layout, HF bf16 rounding replicated) + paged KV write.
// qkv row layout: [Hq*D | Hkv*D | Hkv*D]. q is rotated in place, k rotated and
// written to k_cache, v copied to v_cache. Cache layout [nblocks][Hkv][BS][D].
// cos/sin tables: [max_pos][D/2] fp32 holding bf16-rounded values.
// slot < 0 means "do not cache" (padding token).
__global__ __launch_bounds__(NT) void rope_kv_kernel(bf16_t* qkv, int ld, const int* __restrict__ positions,
                                                     const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                     const int* __restrict__ slots, bf16_t* kc, bf16_t* vc, int Hq,
                                                     int Hkv, int D, int BS, int apply_rope) {
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int slot = slots ? slots[t] : -1;
  bf16_t* row = qkv + (size_t)t * ld;
  const int half = D >> 1;
  const int vpr = half >> 3;  // 8-wide vectors per half head
  const float* ct = cos_t + (size_t)pos * half;
  const float* st = sin_t + (size_t)pos * half;
  const int nrot = (Hq + Hkv) * vpr;
  for (int i = threadIdx.x; i < nrot; i += NT) {
    const int h = i / vpr, v = i % vpr;
    bf16_t* hp = row + h * D;
    float x1[8], x2[8], o1[8], o2[8];
    unpack8(*reinterpret_cast<const u32x4*>(hp + v * 8), x1);
    unpack8(*reinterpret_cast<const u32x4*>(hp + half + v * 8), x2);
    if (apply_rope) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float c = ct[v * 8 + e], s = st[v * 8 + e];
        // q*cos + rotate_half(q)*sin, each op rounded to bf16 like torch bf16 math
        o1[e] = bf2f(f2bf(bf2f(f2bf(x1[e] * c)) + bf2f(f2bf(-x2[e] * s))));
        o2[e] = bf2f(f2bf(bf2f(f2bf(x2[e] * c)) + bf2f(f2bf(x1[e] * s))));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { o1[e] = x1[e]; o2[e] = x2[e]; }
    }
    const u32x4 p1 = pack8(o1), p2 = pack8(o2);
    if (h < Hq) {
      *reinterpret_cast<u32x4*>(hp + v * 8) = p1;
      *reinterpret_cast<u32x4*>(hp + half + v * 8) = p2;
    } else if (slot >= 0) {
      const int kh = h - Hq;
      bf16_t* dst = kc + (((size_t)(slot / BS) * Hkv + kh) * BS + (slot % BS)) * D;
      *reinterpret_cast<u32x4*>(dst + v * 8) = p1;
      *reinterpret_cast<u32x4*>(dst + half + v * 8) = p2;
      // keep the rotated k in qkv too (encoder-style consumers / debugging)
      *reinterpret_cast<u32x4*>(hp + v * 8) = p1;
      *reinterpret_cast<u32x4*>(hp + half + v * 8) = p2;
    } else {
      *reinterpret_cast<u32x4*>(hp + v * 8) = p1;
      *reinterpret_cast<u32x4*>(hp + half + v * 8) = p2;
    }
  }
  if (slot >= 0) {
    const int vpd = D >> 3;
    for (int i = threadIdx.x; i < Hkv * vpd; i += NT) {
      const int kh = i / vpd, v = i % vpd;
      const bf16_t* src = row + (Hq + Hkv + kh) * D + v * 8;
      bf16_t* dst = vc + (((size_t)(slot / BS) * Hkv + kh) * BS + (slot % BS)) * D + v * 8;
      *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
    }
  }
}

// out[b] = normalize(pool(hidden[cu[b]:cu[b+1]])) in fp32. mode 0 = CLS (first token),
// mode 1 = masked mean over the sequence, mode 2 = last token.
__global__ __launch_bounds__(NT) void pool_l2norm_kernel(const bf16_t* __restrict__ hidden, int ld,
                                                         const int* __restrict__ cu, float* out, int H, int mode,
                                                         int normalize) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.x;
  const int s0 = cu[b], s1 = cu[b + 1];
  const int len = s1 - s0;
  float ss = 0.f;
  // each thread owns columns c = threadIdx.x + k*NT
  constexpr int MAXC = 8;  // H <= 2048
  float acc[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) acc[k] = 0.f;
  if (mode == 1) {
    for (int t = s0; t < s1; ++t)
#pragma unroll
      for (int k = 0; k < MAXC; ++k) {
        const int c = threadIdx.x + k * NT;
        if (c < H) acc[k] += bf2f(hidden[(size_t)t * ld + c]);
      }
    const float inv = len > 0 ? 1.f / (float)len : 0.f;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) acc[k] *= inv;
  } else {
    const int t = mode == 0 ? s0 : s1 - 1;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int c = threadIdx.x + k * NT;
      if (c < H) acc[k] = bf2f(hidden[(size_t)t * ld + c]);
    }
  }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) ss += acc[k] * acc[k];
  float scale = 1.f;
  if (normalize) {
    ss = block_sum(ss, red);
    scale = 1.f / fmaxf(sqrtf(ss), 1e-12f);  // torch.nn.functional.normalize eps
  }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * NT;
    if (c < H) out[(size_t)b * H + c] = acc[k] * scale;
  }
}

// out[t, j] = silu(x[t, j]) * x[t, I + j]   (unpacked [gate | up] rows)
__global__ __launch_bounds__(NT) void silu_mul_kernel(const bf16_t* x, int ldx, bf16_t* out, int ldo, int I) {
  const int t = blockIdx.x;
  for (int v = threadIdx.x; v < (I >> 3); v += NT) {
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + (size_t)t * ldx + v * 8), g);
    unpack8(*reinterpret_cast<const u32x4*>(x + (size_t)t * ldx + I + v * 8), u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
    *reinterpret_cast<u32x4*>(out + (size_t)t * ldo + v * 8) = pack8(o);
  }
}

// gather rows: out[i] = x[idx[i]]   (last-token selection before lm_head)
__global__ __launch_bounds__(NT) void gather_rows_kernel(const bf16_t* x, int ldx, const int* __restrict__ idx,
                                                         bf16_t* out, int ldo, int H) {
  const int i = blockIdx.x;
  const bf16_t* src = x + (size_t)idx[i] * ldx;
  for (int v = threadIdx.x; v < (H >> 3); v += NT)
    *reinterpret_cast<u32x4*>(out + (size_t)i * ldo + v * 8) = *reinterpret_cast<const u32x4*>(src + v * 8);
}


// ---- consumers of the split-K decode GEMM (gemm_part.hip): they sum the S fp32 partial slabs
// P[S][M][ldp] while doing their own row work, so the reduction needs no extra launch.

// h = bf16(h + bf16(sum_s P[s][row]))  (HF: bf16 linear output, then the bf16 residual add), written
// back to h; out = rmsnorm(h) * w exactly as rmsnorm_kernel. One block of 512 threads per row.
constexpr int PNT = 512;
__global__ __launch_bounds__(PNT) void add_partials_rmsnorm_kernel(const float* __restrict__ P, int S, int M,
                                                                   bf16_t* h, int ldh,
                                                                   const bf16_t* __restrict__ w, bf16_t* out,
                                                                   int ldo, int H, float eps) {
  __shared__ float red[PNT / 64];
  const int row = blockIdx.x;
  bf16_t* hr = h + (size_t)row * ldh;
  constexpr int MAXV = 2;  // up to 2 x 8 x 512 = 8192 columns in registers
  float v[MAXV][8];
  const int nvec = H >> 3;
  float ss = 0.f;
  // every independent load in flight together (one memory round trip, not three): the first PSU
  // slabs, the residual row and the norm weights
  f32x4 pv[MAXV][PSU][2];
  u32x4 hv[MAXV], gv[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = min((int)threadIdx.x + i * PNT, nvec - 1);
    if (i * PNT < nvec) {  // block-uniform
      load_slabs8(P + (size_t)row * H + vi * 8, S, (size_t)M * H, pv[i]);
      hv[i] = *reinterpret_cast<const u32x4*>(hr + vi * 8);
      gv[i] = *reinterpret_cast<const u32x4*>(w + vi * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * PNT;
    if (vi < nvec) {
      float a[8];
      add_slabs8(pv[i], P + (size_t)row * H + vi * 8, S, (size_t)M * H, a);
      unpack8(hv[i], v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = bf2f(f2bf(v[i][e] + bf2f(f2bf(a[e]))));
      *reinterpret_cast<u32x4*>(hr + vi * 8) = pack8(v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * PNT;
    if (vi < nvec) {
      float wv[8], o[8];
      unpack8(gv[i], wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = wv[e] * bf2f(f2bf(v[i][e] * inv));
      *reinterpret_cast<u32x4*>(out + (size_t)row * ldo + vi * 8) = pack8(o);
    }
  }
}

// rope_kv_kernel fed by qkv partial slabs: qkv = bf16(sum_s P[s][t]) (the bf16 linear output), then
// the same rotate_half RoPE (HF bf16 op rounding) and paged-KV write. Rotated q goes to q_out
// (row stride ldq); k / v go to the cache only. grid = (T, HG): head groups split over blocks.

__global__ __launch_bounds__(NT) void rope_kv_partials_kernel(const float* __restrict__ P, int S, int T, int ldp,
                                                              bf16_t* q_out, int ldq,
                                                              const int* __restrict__ positions,
                                                              const float* __restrict__ cos_t,
                                                              const float* __restrict__ sin_t,
                                                              const int* __restrict__ slots, bf16_t* kc, bf16_t* vc,
                                                              int Hq, int Hkv, int D, int BS) {
  const int t = blockIdx.x, hg = blockIdx.y, ngroups = gridDim.y;
  const int pos = positions[t];
  const int slot = slots ? slots[t] : -1;
  const size_t slab = (size_t)T * ldp;
  const float* prow = P + (size_t)t * ldp;
  const int half = D >> 1;
  const int vpr = half >> 3;
  const float* ct = cos_t + (size_t)pos * half;
  const float* st = sin_t + (size_t)pos * half;
  const int nh = Hq + 2 * Hkv;
  for (int i = threadIdx.x + hg * NT; i < nh * vpr; i += NT * ngroups) {
    const int hd = i / vpr, v = i % vpr;
    float x1[8], x2[8];
    sum_partials8(prow + hd * D + v * 8, S, slab, x1);
    sum_partials8(prow + hd * D + half + v * 8, S, slab, x2);
    if (hd >= Hq + Hkv) {  // v head: straight to the cache
      if (slot >= 0) {
        bf16_t* dst = vc + (((size_t)(slot / BS) * Hkv + (hd - Hq - Hkv)) * BS + (slot % BS)) * D;
        *reinterpret_cast<u32x4*>(dst + v * 8) = pack8(x1);
        *reinterpret_cast<u32x4*>(dst + half + v * 8) = pack8(x2);
      }
      continue;
    }
    float o1[8], o2[8];
    rope8(x1, x2, ct + v * 8, st + v * 8, o1, o2);
    if (hd < Hq) {
      bf16_t* qp = q_out + (size_t)t * ldq + hd * D;
      *reinterpret_cast<u32x4*>(qp + v * 8) = pack8(o1);
      *reinterpret_cast<u32x4*>(qp + half + v * 8) = pack8(o2);
    } else if (slot >= 0) {
      bf16_t* dst = kc + (((size_t)(slot / BS) * Hkv + (hd - Hq)) * BS + (slot % BS)) * D;
      *reinterpret_cast<u32x4*>(dst + v * 8) = pack8(o1);
      *reinterpret_cast<u32x4*>(dst + half + v * 8) = pack8(o2);
    }
  }
}

}  // namespace

RAGK_API int ragk_rmsnorm(const void* x, int ldx, void* resid, int ldr, const void* w, void* out, int ldo, int rows,
                          int H, float eps, hipStream_t st) {
  if (rows <= 0) return 0;
  if (H % 8 || H > 8 * NT * 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(rows), dim3(NT), 0, st, (const bf16_t*)x, ldx, (bf16_t*)resid, ldr,
                     (const bf16_t*)w, (bf16_t*)out, ldo, H, eps);
  return (int)hipGetLastError();
}

RAGK_API int ragk_layernorm(const void* x, int ldx, const void* resid, int ldr, const void* g, const void* b,
                            void* out, int ldo, int rows, int H, float eps, hipStream_t st) {
  if (rows <= 0) return 0;
  if (H % 8 || H > 8 * NT * 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(layernorm_kernel, dim3(rows), dim3(NT), 0, st, (const bf16_t*)x, ldx, (const bf16_t*)resid,
                     ldr, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)out, ldo, H, eps);
  return (int)hipGetLastError();
}

RAGK_API int ragk_embed(const int* ids, const void* table, void* out, int T, int H, int vocab, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(NT), 0, st, const_cast<int*>(ids), (const bf16_t*)table,
                     (bf16_t*)out, H, vocab, (const int*)nullptr, (const int*)nullptr);
  return (int)hipGetLastError();
}

// Embedding gather whose token ids may come from the previous step's device-side sampler output:
// carry[t] >= 0 -> id = prev[carry[t]] (also stored to ids[t]); carry[t] < 0 -> ids[t].
RAGK_API int ragk_embed_carry(int* ids, const int* carry, const int* prev, const void* table, void* out, int T,
                              int H, int vocab, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 8 || !carry || !prev) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(NT), 0, st, ids, (const bf16_t*)table, (bf16_t*)out, H, vocab,
                     carry, prev);
  return (int)hipGetLastError();
}

RAGK_API int ragk_embed_ln(const int* ids, const int* pos_ids, const void* word, const void* pos, const void* type,
                           const void* g, const void* b, void* out, int T, int H, float eps, int do_ln,
                           hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 8 || H > 8 * NT * 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_ln_kernel, dim3(T), dim3(NT), 0, st, ids, pos_ids, (const bf16_t*)word,
                     (const bf16_t*)pos, (const bf16_t*)type, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)out, H,
                     eps, do_ln);
  return (int)hipGetLastError();
}

RAGK_API int ragk_rope_kv(void* qkv, int ld, const int* positions, const float* cos_t, const float* sin_t,
                          const int* slots, void* kc, void* vc, int T, int Hq, int Hkv, int D, int BS,
                          int apply_rope, hipStream_t st) {
  if (T <= 0) return 0;
  if (D % 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(NT), 0, st, (bf16_t*)qkv, ld, positions, cos_t, sin_t, slots,
                     (bf16_t*)kc, (bf16_t*)vc, Hq, Hkv, D, BS, apply_rope);
  return (int)hipGetLastError();
}

RAGK_API int ragk_pool_l2norm(const void* hidden, int ld, const int* cu, float* out, int B, int H, int mode,
                              int normalize, hipStream_t st) {
  if (B <= 0) return 0;
  if (H > 8 * NT) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pool_l2norm_kernel, dim3(B), dim3(NT), 0, st, (const bf16_t*)hidden, ld, cu, out, H, mode,
                     normalize);
  return (int)hipGetLastError();
}

RAGK_API int ragk_silu_mul(const void* x, int ldx, void* out, int ldo, int T, int I, hipStream_t st) {
  if (T <= 0) return 0;
  if (I % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(T), dim3(NT), 0, st, (const bf16_t*)x, ldx, (bf16_t*)out, ldo, I);
  return (int)hipGetLastError();
}

RAGK_API int ragk_gather_rows(const void* x, int ldx, const int* idx, void* out, int ldo, int n, int H,
                              hipStream_t st) {
  if (n <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(n), dim3(NT), 0, st, (const bf16_t*)x, ldx, idx, (bf16_t*)out, ldo, H);
  return (int)hipGetLastError();
}

RAGK_API int ragk_add_partials_rmsnorm(const float* P, int S, int M, void* h, int ldh, const void* w, void* out,
                                       int ldo, int H, float eps, hipStream_t st) {
  if (M <= 0) return 0;
  if (H % 8 || H > 8 * PNT * 2 || S < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(add_partials_rmsnorm_kernel, dim3(M), dim3(PNT), 0, st, P, S, M, (bf16_t*)h, ldh,
                     (const bf16_t*)w, (bf16_t*)out, ldo, H, eps);
  return (int)hipGetLastError();
}

// P: [S][T][ldp] fp32 qkv partials (ldp >= (Hq + 2 Hkv) * D); q_out: rotated q [T][ldq] bf16.
RAGK_API int ragk_rope_kv_partials(const float* P, int S, int T, int ldp, void* q_out, int ldq,
                                   const int* positions, const float* cos_t, const float* sin_t, const int* slots,
                                   void* kc, void* vc, int Hq, int Hkv, int D, int BS, hipStream_t st) {
  if (T <= 0) return 0;
  if (D % 16 || S < 1) return (int)hipErrorInvalidValue;
  // head groups per row: enough blocks to spread the slab reads over the CUs at decode batch sizes,
  // at least one wave of (head, 8-column) items per block
  const int items = (Hq + 2 * Hkv) * (D / 16);
  const int groups = std::max(1, std::min((items + 63) / 64, std::max(4, (512 + T - 1) / T)));
  hipLaunchKernelGGL(rope_kv_partials_kernel, dim3(T, groups), dim3(NT), 0, st, P, S, T, ldp, (bf16_t*)q_out,
                     ldq, positions, cos_t, sin_t, slots, (bf16_t*)kc, (bf16_t*)vc, Hq, Hkv, D, BS);
  return (int)hipGetLastError();
}
