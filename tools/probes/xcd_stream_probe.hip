// Per-XCD HBM stream rate probe (MI355X): G workgroups (one per CU), each streams its own contiguous
// region with 16-B non-temporal loads (plain or LDS-DMA), stamping s_memrealtime at start and end.
// Prints per-XCD (dispatch order w % 8) median stream time. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// MODE 0: sequential (each wave 8 KB contiguous per step, the 4 waves adjacent: 32 KB per step);
// MODE 1: the decode engine's slot order: 16 rows of ROWB bytes (a weight matrix row), 1 KiB from each
// row per slot (K-chunk kc of all 16 rows), then the next K chunk; 16-row groups one after another.
// MODE 2: the stream GEMM's stage order (gemm_stream.hip, 64-row tiles): each 1 KiB LDS-DMA piece is 8 rows
// x 128 B, a stage = 64 rows x 128 B (one 64-element K-step), consecutive stages advance 128 B along the rows;
// per wave 4 stages (8 pieces) in flight. MODE 3: as 2 with 256 B per row per stage (4 rows x 256 B per piece).
template <bool DMA, int MODE>
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ src, size_t per_wg, unsigned long long* t,
                                                     unsigned* sink, int rowb) {
  __shared__ u32x4 lds[4][64 * 8];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const u32x4* p = src + (size_t)blockIdx.x * per_wg;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 acc = {0u, 0u, 0u, 0u};
  if constexpr (MODE == 1) {
    // per slot 16 rows x 1 KiB = 16 x 64 vectors; wave w handles rows 4w..4w+3 (4 KiB), 2 slots per step
    const size_t rowv = rowb / 16, kcs = rowv / 64, groups = per_wg / (16 * rowv);
    for (size_t g = 0; g < groups; ++g)
      for (size_t kc = 0; kc < kcs; kc += 2) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = 4 * wid + (u & 3);
          const size_t off = (g * 16 + r) * rowv + (kc + (u >> 2)) * 64 + lane;
          if constexpr (DMA)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + off),
                                             (__attribute__((address_space(3))) void*)&lds[wid][64 * u], 16, 0, 2);
          else
            acc ^= __builtin_nontemporal_load(p + off);
        }
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
  }
  if constexpr (MODE == 2 || MODE == 3) {
    // rows of rowb bytes, 64-row tiles, stage = 64 rows x SEG bytes; piece q of a stage = 64 lanes x 16 B
    constexpr int SEG = MODE == 2 ? 128 : 256;        // bytes per row per stage
    constexpr int RPP = 1024 / SEG;                   // rows per 1 KiB piece
    constexpr int LPR = SEG / 16;                     // lanes per row
    const size_t rowv = rowb / 16, tiles = per_wg / (64 * rowv), steps = rowb / SEG;
    for (size_t tl = 0; tl < tiles; ++tl)
      for (size_t k = 0; k < steps; k += 8 / (64 / RPP / 4)) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {  // 8 pieces per wave: (64 / RPP) / 4 pieces per wave per stage
          constexpr int PPW = 64 / RPP / 4;
          const int st = u / PPW, q = wid * PPW + (u % PPW);
          const int r = q * RPP + lane / LPR;
          const size_t off = (tl * 64 + r) * rowv + (k + st) * (SEG / 16) + (lane % LPR);
          if (k + st < steps) {
            if constexpr (DMA)
              __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + off),
                                               (__attribute__((address_space(3))) void*)&lds[wid][64 * u], 16, 0, 2);
            else
              acc ^= __builtin_nontemporal_load(p + off);
          }
        }
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
  }
  for (size_t i = (size_t)wid * 64 * 8; MODE == 0 && i < per_wg; i += 4 * 64 * 8) {
    if constexpr (DMA) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + i + 64 * u + lane),
                                         (__attribute__((address_space(3))) void*)&lds[wid][64 * u], 16, 0, 2);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= __builtin_nontemporal_load(p + i + 64 * u + lane);
    }
  }
  if (acc.x == 0x12345678u) sink[0] = acc.y;
  __syncthreads();
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x] = t0;
    t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

int main() {
  int dev = 0, G = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, dev);
  const size_t per_wg_bytes = 4u << 20;  // 4 MiB per workgroup, 1 GiB total at G = 256
  const size_t per_wg = per_wg_bytes / 16;
  u32x4* src;
  unsigned long long* t;
  unsigned* sink;
  if (hipMalloc(&src, per_wg_bytes * G) || hipMalloc(&t, 16 * G) || hipMalloc(&sink, 4)) return 1;
  hipMemset(src, 1, per_wg_bytes * G);
  std::vector<unsigned long long> h(2 * G);
  const int rowbs[5] = {0, 8192, 28672, 8192, 8192};
  for (int pat = 0; pat < 5; ++pat)
    for (int mode = 0; mode < 2; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        const int rb = rowbs[pat];
        if (pat == 0)
          hipLaunchKernelGGL((mode ? stream_kernel<true, 0> : stream_kernel<false, 0>), dim3(G), dim3(256), 0, 0, src,
                             per_wg, t, sink, rb);
        else if (pat == 3)
          hipLaunchKernelGGL((mode ? stream_kernel<true, 2> : stream_kernel<false, 2>), dim3(G), dim3(256), 0, 0, src,
                             per_wg, t, sink, rb);
        else if (pat == 4)
          hipLaunchKernelGGL((mode ? stream_kernel<true, 3> : stream_kernel<false, 3>), dim3(G), dim3(256), 0, 0, src,
                             per_wg, t, sink, rb);
        else
          hipLaunchKernelGGL((mode ? stream_kernel<true, 1> : stream_kernel<false, 1>), dim3(G), dim3(256), 0, 0, src,
                             per_wg, t, sink, rb);
        if (hipDeviceSynchronize()) return 2;
        hipMemcpy(h.data(), t, 16 * G, hipMemcpyDeviceToHost);
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int w = 0; w < G; ++w) {
          t0 = std::min(t0, h[2 * w]);
          t1 = std::max(t1, h[2 * w + 1]);
        }
        // bytes actually read in the slot pattern: whole 16-row groups
        const size_t rowv = rb / 16;
        const size_t bytes = pat == 0 ? per_wg_bytes
                             : (pat >= 3 ? (per_wg / (64 * rowv)) * 64 * rowv * 16 : (per_wg / (16 * rowv)) * 16 * rowv * 16);
        const char* names[5] = {"sequential   ", "slots row 8K ", "slots row 28K", "stages 128 B ", "stages 256 B "};
        printf("%s %s rep %d: total %.1f us (%.2f TB/s); per-XCD median us:", names[pat], mode ? "lds-dma" : "plain  ",
               rep, (t1 - t0) / 100.0, bytes * G / ((t1 - t0) / 100.0) / 1e6);
        for (int x = 0; x < 8; ++x) {
          std::vector<double> d;
          for (int w = x; w < G; w += 8) d.push_back((h[2 * w + 1] - h[2 * w]) / 100.0);
          std::sort(d.begin(), d.end());
          printf(" %.1f", d[d.size() / 2]);
        }
        printf("\n");
      }
    }
  return 0;
}
