// Per-CU vs chip-wide HBM stream limit (MI355X): the same 1 GiB LDS-DMA nt stream split over G workgroups
// of W waves (one or two per CU), each workgroup a contiguous region. If the aggregate rate stays with
// fewer workgroups, the chip's memory system is the limit; if it scales with G, a CU's own rate is.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int W>
__global__ __launch_bounds__(64 * W) void stream_kernel(const u32x4* __restrict__ src, size_t per_wg, unsigned long long* t) {
  __shared__ u32x4 lds[W][64 * 8];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const u32x4* p = src + (size_t)blockIdx.x * per_wg;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (size_t i = (size_t)wid * 64 * 8; i < per_wg; i += W * 64 * 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + i + 64 * u + lane),
                                       (__attribute__((address_space(3))) void*)&lds[wid][64 * u], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x] = t0;
    t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

int main() {
  const size_t total = 1ull << 30;
  u32x4* src;
  unsigned long long* t;
  if (hipMalloc(&src, total) || hipMalloc(&t, 16 * 2048) || hipMemset(src, 1, total)) return 1;
  std::vector<unsigned long long> h(2 * 2048);
  const int Gs[] = {256, 192, 128, 64, 512, 224, 448};
  for (int w = 0; w < 2; ++w)
    for (int G : Gs) {
      for (int rep = 0; rep < 3; ++rep) {
        const size_t per_wg = total / G / 16 / 512 * 512;
        if (w == 0) hipLaunchKernelGGL(stream_kernel<4>, dim3(G), dim3(256), 0, 0, src, per_wg, t);
        else hipLaunchKernelGGL(stream_kernel<8>, dim3(G), dim3(512), 0, 0, src, per_wg, t);
        if (hipDeviceSynchronize()) return 2;
        if (hipMemcpy(h.data(), t, 16 * G, hipMemcpyDeviceToHost)) return 3;
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int i = 0; i < G; ++i) {
          t0 = std::min(t0, h[2 * i]);
          t1 = std::max(t1, h[2 * i + 1]);
        }
        const double us = (t1 - t0) / 100.0, bytes = (double)per_wg * 16 * G;
        if (rep == 2)
          printf("G=%4d waves=%d: %.1f us, %.2f TB/s aggregate, %.1f GB/s per workgroup\n", G, w ? 8 : 4, us,
                 bytes / us / 1e6, bytes / G / us / 1e3);
      }
    }
  return 0;
}
