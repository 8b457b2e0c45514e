// Does a weight / KV stream run slower when its address translations are cold? (MI355X)
// A 1 GiB stream (256 workgroups x 4 MiB, LDS-DMA nt, the stream GEMM's access pattern) is timed cold, warm,
// and again after a large "evict" stream touched EVICT_GB of other memory (as a decode step does: ~38 GB of
// weights and KV between two reads of the same layer), for a hipMalloc buffer and for a
// hipExtMallocWithFlags(hipDeviceMallocContiguous) buffer. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ src, size_t per_wg, unsigned long long* t) {
  __shared__ u32x4 lds[4][64 * 8];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const u32x4* p = src + (size_t)blockIdx.x * per_wg;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (size_t i = (size_t)wid * 64 * 8; i < per_wg; i += 4 * 64 * 8) {
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

static double run(const u32x4* src, size_t per_wg, unsigned long long* t, std::vector<unsigned long long>& h, int G) {
  hipLaunchKernelGGL(stream_kernel, dim3(G), dim3(256), 0, 0, src, per_wg, t);
  if (hipDeviceSynchronize()) exit(2);
  if (hipMemcpy(h.data(), t, 16 * G, hipMemcpyDeviceToHost)) exit(3);
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int w = 0; w < G; ++w) {
    t0 = std::min(t0, h[2 * w]);
    t1 = std::max(t1, h[2 * w + 1]);
  }
  return (t1 - t0) / 100.0;  // us
}

int main(int argc, char** argv) {
  int dev = 0, G = 0;
  if (hipGetDevice(&dev) || hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, dev)) return 1;
  const double evict_gb = argc > 1 ? atof(argv[1]) : 24.0;
  const size_t per_wg_bytes = 4u << 20, bytes = per_wg_bytes * G, per_wg = per_wg_bytes / 16;
  unsigned long long* t;
  if (hipMalloc(&t, 16 * G)) return 1;
  std::vector<unsigned long long> h(2 * G);
  // the evict region: evict_gb of other memory, streamed in 1 GiB launches
  const size_t ev_chunks = (size_t)(evict_gb);
  std::vector<u32x4*> ev(ev_chunks, nullptr);
  for (auto& e : ev) {
    if (hipMalloc(&e, bytes)) return 4;
    if (hipMemset(e, 2, bytes)) return 4;
  }
  for (int kind = 0; kind < 2; ++kind) {
    u32x4* src = nullptr;
    if (kind == 0 ? hipMalloc(&src, bytes) : hipExtMallocWithFlags((void**)&src, bytes, hipDeviceMallocContiguous)) {
      printf("%s allocation failed\n", kind ? "contiguous" : "hipMalloc");
      continue;
    }
    if (hipMemset(src, 1, bytes) || hipDeviceSynchronize()) return 5;
    const char* name = kind ? "contiguous" : "hipMalloc ";
    for (int round = 0; round < 2; ++round) {
      for (auto e : ev) run(e, per_wg, t, h, G);  // touch the evict region
      const double cold = run(src, per_wg, t, h, G);
      const double warm = run(src, per_wg, t, h, G);
      const double warm2 = run(src, per_wg, t, h, G);
      printf("%s round %d, after %.0f GB of other streams: cold %.1f us (%.2f TB/s), warm %.1f / %.1f us (%.2f TB/s)\n",
             name, round, evict_gb, cold, bytes / cold / 1e6, warm, warm2, bytes / warm2 / 1e6);
    }
    hipFree(src);
  }
  return 0;
}
