// Diagnostic: workgroup dispatch rate on gfx950.  Each workgroup stamps its start
// (s_memrealtime, 100 MHz) and spins `work` iterations; the host reports the spread of
// start times per (block size, LDS bytes, grid) configuration.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

template <int LDS>
__global__ void stamp(uint64_t* t, int work, uint32_t* sink) {
  __shared__ uint32_t l[LDS / 4 > 0 ? LDS / 4 : 1];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x;
  for (int i = 0; i < work; ++i) a = a * 1664525u + 1013904223u;
  if (LDS > 0) {
    l[threadIdx.x % (LDS / 4)] = a;
    __syncthreads();
    a += l[(threadIdx.x + 1) % (LDS / 4)];
  }
  if (threadIdx.x == 0) t[blockIdx.x] = t0;
  if (a == 0x12345u) sink[0] = a;
}

__global__ void stamp_dyn(uint64_t* t, int work, uint32_t* sink, int words) {
  extern __shared__ uint32_t dl[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x;
  for (int i = 0; i < work; ++i) a = a * 1664525u + 1013904223u;
  dl[threadIdx.x % words] = a;
  __syncthreads();
  a += dl[(threadIdx.x + 1) % words];
  if (threadIdx.x == 0) t[blockIdx.x] = t0;
  if (a == 0x12345u) sink[0] = a;
}

void run_dyn(int block, int grid, int work, int bytes) {
  uint64_t* t;
  uint32_t* sink;
  (void)hipMalloc(&t, 8 * grid);
  (void)hipMalloc(&sink, 4);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(stamp_dyn, dim3(grid), dim3(block), bytes, 0, t, work, sink, bytes / 4);
    (void)hipDeviceSynchronize();
  }
  std::vector<uint64_t> h(grid);
  (void)hipMemcpy(h.data(), t, 8 * grid, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("DYN block %4d lds %6d grid %6d work %6d: start spread %8.2f us (p50 %8.2f)\n", block, bytes,
         grid, work, (h[grid - 1] - h[0]) / 100.0, (h[grid / 2] - h[0]) / 100.0);
  (void)hipFree(t);
  (void)hipFree(sink);
}

template <int LDS>
void run(int block, int grid, int work) {
  uint64_t* t;
  uint32_t* sink;
  hipMalloc(&t, 8 * grid);
  hipMalloc(&sink, 4);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(stamp<LDS>, dim3(grid), dim3(block), 0, 0, t, work, sink);
    hipDeviceSynchronize();
  }
  std::vector<uint64_t> h(grid);
  hipMemcpy(h.data(), t, 8 * grid, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("block %4d lds %6d grid %6d work %6d: start spread %8.2f us (p50 %8.2f)\n", block, LDS,
         grid, work, (h[grid - 1] - h[0]) / 100.0, (h[grid / 2] - h[0]) / 100.0);
  hipFree(t);
  hipFree(sink);
}

int main() {
  for (int bytes : {32768, 49152, 57344, 65536}) run_dyn(1024, 512, 20000, bytes);
  run_dyn(256, 1024, 20000, 57344);
  run<0>(256, 1536, 20000);
  run<0>(256, 1280, 20000);
  run<16384>(256, 1024, 20000);
  run<16384>(256, 1280, 20000);
  run<8192>(256, 1536, 20000);
  for (int work : {20000}) {
    run<0>(64, 4096, work);
    run<0>(256, 1024, work);
    run<0>(256, 4096, work);
    run<0>(1024, 512, work);
    run<0>(1024, 256, work);
    run<16384>(256, 1536, work);
    run<57344>(1024, 512, work);
    run<57344>(256, 512, work);
  }
  return 0;
}
