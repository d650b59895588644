// Diagnostic only (not part of libkcc): streaming-read ceilings for the reduce's access
// pattern on gfx950.  Each kernel reads two u64 arrays of n elements and writes one
// u64 per wave (so the reads cannot be elided).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// (a) contiguous: lane l reads 16 B at 16*l of a 1 KiB slab per instruction
// (b) strided:    lane l reads 32 B at 32*l as two 16-B loads (the reduce's pattern)
template <int MODE, int UNROLL>
__global__ __launch_bounds__(256) void probe(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                             int64_t n, int64_t per_wave, uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t base = w * per_wave;
  if (base >= n) return;
  const int64_t len = n - base < per_wave ? n - base : per_wave;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + base), (short)0, (int)(len * 8), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + base), (short)0, (int)(len * 8), 0x00020000);
  uint64_t acc = 0;
  for (int64_t t = 0; t < len; t += 256 * UNROLL) {
    u64x2 v[2 * UNROLL][2];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int so = (int)((t + 256 * u) * 8);
      if (MODE == 0) {
        v[2 * u][0] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, lane * 16, so, 0));
        v[2 * u + 1][0] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, lane * 16 + 1024, so, 0));
        v[2 * u][1] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rb, lane * 16, so, 0));
        v[2 * u + 1][1] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rb, lane * 16 + 1024, so, 0));
      } else {
        v[2 * u][0] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, lane * 32, so, 0));
        v[2 * u + 1][0] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, lane * 32 + 16, so, 0));
        v[2 * u][1] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rb, lane * 32, so, 0));
        v[2 * u + 1][1] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rb, lane * 32 + 16, so, 0));
      }
    }
#pragma unroll
    for (int u = 0; u < 2 * UNROLL; ++u) acc += v[u][0].x + v[u][0].y + v[u][1].x + v[u][1].y;
  }
  if (acc == 0x1234567ull) out[w] = acc;
}

extern "C" int probe_launch(int mode, int unroll, const void* a, const void* b, int64_t n,
                            int64_t per_wave, void* out, void* stream) {
  const int64_t waves = (n + per_wave - 1) / per_wave;
  dim3 g((unsigned)((waves + 3) / 4)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t* A = (const uint64_t*)a;
  const uint64_t* B = (const uint64_t*)b;
  uint64_t* O = (uint64_t*)out;
  if (mode == 0 && unroll == 1) hipLaunchKernelGGL((probe<0, 1>), g, blk, 0, s, A, B, n, per_wave, O);
  else if (mode == 0 && unroll == 2) hipLaunchKernelGGL((probe<0, 2>), g, blk, 0, s, A, B, n, per_wave, O);
  else if (mode == 0 && unroll == 4) hipLaunchKernelGGL((probe<0, 4>), g, blk, 0, s, A, B, n, per_wave, O);
  else if (mode == 1 && unroll == 1) hipLaunchKernelGGL((probe<1, 1>), g, blk, 0, s, A, B, n, per_wave, O);
  else if (mode == 1 && unroll == 2) hipLaunchKernelGGL((probe<1, 2>), g, blk, 0, s, A, B, n, per_wave, O);
  else if (mode == 1 && unroll == 4) hipLaunchKernelGGL((probe<1, 4>), g, blk, 0, s, A, B, n, per_wave, O);
  else return -1;
  return (int)hipGetLastError();
}
