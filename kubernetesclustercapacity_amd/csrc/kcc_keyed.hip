// kcc_keyed.hip — per-node request sums from containers in LIST order (SURVEY.md §8f
// row 1, the lister side of (a)).
//
// The reference lists the pods of one node at a time (CC:232-253, one List per node) and
// sums their containers' requests (CC:290-293).  A cluster-wide `Pods("").List` returns
// the pods in namespace/name order instead, each container tagged with the row of its
// node (key).  kcc_reduce_requests_keyed sums such an unsorted stream without sorting it:
// uint64/int64 wrapping addition is commutative and associative, so per-key atomic adds
// give the reference's sums bit for bit in any order.  kcc_count_by_key counts the pods
// per key (len(pods), CC:106/135).
//
// Byte work, HBM- and atomic-bound: each lane takes KY_IPL consecutive
// containers (one 16-B key load, two 16-B loads per value array), merges runs of equal
// keys in registers (a pod's containers are consecutive in the list), and issues one
// 64-bit no-return atomic per array and run.  Keys < 0 or >= n_keys are skipped (pods
// whose node is not a listed row).
#include "kcc_internal.h"

namespace kcc {
namespace {

constexpr int KY_THREADS = 256;
constexpr int KY_IPL = 4;                             // containers per lane
constexpr int KY_BLOCK = KY_THREADS * KY_IPL;         // containers per workgroup

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void add_u64(uint64_t* p, uint64_t v) {
  __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NA>  // 2: requests; 4: requests and limits
__global__ __launch_bounds__(KY_THREADS) void reduce_keyed_kernel(
    int64_t n, int64_t n_keys, const int32_t* __restrict__ key, const uint64_t* __restrict__ a0,
    const uint64_t* __restrict__ a1, const uint64_t* __restrict__ a2, const uint64_t* __restrict__ a3,
    uint64_t* __restrict__ o0, uint64_t* __restrict__ o1, uint64_t* __restrict__ o2,
    uint64_t* __restrict__ o3) {
  const uint64_t* in[4] = {a0, a1, a2, a3};
  uint64_t* out[4] = {o0, o1, o2, o3};
  const int64_t c = ((int64_t)blockIdx.x * KY_THREADS + threadIdx.x) * KY_IPL;
  if (c >= n) return;
  int32_t k[KY_IPL];
  uint64_t v[NA][KY_IPL];
  if (c + KY_IPL <= n) {  // whole quad: vector loads (the arrays are 16-byte aligned)
    const i32x4 kk = *reinterpret_cast<const i32x4*>(key + c);
    k[0] = kk.x;
    k[1] = kk.y;
    k[2] = kk.z;
    k[3] = kk.w;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const u64x2 lo = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c));
      const u64x2 hi = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c + 2));
      v[a][0] = lo.x;
      v[a][1] = lo.y;
      v[a][2] = hi.x;
      v[a][3] = hi.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < KY_IPL; ++j) {
      const bool in_range = c + j < n;
      k[j] = in_range ? key[c + j] : -1;
#pragma unroll
      for (int a = 0; a < NA; ++a) v[a][j] = in_range ? in[a][c + j] : 0;
    }
  }
  // runs of equal keys: container j folds into the run that ends at j + 1 when the key
  // repeats, else the run's sums are added to the key's totals
  uint64_t run[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) run[a] = v[a][0];
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) {
    const bool last = j + 1 == KY_IPL || k[j + 1] != k[j];
    if (last) {
      if (k[j] >= 0 && (int64_t)k[j] < n_keys) {
#pragma unroll
        for (int a = 0; a < NA; ++a) add_u64(out[a] + k[j], run[a]);
      }
      if (j + 1 < KY_IPL) {
#pragma unroll
        for (int a = 0; a < NA; ++a) run[a] = v[a][j + 1];
      }
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a) run[a] += v[a][j + 1];
    }
  }
}

__global__ __launch_bounds__(KY_THREADS) void count_keyed_kernel(int64_t n, int64_t n_keys,
                                                                 const int32_t* __restrict__ key,
                                                                 uint64_t* __restrict__ count) {
  const int64_t c = ((int64_t)blockIdx.x * KY_THREADS + threadIdx.x) * KY_IPL;
  if (c >= n) return;
  int32_t k[KY_IPL];
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) k[j] = c + j < n ? key[c + j] : -1;
  uint64_t run = 1;
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) {
    if (j + 1 == KY_IPL || k[j + 1] != k[j]) {
      if (k[j] >= 0 && (int64_t)k[j] < n_keys) add_u64(count + k[j], run);
      run = 1;
    } else {
      ++run;
    }
  }
}

}  // namespace

hipError_t launch_reduce_keyed(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* cpu,
                               const int64_t* mem, const uint64_t* cpul, const int64_t* meml,
                               uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                               int64_t* lim_mem, hipStream_t s) {
  if (n_keys > 0) {  // the sums start from zero (CC:257-260)
    hipError_t e = hipMemsetAsync(used_cpu, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess) e = hipMemsetAsync(used_mem, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess && cpul) e = hipMemsetAsync(lim_cpu, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess && cpul) e = hipMemsetAsync(lim_mem, 0, 8 * (size_t)n_keys, s);
    if (e != hipSuccess) return e;
  }
  if (n <= 0 || n_keys <= 0) return hipSuccess;
  const int64_t grid = (n + KY_BLOCK - 1) / KY_BLOCK;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  if (cpul)
    hipLaunchKernelGGL(reduce_keyed_kernel<4>, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n,
                       n_keys, key, cpu, reinterpret_cast<const uint64_t*>(mem), cpul,
                       reinterpret_cast<const uint64_t*>(meml), used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                       reinterpret_cast<uint64_t*>(lim_mem));
  else
    hipLaunchKernelGGL(reduce_keyed_kernel<2>, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n,
                       n_keys, key, cpu, reinterpret_cast<const uint64_t*>(mem), nullptr, nullptr,
                       used_cpu, reinterpret_cast<uint64_t*>(used_mem), nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_count_keyed(int64_t n_keys, int64_t n, const int32_t* key, int64_t* count,
                              hipStream_t s) {
  if (n_keys > 0) {
    hipError_t e = hipMemsetAsync(count, 0, 8 * (size_t)n_keys, s);
    if (e != hipSuccess) return e;
  }
  if (n <= 0 || n_keys <= 0) return hipSuccess;
  const int64_t grid = (n + KY_BLOCK - 1) / KY_BLOCK;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(count_keyed_kernel, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n, n_keys,
                     key, reinterpret_cast<uint64_t*>(count));
  return hipGetLastError();
}

}  // namespace kcc
