// kcc_rows.hip — per-node rows of one spec for the verbose report.
//
// The reference prints, for every node row, its "Max replicas" (CC:137) — the row's
// contribution q(i) to the total, CC:119-136.  kcc_fit_rows returns q(i) for all rows of
// one spec in one launch (the fit kernels only keep per-spec totals), with Go's exact
// 64-bit semantics: uint64 CPU division reinterpreted as int, int64 memory division
// (truncating, MinInt64 / -1 == MinInt64), signed min, the pod-slot clamp
// allocatablePods - len(pods), and a per-row flag where Go would panic (divide by zero).
// One thread per row; 64-bit integer division is a software sequence on the VALU, but
// there is one per row and per resource.
#include "kcc_internal.h"

namespace kcc {
namespace {

__global__ __launch_bounds__(256) void fit_rows_kernel(
    int64_t n, const uint64_t* __restrict__ alloc_cpu, const int64_t* __restrict__ alloc_mem,
    const int64_t* __restrict__ alloc_pods, const int64_t* __restrict__ pod_count,
    const uint64_t* __restrict__ used_cpu, const int64_t* __restrict__ used_mem, uint64_t c,
    int64_t m, int64_t* __restrict__ q_out, int32_t* __restrict__ err_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ac = alloc_cpu[i], uc = used_cpu[i];
  const int64_t am = alloc_mem[i], um = used_mem[i];
  const int64_t P = alloc_pods[i], pc = pod_count[i];
  bool z = false;
  int64_t qc = 0, qm = 0;
  if (ac > uc) {  // CC:119-124 (uint64 compare and division, int() reinterprets)
    if (c == 0) z = true;
    else qc = (int64_t)((ac - uc) / c);
  }
  if (am > um) {  // CC:125-130 (int64, the difference wraps)
    const int64_t fm = (int64_t)((uint64_t)am - (uint64_t)um);
    if (m == 0) z = true;
    else if (m == -1) qm = (int64_t)(0ull - (uint64_t)fm);  // MinInt64 / -1 == MinInt64
    else qm = fm / m;
  }
  int64_t q = qc <= qm ? qc : qm;                            // findMin, CC:133, CC:159-164
  if (q >= P) q = (int64_t)((uint64_t)P - (uint64_t)pc);     // CC:134-136
  q_out[i] = z ? 0 : q;
  err_out[i] = z ? 1 : 0;
}

}  // namespace

hipError_t launch_fit_rows(int64_t n, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
                           const int64_t* alloc_pods, const int64_t* pod_count,
                           const uint64_t* used_cpu, const int64_t* used_mem, uint64_t spec_cpu,
                           int64_t spec_mem, int64_t* q, int32_t* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t grid = (n + 255) / 256;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fit_rows_kernel, dim3((unsigned)grid), dim3(256), 0, s, n, alloc_cpu,
                     alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, spec_cpu, spec_mem, q,
                     err);
  return hipGetLastError();
}

}  // namespace kcc
