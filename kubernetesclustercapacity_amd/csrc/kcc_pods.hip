// kcc_pods.hip — OPT-IN scheduler request model.
//
// NOT the reference's semantics: the reference sums the app containers of a node's
// pods (CC:276-294, kcc_reduce_requests).  This entry point gives the kube-scheduler's
// effective pod request instead — init containers (max with the app sum), sidecars
// (restartable init containers, which run for the pod's life) and pod overhead — per
// resource, in the same 64-bit wrapping domain as the rest of the engine (cpu uint64,
// memory int64):
//   app = sum of app containers; side = 0; init = identity of max
//   for each init container k, in order:
//     restartable: app += r_k; side += r_k; init = max(init, side)
//     otherwise:   init = max(init, r_k + side)
//   req(p) = max(app, init) + overhead(p)
// The per-node sums are then the ordinary segmented reduce (reduce_kernel) over the
// pods of each node, so used_cpu / used_mem feed kcc_fit unchanged.
//
// One lane per pod: pods hold 1-3 containers, so a lane's loop is short
// and the lanes of a wave read consecutive runs of the container arrays (the CSR keeps
// a pod's containers contiguous).  HBM-bound: 16 B per pod of offsets (app + init),
// 16 B per container, 16 B per pod of overhead in, 16 B per pod out.
#include "kcc_internal.h"

namespace kcc {
namespace {

constexpr int POD_BATCH = 4;   // app containers loaded per round trip
constexpr int INIT_BATCH = 2;  // init containers loaded per round trip

__global__ __launch_bounds__(256) void pod_requests_kernel(
    int64_t n_pods, int64_t n_cont, int64_t n_init, const int64_t* __restrict__ pod_ptr,
    const uint64_t* __restrict__ cpu_req, const int64_t* __restrict__ mem_req,
    const int64_t* __restrict__ init_ptr, const uint64_t* __restrict__ init_cpu,
    const int64_t* __restrict__ init_mem, const uint8_t* __restrict__ restartable,
    const uint64_t* __restrict__ ovh_cpu, const int64_t* __restrict__ ovh_mem,
    uint64_t* __restrict__ pod_cpu, int64_t* __restrict__ pod_mem) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pods) return;
  // offsets clamped into the arrays: a malformed CSR gives wrong sums, never a fault
  int64_t lo = pod_ptr[p], hi = pod_ptr[p + 1];
  lo = lo < 0 ? 0 : (lo > n_cont ? n_cont : lo);
  hi = hi < lo ? lo : (hi > n_cont ? n_cont : hi);
  // the overhead loads go out first (independent of everything else), then the
  // containers in batches whose loads are all issued before their sums (a pod's loop
  // is 1-3 iterations: one memory round trip per batch, not per container)
  const uint64_t oc = ovh_cpu ? ovh_cpu[p] : 0;
  const uint64_t om = ovh_mem ? (uint64_t)ovh_mem[p] : 0;
  uint64_t ac = 0, am = 0;
  for (int64_t c = lo; c < hi; c += POD_BATCH) {
    uint64_t vc[POD_BATCH], vm[POD_BATCH];
#pragma unroll
    for (int u = 0; u < POD_BATCH; ++u) {
      const bool in = c + u < hi;
      vc[u] = in ? cpu_req[c + u] : 0;
      vm[u] = in ? (uint64_t)mem_req[c + u] : 0;
    }
#pragma unroll
    for (int u = 0; u < POD_BATCH; ++u) {
      ac += vc[u];
      am += vm[u];
    }
  }
  uint64_t sc = 0, sm = 0, ic = 0;
  int64_t im = INT64_MIN;
  if (init_ptr) {
    int64_t a = init_ptr[p], b = init_ptr[p + 1];
    a = a < 0 ? 0 : (a > n_init ? n_init : a);
    b = b < a ? a : (b > n_init ? n_init : b);
    for (int64_t k0 = a; k0 < b; k0 += INIT_BATCH) {
      uint64_t rcv[INIT_BATCH], rmv[INIT_BATCH];
      bool rs[INIT_BATCH];
#pragma unroll
      for (int u = 0; u < INIT_BATCH; ++u) {
        const bool in = k0 + u < b;
        rcv[u] = in ? init_cpu[k0 + u] : 0;
        rmv[u] = in ? (uint64_t)init_mem[k0 + u] : 0;
        rs[u] = in && restartable ? restartable[k0 + u] != 0 : false;
      }
#pragma unroll
      for (int u = 0; u < INIT_BATCH; ++u) {
        if (k0 + u >= b) break;
        const uint64_t rc = rcv[u], rm = rmv[u];
        if (rs[u]) {  // a sidecar: runs for the pod's life
          ac += rc;
          am += rm;
          sc += rc;
          sm += rm;
          ic = sc > ic ? sc : ic;
          im = (int64_t)sm > im ? (int64_t)sm : im;
        } else {
          const uint64_t tc = rc + sc;
          const int64_t tm = (int64_t)(rm + sm);
          ic = tc > ic ? tc : ic;
          im = tm > im ? tm : im;
        }
      }
    }
  }
  const uint64_t rc = (ac > ic ? ac : ic) + oc;
  const uint64_t rm = ((int64_t)am > im ? am : (uint64_t)im) + om;
  pod_cpu[p] = rc;
  pod_mem[p] = (int64_t)rm;
}

}  // namespace

hipError_t launch_pod_requests(int64_t n_pods, int64_t n_cont, int64_t n_init,
                               const int64_t* pod_ptr, const uint64_t* cpu_req,
                               const int64_t* mem_req, const int64_t* init_ptr,
                               const uint64_t* init_cpu, const int64_t* init_mem,
                               const uint8_t* restartable, const uint64_t* ovh_cpu,
                               const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem,
                               hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  const int64_t grid = (n_pods + 255) / 256;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pod_requests_kernel, dim3((unsigned)grid), dim3(256), 0, s, n_pods, n_cont,
                     n_init, pod_ptr, cpu_req, mem_req, init_ptr, init_cpu, init_mem, restartable,
                     ovh_cpu, ovh_mem, pod_cpu, pod_mem);
  return hipGetLastError();
}

}  // namespace kcc
