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
// One lane per pod (pods hold 1-3 containers): the lanes of a wave read
// consecutive runs of the container arrays (the CSR keeps a pod's containers contiguous),
// in batches whose loads are all issued before their sums.  HBM-bound: 16 B per pod of offsets (app + init), 16 B per
// container, 17 B per init container, 16 B per pod of overhead in, 16 B per pod out.
#include "kcc_internal.h"

namespace kcc {
namespace {

constexpr int POD_BATCH = 4;   // app containers loaded per round trip
constexpr int INIT_BATCH = 2;  // init containers loaded per round trip

// (Staging each workgroup's container ranges in LDS by coalesced loads first measured
// slower at C4 and was deleted: scripts/ab_pods.py 0.359 vs 0.347 ms; the per-lane loads
// already move only the algorithmic bytes, PMC 1.69 GB vs 1.72 GB.)
constexpr int POD_WG = 256;

// Clamp [lo, hi) into [0, n).
__device__ __forceinline__ void clamp_range(int64_t& lo, int64_t& hi, int64_t n) {
  lo = lo < 0 ? 0 : (lo > n ? n : lo);
  hi = hi < lo ? lo : (hi > n ? n : hi);
}

// One pod's request from loaders for its app / init containers (staged or global).
template <class AppAt, class InitAt>
__device__ __forceinline__ void pod_request(int64_t lo, int64_t hi, int64_t a, int64_t b,
                                            bool has_init, uint64_t oc, uint64_t om,
                                            AppAt app_at, InitAt init_at, uint64_t& out_c,
                                            uint64_t& out_m) {
  uint64_t ac = 0, am = 0;
  for (int64_t c = lo; c < hi; c += POD_BATCH) {
    uint64_t vc[POD_BATCH], vm[POD_BATCH];
#pragma unroll
    for (int u = 0; u < POD_BATCH; ++u) {
      vc[u] = 0;
      vm[u] = 0;
      if (c + u < hi) app_at(c + u, vc[u], vm[u]);
    }
#pragma unroll
    for (int u = 0; u < POD_BATCH; ++u) {
      ac += vc[u];
      am += vm[u];
    }
  }
  uint64_t sc = 0, sm = 0, ic = 0;
  int64_t im = INT64_MIN;
  if (has_init) {
    for (int64_t k0 = a; k0 < b; k0 += INIT_BATCH) {
      uint64_t rcv[INIT_BATCH], rmv[INIT_BATCH];
      bool rs[INIT_BATCH];
#pragma unroll
      for (int u = 0; u < INIT_BATCH; ++u) {
        rcv[u] = 0;
        rmv[u] = 0;
        rs[u] = false;
        if (k0 + u < b) init_at(k0 + u, rcv[u], rmv[u], rs[u]);
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
  out_c = (ac > ic ? ac : ic) + oc;
  out_m = ((int64_t)am > im ? am : (uint64_t)im) + om;
}

// One lane per pod: each lane walks its pod's app and init containers (CSR) from global
// memory, its loads batched (POD_BATCH / INIT_BATCH per round trip).
__global__ __launch_bounds__(POD_WG) void pod_requests_kernel(
    int64_t n_pods, int64_t n_cont, int64_t n_init, const int64_t* __restrict__ pod_ptr,
    const uint64_t* __restrict__ cpu_req, const int64_t* __restrict__ mem_req,
    const int64_t* __restrict__ init_ptr, const uint64_t* __restrict__ init_cpu,
    const int64_t* __restrict__ init_mem, const uint8_t* __restrict__ restartable,
    const uint64_t* __restrict__ ovh_cpu, const int64_t* __restrict__ ovh_mem,
    uint64_t* __restrict__ pod_cpu, int64_t* __restrict__ pod_mem) {
  const int64_t p0 = (int64_t)blockIdx.x * POD_WG;
  const int64_t p = p0 + threadIdx.x;
  const bool live = p < n_pods;
  const bool has_init = init_ptr != nullptr;
  // offsets clamped into the arrays: a malformed CSR gives wrong sums, never a fault
  int64_t lo = 0, hi = 0, a = 0, b = 0;
  uint64_t oc = 0, om = 0;
  if (live) {
    lo = pod_ptr[p];
    hi = pod_ptr[p + 1];
    clamp_range(lo, hi, n_cont);
    if (has_init) {
      a = init_ptr[p];
      b = init_ptr[p + 1];
      clamp_range(a, b, n_init);
    }
    oc = ovh_cpu ? ovh_cpu[p] : 0;
    om = ovh_mem ? (uint64_t)ovh_mem[p] : 0;
  }
  if (!live) return;
  uint64_t rc, rm;
  pod_request(
      lo, hi, a, b, has_init, oc, om,
      [&](int64_t c, uint64_t& vc, uint64_t& vm) {
        vc = cpu_req[c];
        vm = (uint64_t)mem_req[c];
      },
      [&](int64_t k, uint64_t& vc, uint64_t& vm, bool& rs) {
        vc = init_cpu[k];
        vm = (uint64_t)init_mem[k];
        rs = restartable ? restartable[k] != 0 : false;
      },
      rc, rm);
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
  const int64_t grid = (n_pods + POD_WG - 1) / POD_WG;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pod_requests_kernel, dim3((unsigned)grid), dim3(POD_WG), 0, s, n_pods, n_cont,
                     n_init, pod_ptr, cpu_req, mem_req, init_ptr, init_cpu, init_mem, restartable,
                     ovh_cpu, ovh_mem, pod_cpu, pod_mem);
  return hipGetLastError();
}

}  // namespace kcc
