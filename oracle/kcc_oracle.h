/*
 * kcc_oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * It is the checker, never the product: libkcc.so does not link or call it.
 *
 * Reference: AshutoshNirkhe/KubernetesClusterCapacity
 *   CC = src/KubeAPI/ClusterCapacity.go, BF = src/bytefmt/bytes.go
 * Parity pinning: the reference publishes no tests, fixtures or golden vectors
 *  and Go is absent from this image, so this restatement is
 * pinned by hand-derived known-answer tests (tests/test_oracle_kat.py, K1-K8 of
 * SURVEY §8c) and cross-checked against an independent Python big-int
 * restatement (oracle/pyoracle.py).
 */
#ifndef KCC_ORACLE_H
#define KCC_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* CC:255-299 — per-node sums over a CSR container list (uint64/int64 wrap). */
void kcco_reduce_requests(int64_t n_nodes, const int64_t* node_ptr,
                          const uint64_t* cpu_req, const int64_t* mem_req,
                          const uint64_t* cpu_lim, const int64_t* mem_lim,
                          uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                          int64_t* lim_mem);

/* CC:119-136 for one (node row, spec): the node's contribution maxReplicas.
 * *div0 is set to 1 when Go would panic (integer divide by zero). */
int64_t kcco_fit_one(uint64_t alloc_cpu, int64_t alloc_mem, int64_t alloc_pods,
                     int64_t pod_count, uint64_t used_cpu, int64_t used_mem,
                     uint64_t spec_cpu, int64_t spec_mem, int* div0);

/* CC:101-140 for S specs; totals[s]=0 and spec_err[s]=1 where Go would panic.
 * n_threads > 1 splits specs over pthreads (CPU baseline timing only). */
void kcco_fit(int64_t n_nodes, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
              const int64_t* alloc_pods, const int64_t* pod_count,
              const uint64_t* used_cpu, const int64_t* used_mem, int64_t n_specs,
              const uint64_t* spec_cpu, const int64_t* spec_mem, int64_t* totals,
              int32_t* spec_err, int n_threads);

/* CC:159-164 */
int64_t kcco_find_min(int64_t x, int64_t y);

/* CC:301-319 — returns the value; *ok = 0 when Atoi failed (Go prints an error and
 * returns 0). */
uint64_t kcco_convert_cpu_to_milis(const char* s, int* ok);

/* BF:75-105 — returns 0 on success, -1 on error (value then 0). */
int kcco_to_bytes(const char* s, int64_t* out);

/* Batch forms of the two conversions over Arrow-style packed strings (string i =
 * bytes[offsets[i], offsets[i+1])); status[i] = 1 ok, 0 error.  n_threads > 1 splits
 * the strings over pthreads (CPU baseline timing only). */
void kcco_parse_cpu_millis(int64_t n, const char* bytes, const int64_t* offsets, uint64_t* out,
                           int8_t* status, int n_threads);
void kcco_parse_bytes(int64_t n, const char* bytes, const int64_t* offsets, int64_t* out,
                      int8_t* status, int n_threads);

/* SURVEY §8f row 4 — OPT-IN scheduler request model, NOT the reference's semantics
 * (the reference sums app containers only, CC:276-294).  Restates the published
 * kube-scheduler pod request (k8s.io/kubernetes pkg/api/v1/resource PodRequests, the
 * sidecar-aware form of k8s >= 1.28; that dependency is absent here, so parity is
 * unpinned beyond hand-derived cases), per resource, over 64-bit wrapping sums:
 *   app = sum of app containers; side = 0; init = 0
 *   for each init container k in order:
 *     restartable: app += r_k; side += r_k; init = max(init, side)
 *     otherwise:   init = max(init, r_k + side)
 *   req(p) = max(app, init) + overhead(p)
 * cpu unsigned (uint64 max), memory signed (int64 max).  init_ptr / init arrays /
 * restartable / overhead may be NULL (none / false / 0). */
void kcco_pod_requests(int64_t n_pods, const int64_t* pod_ptr, const uint64_t* cpu_req,
                       const int64_t* mem_req, const int64_t* init_ptr,
                       const uint64_t* init_cpu, const int64_t* init_mem,
                       const uint8_t* restartable, const uint64_t* ovh_cpu,
                       const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem);

#ifdef __cplusplus
}
#endif
#endif
