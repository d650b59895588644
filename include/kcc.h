/*
 * kcc.h — C-ABI of the MI355X capacity engine (libkcc.so).
 *
 * This is the drop-in boundary for the hot path of
 * AshutoshNirkhe/KubernetesClusterCapacity, src/KubeAPI/ClusterCapacity.go (CC):
 *
 *   (a) the per-container request summation inside getPodCPUMemoryRequestsLimits
 *       (CC:255-299, the adds at CC:290-293)           -> kcc_reduce_requests*
 *   (b) the per-node fit + pod-slot clamp + total in main's node loop
 *       (CC:101-140, findMin CC:159-164)               -> kcc_fit*
 *
 * generalised from the reference's single pod spec to a batch of S what-if specs.
 * The Go host keeps flags, client-go listing and printing; a cgo package binds
 * these symbols.  Every result is bit-exact to the Go integer
 * arithmetic (uint64/int64 wrap, Go `int` = int64 on amd64, signed min, clamp quirk).
 *
 * Conventions
 *   - Return 0 (KCC_OK) on success, a negative KCC_E* code otherwise; the message
 *     is available from kcc_last_error(ctx) until the next call on ctx.
 *   - Host-array entry points (no suffix) are synchronous: they copy inputs to the
 *     device, run, copy results back and never retain a caller pointer.
 *   - *_async entry points take DEVICE pointers and a hipStream_t (as void*, NULL =
 *     the null stream) and only enqueue work: they never synchronise, and allocate
 *     only when the context workspace must grow — call kcc_reserve first and they
 *     can be captured into a hipGraph and replayed (no launch depends on host-side
 *     state that a replay would freeze: the reduce's look-back records are left free by
 *     every launch, the exchange's epoch is a device word).  Container arrays must be
 *     16-byte aligned.
 *   - Device faults: the reduce's look-back and node-prep waits, the keyed gather's
 *     part wait and the exchange's flag waits are bounded; one that gives up (never on
 *     a healthy device) sets a sticky fault word of the device.  While it is set every
 *     finalize marks every spec KCC_SPEC_FAULT (totals 0) and the synchronous entry
 *     points (the keyed ones included) return KCC_EFAULT; kcc_clear_faults resets it
 *     and every device counter a give-up can leave set.  The fault also travels with the data: a partial produced on a
 *     faulted device (kcc_*_partial_async, kcc_fit_run_async) carries a fault mark in
 *     its per-spec counts, so every rank that sums it — over the p2p exchange, an RCCL
 *     or any other all-reduce, the in-library device fold — marks every spec
 *     KCC_SPEC_FAULT too, without reading the faulted device's words.
 *     kcc_reduce_requests_async alone has no per-spec output: check kcc_reduce_faults
 *     after synchronising.
 *   - A context is not thread-safe; every entry calls hipSetDevice(ctx device), so
 *     Go OS-thread migration between cgo calls is harmless.
 *   - There is no CPU backend: without a usable gfx950 device kcc_create fails.
 */
#ifndef KCC_H
#define KCC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5): kcc_fit_mskip_groups removed; partial[S..2S) carries the device fault mark
 * (a count >= 2^48, see kcc_fit_partial_async).  1: the first release. */
#define KCC_ABI_VERSION 2

enum {
  KCC_OK = 0,
  KCC_EINVAL = -1,   /* bad argument (null pointer, negative size, malformed CSR) */
  KCC_ENOMEM = -2,   /* device allocation failed                                  */
  KCC_EHIP = -3,     /* HIP runtime error                                         */
  KCC_ENODEV = -4,   /* no usable device                                          */
  KCC_ERCCL = -5,    /* RCCL error (multi-GPU contexts)                           */
  KCC_EFAULT = -6    /* a bounded device wait gave up: results invalid (see above) */
};

/* spec_err values of the fit entry points */
enum {
  KCC_SPEC_OK = 0,
  KCC_SPEC_DIVZERO = 1, /* Go would panic with an integer divide by zero; total 0    */
  KCC_SPEC_FAULT = 2    /* the device faulted (kcc_clear_faults); total 0, not valid */
};

typedef struct kcc_ctx kcc_ctx;

/* Library / ABI version (KCC_ABI_VERSION). */
int kcc_abi_version(void);
/* Build flavour: "release" for the product library; an experiment build (csrc/Makefile
 * `variant`, its own .so) returns "variant" plus the knobs it was compiled with. */
const char* kcc_build_info(void);

/* Create a context on `n_gpus` devices starting at `first_device`.
 * n_gpus == 1: one device.  n_gpus > 1: nodes are sharded in contiguous ranges
 * over devices first_device .. first_device+n_gpus-1 and the per-spec totals are
 * combined with an RCCL int64 all-reduce (replaces nothing in the reference: the
 * reference is single-threaded, CC:105).  n_gpus <= 0 is KCC_EINVAL. */
int kcc_create(kcc_ctx** out, int first_device, int n_gpus);
void kcc_destroy(kcc_ctx* ctx);
const char* kcc_last_error(const kcc_ctx* ctx);
/* Thread-local message of the last failed kcc_create (ctx did not exist yet). */
const char* kcc_create_error(void);

/* In-library all-reduce check (contexts of n_gpus > 1, host-array entry points): the
 * context's FIRST all-reduce is verified against the host's sum of the devices' partials
 * (KCC_ERCCL on a mismatch); later calls are not, unless every_call != 0 (then every call
 * pays two device-to-host copies and stream syncs per device).  Default 0. */
int kcc_set_allreduce_verify(kcc_ctx* ctx, int every_call);

/* Pre-size the device workspace used by the *_async entry points (device 0 of ctx). */
int kcc_reserve(kcc_ctx* ctx, int64_t max_nodes, int64_t max_containers, int64_t max_specs);

/* ---------------------------------------------------------------------------
 * (a) Segmented request reduction.  Replaces the accumulation at CC:290-293:
 *       cpuRequestsMiliTotal     += cpuRequestsMili     (uint64, wraps)
 *       cpuLimitsMiliTotal       += cpuLimitsMili       (uint64, wraps)
 *       memoryRequestsBytesTotal += memoryRequestsBytes (int64,  wraps)
 *       memoryLimitsBytesTotal   += memoryLimitsBytes   (int64,  wraps)
 *     over every container of every non-terminated pod of a node.
 *   Containers are grouped by node in CSR form: node i owns containers
 *   [node_ptr[i], node_ptr[i+1]); node_ptr[0] == 0, non-decreasing,
 *   node_ptr[n_nodes] == n_containers.  Empty nodes get 0 sums.
 *   At most 2^28 - 1 nodes per device (per call, or per shard for a multi-GPU ctx).
 *   cpu_lim/mem_lim may both be NULL (then lim_cpu/lim_mem are ignored): the limit
 *   sums are only printed by the reference (CC:110, CC:115-117).
 * ------------------------------------------------------------------------- */
int kcc_reduce_requests(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                        const int64_t* node_ptr, const uint64_t* cpu_req,
                        const int64_t* mem_req, const uint64_t* cpu_lim,
                        const int64_t* mem_lim, uint64_t* used_cpu, int64_t* used_mem,
                        uint64_t* lim_cpu, int64_t* lim_mem);

int kcc_reduce_requests_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                              const int64_t* d_node_ptr, const uint64_t* d_cpu_req,
                              const int64_t* d_mem_req, const uint64_t* d_cpu_lim,
                              const int64_t* d_mem_lim, uint64_t* d_used_cpu,
                              int64_t* d_used_mem, uint64_t* d_lim_cpu,
                              int64_t* d_lim_mem, void* stream);

/* ---------------------------------------------------------------------------
 * (b) Fit.  Replaces main's node loop CC:105-140 for S specs at once:
 *   for every node row i (zero rows for unhealthy nodes included, CC:221-226):
 *     qc = alloc_cpu[i] <= used_cpu[i] ? 0 : int((alloc_cpu[i]-used_cpu[i]) / spec_cpu[s])   CC:119-124
 *     qm = alloc_mem[i] <= used_mem[i] ? 0 :     (alloc_mem[i]-used_mem[i]) / spec_mem[s]    CC:125-130
 *     q  = findMin(qc, qm)                                                                   CC:133
 *     if q >= alloc_pods[i] { q = alloc_pods[i] - pod_count[i] }                             CC:134-136
 *     totals[s] += q                                                                         CC:138
 *   spec_err[s] = KCC_SPEC_DIVZERO (1) iff the Go code would panic with an integer divide
 *   by zero (spec_cpu[s] == 0 reached on a row with free CPU, or spec_mem[s] == 0 on a
 *   row with free memory); totals[s] is then 0.  KCC_SPEC_FAULT (2): a device fault, see
 *   the conventions above.  pod_count = len(pods) (CC:106, CC:135).
 *   The verdict (CC:144) is totals[s] >= replicas[s], left to the caller.
 *   At most 2^26 - 1 specs per call.
 * ------------------------------------------------------------------------- */
int kcc_fit(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* alloc_cpu,
            const int64_t* alloc_mem, const int64_t* alloc_pods,
            const int64_t* pod_count, const uint64_t* used_cpu, const int64_t* used_mem,
            int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
            int64_t* totals, int32_t* spec_err);

/* Fused (a)+(b): containers -> used sums -> fit, one device round trip. */
int kcc_capacity(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                 const int64_t* node_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
                 const uint64_t* alloc_cpu, const int64_t* alloc_mem,
                 const int64_t* alloc_pods, const int64_t* pod_count, int64_t n_specs,
                 const uint64_t* spec_cpu, const int64_t* spec_mem, int64_t* totals,
                 int32_t* spec_err);

/* Device-level fit, split so that a node-sharded caller can all-reduce in between:
 *   kcc_fit_partial_async: partial[0..S)  = wrapping Σ over this call's nodes of q(i,s)
 *                          partial[S..2S) = number of divide-by-zero rows (< 2^48), or
 *                          on a faulted device that count plus one or more fault marks
 *                          of 2^48 (a count >= 2^48 after any sum over shards means a
 *                          faulted shard; a host-side finalize must test it BEFORE
 *                          count > 0 -> DIVZERO; kcc_fit_finalize -> KCC_SPEC_FAULT)
 *                          (both in an internal spec order; zeroed by this call)
 *   <optional all-reduce(sum, int64) of partial[0..2S) over node shards>
 *   kcc_fit_finalize_async: totals[s], spec_err[s] in caller order.
 * All ranks of a sharded run must pass the same specs.  `d_partial` holds 2*S int64. */
int kcc_fit_partial_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                          const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                          const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                          const int64_t* d_used_mem, int64_t n_specs,
                          const uint64_t* d_spec_cpu, const int64_t* d_spec_mem,
                          int64_t* d_partial, void* stream);
int kcc_fit_finalize_async(kcc_ctx* ctx, int64_t n_specs, const int64_t* d_partial,
                           int64_t* d_totals, int32_t* d_spec_err, void* stream);
/* kcc_fit_partial_async == kcc_fit_prepare_async + kcc_fit_run_async:
 *   prepare: zero d_partial, partition the specs (fast-path specs first) and build
 *            the per-node free-capacity records in the context workspace;
 *   run:     the nodes x specs fit kernel alone (what a profiler should attribute
 *            to the fit), accumulating into d_partial.
 * run must follow prepare on the same stream with the same sizes. */
int kcc_fit_prepare_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                          const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                          const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                          const int64_t* d_used_mem, int64_t n_specs,
                          const uint64_t* d_spec_cpu, const int64_t* d_spec_mem,
                          int64_t* d_partial, void* stream);
int kcc_fit_run_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_specs, int64_t* d_partial,
                      void* stream);

/* Convenience: partial + finalize on one device. */
int kcc_fit_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                  const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                  const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                  const int64_t* d_used_mem, int64_t n_specs, const uint64_t* d_spec_cpu,
                  const int64_t* d_spec_mem, int64_t* d_totals, int32_t* d_spec_err,
                  void* stream);

/* ---------------------------------------------------------------------------
 * Pipelined (a)+(b) on one device: reduce + fit partial of the whole hot path in one
 * call, d_partial as kcc_fit_partial_async (follow with an optional all-reduce and
 * kcc_fit_finalize_async).  n_chunks > 1 cuts the nodes into that many contiguous
 * ranges (fewer when chunks would be small) and runs the reduce of range k on a
 * library-owned side stream while `stream` fits range k-1; 0 = library default (1:
 * the overlap measured slower on MI355X).  h_node_ptr is a HOST copy
 * of the CSR offsets in d_node_ptr (used only to place the chunk boundaries; NULL =
 * one chunk).  The
 * per-node request sums land in d_used_cpu / d_used_mem (CC:290-293).  Everything is
 * ordered after the work already queued on `stream`, and `stream` waits for the side
 * stream before the call's last kernel: capturable into a hipGraph.
 * ------------------------------------------------------------------------- */
int kcc_capacity_partial_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                               const int64_t* h_node_ptr, const int64_t* d_node_ptr,
                               const uint64_t* d_cpu_req, const int64_t* d_mem_req,
                               const uint64_t* d_alloc_cpu, const int64_t* d_alloc_mem,
                               const int64_t* d_alloc_pods, const int64_t* d_pod_count,
                               uint64_t* d_used_cpu, int64_t* d_used_mem, int64_t n_specs,
                               const uint64_t* d_spec_cpu, const int64_t* d_spec_mem,
                               int64_t* d_partial, int n_chunks, void* stream);
/* The whole step on one device without a cross-GPU exchange: kcc_capacity_partial_async
 * (one chunk, the partial in a library buffer) followed by the finalize, which rides in
 * the clamp correction's launch (its last workgroup to finish writes d_totals / d_spec_err):
 * the same results as partial + kcc_fit_finalize_async, one launch fewer
 * (ClusterCapacity.go:101-140 for a batch of specs, all on the device). */
int kcc_capacity_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                       const int64_t* h_node_ptr, const int64_t* d_node_ptr,
                       const uint64_t* d_cpu_req, const int64_t* d_mem_req,
                       const uint64_t* d_alloc_cpu, const int64_t* d_alloc_mem,
                       const int64_t* d_alloc_pods, const int64_t* d_pod_count,
                       uint64_t* d_used_cpu, int64_t* d_used_mem, int64_t n_specs,
                       const uint64_t* d_spec_cpu, const int64_t* d_spec_mem, int64_t* d_totals,
                       int32_t* d_spec_err, void* stream);

/* ---------------------------------------------------------------------------
 * Node sharding.  Nodes are independent and each per-spec total is a
 * wrapping int64 sum, so a cluster splits into contiguous node ranges whose partial
 * vectors (kcc_fit_partial_async / kcc_capacity_partial_async) add up to the whole.
 *
 * kcc_set_node_shards: the host-array entry points (kcc_fit, kcc_capacity) cut the
 *   nodes into max(n_shards, devices) contiguous ranges (balanced by node count),
 *   dealt round-robin over the context's devices; a device's shards run one after the
 *   other and their partials are summed on it before the RCCL all-reduce over devices.
 *   0 (default) = one shard per device.  Same results for every shard count; more
 *   shards than devices rehearse a multi-GPU split on fewer GPUs.
 *
 * One process per GPU (the Go host as one process per device, or torchrun): every
 *   rank owns one node range and a single-device context; rank 0 creates an id with
 *   kcc_comm_unique_id and hands it to the other ranks (any channel: the bytes are
 *   opaque), every rank calls kcc_comm_init (collective: blocks until all joined), and
 *   each step runs kcc_capacity_partial_async -> kcc_allreduce_partial_async ->
 *   kcc_fit_finalize_async on one stream: an RCCL all-reduce (sum, int64) of the 2*S
 *   partial vector over xGMI, the only exchange.  Every rank must pass the same specs.
 * ------------------------------------------------------------------------- */
#define KCC_COMM_ID_BYTES 128
int kcc_set_node_shards(kcc_ctx* ctx, int n_shards);
int kcc_comm_unique_id(uint8_t* id /* [KCC_COMM_ID_BYTES] */);
int kcc_comm_init(kcc_ctx* ctx, const uint8_t* id, int n_ranks, int rank);
int kcc_allreduce_partial_async(kcc_ctx* ctx, int64_t n_specs, int64_t* d_partial, void* stream);

/* One-shot exchange over xGMI peer memory: the MI355X-native replacement for
 * kcc_allreduce_partial_async + kcc_fit_finalize_async when each rank is one process on
 * its own GPU (<= 8 ranks, a 2*S int64 payload: latency-bound, so one push over the
 * full mesh beats a ring).  Setup, once: kcc_p2p_export allocates this rank's mailbox
 * (2 parities x n_ranks x (2 * max_specs) int64 + flags) in fine-grained, uncached device
 * memory (peers write it while this GPU polls it) and returns its IPC handle;
 * every rank's handle travels to every rank (any channel: the bytes are opaque);
 * kcc_p2p_open maps the peers' mailboxes.  Each step: kcc_exchange_finalize_async (one
 * kernel on the caller's stream, after kcc_capacity_partial_async) pushes this rank's
 * partial into every mailbox, waits for every peer's push of the same step, sums and
 * finalizes totals / spec_err exactly as the all-reduce + finalize do.  Every rank must
 * call it the same number of times with the same specs.  A wait for a peer that never
 * pushes gives up after seconds and is counted (kcc_p2p_faults): that launch and every
 * finalize after it mark every spec KCC_SPEC_FAULT (see the conventions above); tests
 * and the bench assert 0.  Replaces RCCL only where its
 * ncclAllReduce(partial) stood (ClusterCapacity.go:138, the total over nodes). */
#define KCC_P2P_HANDLE_BYTES 64
#define KCC_P2P_MAX_SPECS (1 << 20)
int kcc_p2p_export(kcc_ctx* ctx, int n_ranks, int64_t max_specs,
                   uint8_t* handle /* [KCC_P2P_HANDLE_BYTES] */);
int kcc_p2p_open(kcc_ctx* ctx, int rank, const uint8_t* handles /* [n_ranks][64] */);
int kcc_exchange_finalize_async(kcc_ctx* ctx, int64_t n_specs, const int64_t* d_partial,
                                int64_t* d_totals, int32_t* d_spec_err, void* stream);
int kcc_p2p_faults(kcc_ctx* ctx, int64_t* faults);

/* Per-launch timing of kcc_capacity_partial_async (HIP events recorded on the stream
 * each kernel runs on): enable (1) / disable (0) resets the sums; read synchronises
 * and returns the summed durations and launch counts of the reduces (mark + reduce,
 * one per chunk) and of the fit kernel (one per chunk). */
int kcc_profile_enable(kcc_ctx* ctx, int on);
int kcc_profile_read(kcc_ctx* ctx, double* reduce_ms, int64_t* reduce_launches, double* fit_ms,
                     int64_t* fit_launches);

/* Look-back waits of the segmented reduce that gave up (summed over the context's
 * devices since the last kcc_clear_faults; synchronises).  A reduce launch assembles a
 * node cut by wave ranges from pieces the other waves publish; a wait that never sees
 * its piece (not expected on a healthy device) is counted here instead of hanging, and
 * the affected node's sums are then wrong.  Tests and the bench assert 0. */
int kcc_reduce_faults(kcc_ctx* ctx, int64_t* faults);
/* Reset the context's fault words and the reduce's look-back records (synchronises).
 * After an exchange fault (kcc_p2p_faults > 0) a late peer push may still land in the
 * mailbox: re-create the mailboxes (a new context) before exchanging again. */
int kcc_clear_faults(kcc_ctx* ctx);

/* The fit streams only the node rows that can add to its fast sum (free CPU, free
 * memory and allocatable pods > 0, within the fast bounds): every other row contributes
 * exactly 0 there (x = findMin(qc, qm) = 0; P <= 0 rows are applied by the clamp
 * correction; rows outside the bounds take the exact path), so the totals are the same
 * bit for bit.  kcc_set_fit_dense(ctx, 1) streams every row instead (diagnostic / A-B).
 * kcc_fit_stream_rows: node rows (padded to groups of 8) the last fit streamed, summed
 * over its node chunks (synchronises the device). */
int kcc_set_fit_dense(kcc_ctx* ctx, int dense);
/* Where the pod-slot clamp (CC:134-135, x >= allocatable pods ? allocatable - pod count : x)
 * is applied by kcc_capacity_partial_async / kcc_capacity_async: by the clamp correction
 * (a dominance count over the specs, one launch of its own; the fit's loop stays at 3 VALU
 * per node and spec wave) or inside the fit (5 VALU, no clamp launch, no clamp tables:
 * cheaper on small shards).  mode -1 (default): inside the fit when node rows x specs <=
 * 1.1e9 and specs <= 4096; 0: never; 1: whenever specs <= 4096 (one node chunk, not dense).
 * The totals are the same bit for bit either way. */
int kcc_set_clamp_in_fit(kcc_ctx* ctx, int mode);
/* 1 when the last kcc_capacity_partial_async / kcc_capacity_async of the context applied
 * the clamp inside the fit (its VALU accounting per node x 64-spec wave: 5 for class-A
 * specs and 6.5 for class B, against 3 and 4.5 with the clamp correction). */
int kcc_clamp_in_fit_used(kcc_ctx* ctx, int* used);
int kcc_fit_stream_rows(kcc_ctx* ctx, int64_t* streamed);

/* Fraction of (node, spec) pairs of the last kcc_fit* call that took the exact
 * 64-bit path instead of the saturating fast path (diagnostic; host-computed from
 * the class counters the fit kernel keeps).  -1 if unknown. */
double kcc_last_slow_fraction(const kcc_ctx* ctx);

/* Same counter for the last kcc_fit_partial_async / kcc_fit_async on device 0 of
 * ctx: (node, spec) pairs that took the exact path, and all pairs.  Synchronises
 * the device. */
int kcc_fit_slow_pairs(kcc_ctx* ctx, int64_t* slow_pairs, int64_t* pairs);

/* ---------------------------------------------------------------------------
 * Quantity strings -> int64 (the caller side of (a)).
 * Strings are packed Arrow-style: string i = bytes[offsets[i], offsets[i+1]),
 * offsets non-decreasing, 0 <= offsets[i] <= n_bytes (n + 1 offsets).  Per string,
 * out[i] is the reference's value and status[i] one of KCC_PARSE_*; the call itself
 * returns KCC_OK unless an argument is invalid (the reference prints per-string errors
 * and carries on with 0, CC:315-316, CC:203-206).
 *
 *   kcc_parse_cpu_millis: convertCPUToMilis (CC:301-319) — one trailing 'm' means
 *     millicores, else cores x 1000 (Go int multiply, wraps); strconv.Atoi failure ->
 *     KCC_PARSE_ERR, value 0.  Replaces the per-container calls at CC:280 and CC:283
 *     (on cpuRequests.String() / cpuLimits.String()) and the node's at CC:197.
 *   kcc_parse_bytes: bytefmt.ToBytes (BF:75-105) — base-2 multiples for K/M/G/T with
 *     the reference's accepted spellings (KI and MI but not GI/TI), ParseFloat > 0,
 *     int64(float64 * multiple) with amd64 overflow (0x8000000000000000).  Replaces
 *     the node allocatable-memory conversion at CC:203 (and the flag parse, CC:78-81).
 *     KCC_PARSE_UNSUPPORTED marks the rare inputs outside the device's exact
 *     ParseFloat domain (more than 19 significant digits below 10^19, or a value at
 *     the float64 overflow / underflow edge); never a silently different value.
 * The *_async forms take device pointers (bytes 4-byte aligned) and a stream.
 * ------------------------------------------------------------------------- */
enum {
  KCC_PARSE_OK = 1,
  KCC_PARSE_ERR = 0,          /* the reference reports an error and uses 0 */
  KCC_PARSE_UNSUPPORTED = -1, /* outside the exact device domain; value 0  */
  KCC_PARSE_BADOFF = -2       /* malformed offsets (async forms only)      */
};
int kcc_parse_cpu_millis(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                         const int64_t* offsets, uint64_t* out, int8_t* status);
int kcc_parse_bytes(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                    const int64_t* offsets, int64_t* out, int8_t* status);
/* resource.Quantity.Value() of ParseQuantity(s) (CC:285-286, the containers' memory
 * requests): [+-] digits [. digits] + "", Ki..Ei, n u m k M G T P E or e<int> suffix;
 * rounded up away from zero, binary (Ki..Ei) magnitudes capped at 2^63 - 1.  Restated
 * from k8s.io/apimachinery's published algorithm, which is not vendored in the reference
 * (version unpinned): parity unpinned.  KCC_PARSE_ERR for strings
 * ParseQuantity rejects; KCC_PARSE_UNSUPPORTED (value 0) for a decimal amount beyond
 * 2^63 - 1 (k8s wraps it), a negative amount off ParseQuantity's int64 fast path and
 * binary-suffixed fractions with more than 19 significant digits. */
int kcc_parse_quantity(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                       const int64_t* offsets, int64_t* out, int8_t* status);
int kcc_parse_quantity_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                             const int64_t* d_offsets, int64_t* d_out, int8_t* d_status,
                             void* stream);
int kcc_parse_cpu_millis_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                               const int64_t* d_offsets, uint64_t* d_out, int8_t* d_status,
                               void* stream);
int kcc_parse_bytes_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                          const int64_t* d_offsets, int64_t* d_out, int8_t* d_status,
                          void* stream);

/* ---------------------------------------------------------------------------
 * Per-node sums from containers in LIST order.  A cluster-wide
 * Pods("").List (one call instead of the per-node List of CC:236) returns pods in
 * namespace/name order; key[i] is the row of container i's node (<0 or >= n_keys:
 * skipped).  Same sums as kcc_reduce_requests on the grouped (CSR) containers, bit for
 * bit (wrapping addition does not depend on order).  kcc_count_by_key gives
 * len(pods) per row (CC:106, CC:135) from the pods' keys.  Arrays 16-byte aligned.
 * ------------------------------------------------------------------------- */
int kcc_reduce_requests_keyed(kcc_ctx* ctx, int64_t n_keys, int64_t n_containers,
                              const int32_t* key, const uint64_t* cpu_req, const int64_t* mem_req,
                              const uint64_t* cpu_lim, const int64_t* mem_lim,
                              uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                              int64_t* lim_mem);
int kcc_reduce_requests_keyed_async(kcc_ctx* ctx, int64_t n_keys, int64_t n_containers,
                                    const int32_t* d_key, const uint64_t* d_cpu_req,
                                    const int64_t* d_mem_req, const uint64_t* d_cpu_lim,
                                    const int64_t* d_mem_lim, uint64_t* d_used_cpu,
                                    int64_t* d_used_mem, uint64_t* d_lim_cpu, int64_t* d_lim_mem,
                                    void* stream);
int kcc_count_by_key(kcc_ctx* ctx, int64_t n_keys, int64_t n, const int32_t* key, int64_t* count);
int kcc_count_by_key_async(kcc_ctx* ctx, int64_t n_keys, int64_t n, const int32_t* d_key,
                           int64_t* d_count, void* stream);

/* ---------------------------------------------------------------------------
 * Per-row "Max replicas" of one spec (the verbose report's
 * CC:137 line for every node row, CC:119-136): q[i] = row i's contribution to the total,
 * row_err[i] = 1 where Go would panic with an integer divide by zero at that row (q[i]
 * is then 0; the reference stops at the first such row).
 * ------------------------------------------------------------------------- */
int kcc_fit_rows(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* alloc_cpu,
                 const int64_t* alloc_mem, const int64_t* alloc_pods, const int64_t* pod_count,
                 const uint64_t* used_cpu, const int64_t* used_mem, uint64_t spec_cpu,
                 int64_t spec_mem, int64_t* q, int32_t* row_err);

/* ---------------------------------------------------------------------------
 * OPT-IN scheduler request model — explicitly NOT the
 * reference's semantics: the reference sums only the app containers of a node's pods
 * (CC:276-294, kcc_reduce_requests above; that stays the default).  This gives the
 * kube-scheduler's effective pod request instead (k8s pkg/api/v1/resource PodRequests,
 * sidecar-aware form; that dependency is absent here, parity unpinned beyond the
 * hand-derived cases of tests/test_pods.py), per resource, in the engine's 64-bit
 * wrapping domain (cpu uint64 with unsigned max, memory int64 with signed max):
 *   app = sum of the pod's app containers; side = 0; init = identity of max
 *   for each init container k of the pod, in order:
 *     restartable[k] (a sidecar): app += r_k; side += r_k; init = max(init, side)
 *     otherwise:                  init = max(init, r_k + side)
 *   req(p) = max(app, init) + overhead(p)
 * pod_ptr[P+1] / init_ptr[P+1]: CSR offsets of each pod's app / init containers.
 * init_ptr (with init_cpu, init_mem), restartable and the overhead pair are nullable
 * (absent = no init containers / none restartable / no overhead).
 * kcc_pod_requests: req(p) per pod.  kcc_reduce_requests_pods: also sums the pods of each
 * node (node_pod_ptr[N+1], pods grouped by node) into used_cpu / used_mem, the inputs
 * kcc_fit takes.  The *_async forms take device pointers (offsets must be in range;
 * the kernel clamps them, so a malformed CSR gives wrong sums, never a fault).
 * ------------------------------------------------------------------------- */
int kcc_pod_requests(kcc_ctx* ctx, int64_t n_pods, int64_t n_containers, int64_t n_init,
                     const int64_t* pod_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
                     const int64_t* init_ptr, const uint64_t* init_cpu, const int64_t* init_mem,
                     const uint8_t* restartable, const uint64_t* ovh_cpu,
                     const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem);
int kcc_pod_requests_async(kcc_ctx* ctx, int64_t n_pods, int64_t n_containers, int64_t n_init,
                           const int64_t* d_pod_ptr, const uint64_t* d_cpu_req,
                           const int64_t* d_mem_req, const int64_t* d_init_ptr,
                           const uint64_t* d_init_cpu, const int64_t* d_init_mem,
                           const uint8_t* d_restartable, const uint64_t* d_ovh_cpu,
                           const int64_t* d_ovh_mem, uint64_t* d_pod_cpu, int64_t* d_pod_mem,
                           void* stream);
int kcc_reduce_requests_pods(kcc_ctx* ctx, int64_t n_nodes, int64_t n_pods,
                             int64_t n_containers, int64_t n_init, const int64_t* node_pod_ptr,
                             const int64_t* pod_ptr, const uint64_t* cpu_req,
                             const int64_t* mem_req, const int64_t* init_ptr,
                             const uint64_t* init_cpu, const int64_t* init_mem,
                             const uint8_t* restartable, const uint64_t* ovh_cpu,
                             const int64_t* ovh_mem, uint64_t* used_cpu, int64_t* used_mem);

#ifdef __cplusplus
}
#endif
#endif /* KCC_H */
