// kcc_abi.cpp — the C-ABI of libkcc.so (include/kcc.h): contexts, device
// workspaces, host<->device staging, node sharding over devices and the RCCL
// all-reduce of per-spec totals.  No CPU compute path: every result comes from
// the gfx950 kernels in kcc_kernels.hip.
#include "kcc.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kcc_internal.h"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

hipError_t ensure(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e == hipSuccess) b.bytes = bytes;
  return e;
}

// Fine-grained, uncached device memory (the p2p mailbox): peers write it over xGMI while
// this device's kernel polls it, and a line of ordinary (coarse-grained) memory may be
// served stale from this device's L2 — coarse-grained memory is only coherent with other
// devices at synchronisation points.  Uncached loads and stores go to memory.
hipError_t ensure_uncached(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  hipError_t e = hipExtMallocWithFlags(&b.p, bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) b.bytes = bytes;
  return e;
}

template <class T>
T* as(DevBuf& b) {
  return static_cast<T*>(b.p);
}

// Timing of the pipelined entry point (kcc_profile_*): event pairs recorded around each
// reduce (side stream) and each fit launch (caller stream), read back on demand.
struct ProfPair {
  hipEvent_t a, b;
  int kind;  // 0 reduce (mark + reduce), 1 fit
};

struct Dev {
  int device = 0;
  hipStream_t stream = nullptr;
  // pipelined capacity (kcc_capacity_partial_async): node chunk k's reduce runs on `side`
  // while the caller's stream fits chunk k-1
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_red[kcc::FIT_MAX_CHUNKS] = {};
  bool prof_on = false;
  std::vector<ProfPair> prof_pending;
  std::vector<hipEvent_t> prof_free;
  double prof_ms[2] = {0.0, 0.0};
  int64_t prof_n[2] = {0, 0};
  // workspace of the *_async entry points
  DevBuf fast_a, fast_b, slow, slow_list, srec, sperm, counters;
  // the reduce's per-wave tail records (look-back): zeroed when allocated, and every
  // launch leaves their tags 0 (each record is cleared by the wave that consumes it)
  DevBuf red_tail;
  // the device's fault words (kcc::FAULT_*): reduce look-back / exchange flag waits that
  // gave up; sticky until kcc_clear_faults
  DevBuf faults;
  DevBuf rank_arrive;  // spec_rank's per-query-block arrival counters (zero between calls)
  DevBuf fit_q;          // the fit's per-column work queues (zero between launches)
  bool fitq_dirty = true;
  // spec setup + clamp correction (kcc::ClampWork)
  DevBuf c_rank, c_bcnt, c_cs, c_ms, c_mrc, c_crm, c_dperm;
  DevBuf c_C, c_H2, c_H3, c_Crow, c_rec, c_dir;
  // the table copies C / H2 / H3 not known to be all zero (fresh allocation or an
  // interrupted call)
  bool clamp_dirty = true;
  int64_t last_pairs = 0;  // node x spec pairs of the last fit_prepare on this device
  int64_t c_stride = 0;    // cells per copy of the clamp table C
  int64_t h_stride = 0;    // cells per copy of the clamp tables H2 / H3
  int64_t d_stride = 0;    // words per pass of the binned records' directory
  bool fit_dense = false;  // kcc_set_fit_dense: stream every node row through the fit
  int clamp_in_fit = -1;   // kcc_set_clamp_in_fit: -1 by size (clamp_in_fit_auto), 0 never, 1 always
  bool last_nc = false;    // the last capacity call applied the clamp in the fit
  DevBuf fast_cl;          // the clamp in the fit: each streamed row's clamp value
  int stream_chunks = 0;   // node chunks of the last fit prepare (their stream counters)
  int64_t prep_nodes = -1, prep_specs = -1;  // sizes the workspace was last prepared for
  // staging of the host-array entry points
  DevBuf ptr, cpu, mem, cpul, meml, used_cpu, used_mem, lim_cpu, lim_mem;
  DevBuf alloc_cpu, alloc_mem, alloc_pods, pod_count, spec_cpu, spec_mem, partial, totals, err;
  DevBuf p_bytes, p_off, p_out, p_st;  // kcc_parse_* staging
  DevBuf k_key;                        // kcc_*_keyed staging
  DevBuf kb_counts, kb_tot, kb_sr, kb_sv;  // kcc::KeyedWork (bucketed keyed reduce)
  DevBuf kb_part, kb_arrive;               // one-sweep gather: part rows, arrivals (zeroed)
  DevBuf kb_esc_n, kb_esc_row, kb_esc_cpu, kb_esc_mem;
  // kcc_pod_requests / kcc_reduce_requests_pods staging (app containers in cpu / mem)
  DevBuf q_ptr, q_iptr, q_icpu, q_imem, q_rst, q_ocpu, q_omem, q_pcpu, q_pmem;
  // one-shot exchange over xGMI peer memory (kcc_p2p_*): this rank's mailbox (exported),
  // the push arrival counter (u32 word 0) and the last pushed epoch (u64 word 1, advanced
  // by the kernel); the peers' mapped mailboxes
  DevBuf p2p_mbox, p2p_arrive;
  DevBuf clamp_arrive;  // clamp_apply's fused finalize: arrivals (zero between launches)
  DevBuf np_sync;       // node prep in the reduce launch: epoch and flag words (NpArgs::sync)
  unsigned char* p2p_peer[kcc::P2P_MAX_RANKS] = {};  // opened peer mailboxes (own: p2p_mbox)
  int p2p_W = 0, p2p_rank = -1;
  int64_t p2p_smax = 0;
  bool p2p_ready = false;
};

}  // namespace

struct kcc_ctx {
  std::vector<Dev> devs;
  std::vector<ncclComm_t> comms;  // in-process devices (kcc_create with n_gpus > 1)
  ncclComm_t proc_comm = nullptr;  // one rank of a multi-process run (kcc_comm_init)
  int proc_ranks = 0, proc_rank = 0;
  int node_shards = 0;  // host-array entry points: node shards (0 = one per device)
  std::string err;
  double slow_frac = -1.0;
  // kcc_fit / kcc_capacity: each shard's counters, copied into pinned host memory on the
  // shard's stream (pageable copies could block the host between devices) and summed
  // after the final synchronisation: exact-path pairs and streamed rows of every shard
  unsigned long long* host_cnt = nullptr;
  size_t host_cnt_n = 0;
  int64_t host_stream_rows = -1;  // streamed rows of the last host-array fit (-1: none)
  // the in-library all-reduce (comms) has been checked against a host-side sum of the
  // devices' partials (the first host-array call of the context does it)
  bool allreduce_verified = false;
  bool allreduce_verify_every = false;  // kcc_set_allreduce_verify(ctx, 1)
};

namespace {

thread_local std::string g_create_error;

int fail(kcc_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

#define KCC_HIP(ctx, expr)                                                              \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail((ctx), e_ == hipErrorOutOfMemory ? KCC_ENOMEM : KCC_EHIP,             \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                   \
  } while (0)

#define KCC_NCCL(ctx, expr)                                                             \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return fail((ctx), KCC_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// CSR sanity on the host (the host-array entry points): a malformed offset array is
// rejected here instead of reaching the device.
int check_csr(kcc_ctx* ctx, int64_t n_nodes, int64_t n_cont, const int64_t* ptr) {
  if (n_nodes < 0 || n_cont < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_nodes == 0) {
    if (n_cont != 0) return fail(ctx, KCC_EINVAL, "containers without nodes");
    return KCC_OK;
  }
  if (!ptr) return fail(ctx, KCC_EINVAL, "node_ptr is NULL");
  if (ptr[0] != 0) return fail(ctx, KCC_EINVAL, "node_ptr[0] != 0");
  for (int64_t i = 0; i < n_nodes; ++i)
    if (ptr[i + 1] < ptr[i]) return fail(ctx, KCC_EINVAL, "node_ptr is not non-decreasing");
  if (ptr[n_nodes] != n_cont) return fail(ctx, KCC_EINVAL, "node_ptr[n_nodes] != n_containers");
  return KCC_OK;
}

// Contiguous node ranges, balanced by node count (the fit dominates).
void shard_nodes(int64_t n_nodes, int n, std::vector<int64_t>& lo, std::vector<int64_t>& hi) {
  lo.resize(n);
  hi.resize(n);
  for (int d = 0; d < n; ++d) {
    lo[d] = n_nodes * d / n;
    hi[d] = n_nodes * (d + 1) / n;
  }
}

template <class T>
int h2d(kcc_ctx* ctx, Dev& dv, DevBuf& buf, const T* src, int64_t count) {
  KCC_HIP(ctx, ensure(buf, sizeof(T) * (size_t)(count > 0 ? count : 1)));
  if (count > 0)
    KCC_HIP(ctx, hipMemcpyAsync(buf.p, src, sizeof(T) * (size_t)count, hipMemcpyHostToDevice,
                                dv.stream));
  return KCC_OK;
}

// ---- device-level pipeline pieces (no host sync, no allocation beyond growth) ----

// The device's fault words, zeroed when allocated (synchronously: kcc_reserve does it
// ahead of any capture).
int faults_ws(kcc_ctx* ctx, Dev& dv, hipStream_t s) {
  if (dv.faults.p) return KCC_OK;
  KCC_HIP(ctx, ensure(dv.faults, 8 * kcc::FAULT_WORDS));
  KCC_HIP(ctx, hipMemsetAsync(dv.faults.p, 0, 8 * kcc::FAULT_WORDS, s));
  KCC_HIP(ctx, hipStreamSynchronize(s));
  return KCC_OK;
}

// The reduce's look-back workspace: tail records for every wave a launch may have, zeroed
// when (re)allocated — synchronously: a stale tag would hand a wave a piece that was
// never published (allocation happens only when the workspace grows; kcc_reserve does it
// ahead of any capture).  Every launch leaves the tags 0.
int reduce_ws(kcc_ctx* ctx, Dev& dv, hipStream_t s) {
  const size_t tb = sizeof(uint64_t) * kcc::RED_TAIL_WORDS * (size_t)kcc::reduce_tail_records();
  if (dv.red_tail.bytes < tb) {
    KCC_HIP(ctx, ensure(dv.red_tail, tb));
    KCC_HIP(ctx, hipMemsetAsync(dv.red_tail.p, 0, dv.red_tail.bytes, s));
    KCC_HIP(ctx, hipStreamSynchronize(s));
  }
  return faults_ws(ctx, dv, s);
}

// After a synchronous entry point's final synchronisation: a set fault word means some
// wait of this (or an earlier, async) call gave up and results are not trustworthy.
int check_faults(kcc_ctx* ctx) {
  unsigned long long red = 0, p2p = 0;
  for (Dev& dv : ctx->devs) {
    if (!dv.faults.p) continue;
    unsigned long long f[2] = {0, 0};
    KCC_HIP(ctx, hipSetDevice(dv.device));
    KCC_HIP(ctx, hipMemcpy(f, dv.faults.p, sizeof(f), hipMemcpyDeviceToHost));
    red += f[kcc::FAULT_RED];
    p2p += f[kcc::FAULT_P2P];
  }
  if (red == 0 && p2p == 0) return KCC_OK;
  return fail(ctx, KCC_EFAULT,
              "device fault: " + std::to_string(red) + " reduce-side wait(s) (look-back, node prep, keyed gather) and " +
                  std::to_string(p2p) +
                  " exchange flag wait(s) gave up; results are not valid (every spec is marked "
                  "KCC_SPEC_FAULT) until kcc_clear_faults");
}

int reduce_async_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, int64_t n_cont, const int64_t* ptr,
                     const uint64_t* cpu, const int64_t* mem, const uint64_t* cpul,
                     const int64_t* meml, uint64_t* used_cpu, int64_t* used_mem,
                     uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s) {
  if (n_nodes < 0 || n_cont < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_nodes == 0) return n_cont == 0 ? KCC_OK : fail(ctx, KCC_EINVAL, "containers without nodes");
  if (n_nodes >= kcc::RED_MAX_NODES)
    return fail(ctx, KCC_EINVAL, "too many nodes per device (max 2^28 - 1)");
  if (!ptr || !used_cpu || !used_mem) return fail(ctx, KCC_EINVAL, "NULL node_ptr/output");
  if (n_cont > 0 && (!cpu || !mem)) return fail(ctx, KCC_EINVAL, "NULL cpu_req/mem_req");
  const bool lim = cpul != nullptr || meml != nullptr;
  if (lim && (!cpul || !meml || !lim_cpu || !lim_mem))
    return fail(ctx, KCC_EINVAL, "limits need cpu_lim, mem_lim, lim_cpu and lim_mem");
  if (!aligned16(cpu) || !aligned16(mem) || (lim && (!aligned16(cpul) || !aligned16(meml))))
    return fail(ctx, KCC_EINVAL, "container arrays must be 16-byte aligned");
  int rc = reduce_ws(ctx, dv, s);
  if (rc) return rc;
  KCC_HIP(ctx, kcc::launch_reduce(n_nodes, 0, n_cont, ptr, cpu, mem, lim ? cpul : nullptr,
                                  lim ? meml : nullptr, used_cpu, used_mem, lim ? lim_cpu : nullptr,
                                  lim ? lim_mem : nullptr, as<uint64_t>(dv.red_tail),
                                  as<unsigned long long>(dv.faults), s));
  return KCC_OK;
}

kcc::SpecPrep spec_prep_of(Dev& dv) {
  kcc::SpecPrep sp;
  sp.rec = as<kcc::SpecRec>(dv.srec);
  sp.perm = as<int32_t>(dv.sperm);
  return sp;
}

int reserve_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, int64_t n_cont, int64_t n_specs) {
  KCC_HIP(ctx, hipSetDevice(dv.device));
  const size_t N = (size_t)(n_nodes > 0 ? n_nodes : 1);
  const size_t S = (size_t)(n_specs > 0 ? n_specs : 1);
  (void)n_cont;  // the reduce's workspace does not depend on the container count
  {
    int rc = reduce_ws(ctx, dv, dv.stream);
    if (rc) return rc;
  }
  KCC_HIP(ctx, ensure(dv.fast_a, sizeof(kcc::FitGroupA) * (size_t)kcc::fit_groups((int64_t)N)));
  KCC_HIP(ctx, ensure(dv.fast_b, sizeof(kcc::FitGroup) * (size_t)kcc::fit_groups((int64_t)N)));
  KCC_HIP(ctx, ensure(dv.fast_cl, sizeof(int32_t) * kcc::FIT_GROUP * (size_t)kcc::fit_groups((int64_t)N)));
  KCC_HIP(ctx, ensure(dv.slow, sizeof(kcc::SlowNode) * N));
  KCC_HIP(ctx, ensure(dv.slow_list, sizeof(int64_t) * N));
  KCC_HIP(ctx, ensure(dv.srec, sizeof(kcc::SpecRec) * S));
  KCC_HIP(ctx, ensure(dv.sperm, 4 * S));
  KCC_HIP(ctx, ensure(dv.counters, sizeof(unsigned long long) * kcc::CNT_N));
  if (!dv.np_sync.p) {  // node prep in the reduce launch: epoch words (kcc::NpArgs::sync)
    const size_t bytes = 4 * (kcc::NP_FLAGS + (size_t)kcc::reduce_tail_records());
    KCC_HIP(ctx, ensure(dv.np_sync, bytes));
    KCC_HIP(ctx, hipMemsetAsync(dv.np_sync.p, 0, bytes, dv.stream));
    // the fused reduce runs on the caller's stream, which nothing orders after dv.stream:
    // the zeroing completes here, on its own
    KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  }
  if (!dv.clamp_arrive.p) {  // the fused finalize's arrivals: every launch leaves them zero
    KCC_HIP(ctx, ensure(dv.clamp_arrive, 64));
    KCC_HIP(ctx, hipMemsetAsync(dv.clamp_arrive.p, 0, 64, dv.stream));
    KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  }
  // (a new allocation is a larger one: compare sizes, hipMalloc may hand back the address)
  const size_t q_before = dv.fit_q.bytes;
  KCC_HIP(ctx, ensure(dv.fit_q, 4 * (size_t)kcc::fit_queue_words((int64_t)S)));
  if (dv.fit_q.bytes != q_before) dv.fitq_dirty = true;
  const size_t S64 = (S + 63) / 64 * 64;
  KCC_HIP(ctx, ensure(dv.c_bcnt, 8 * (S64 / 64)));
  KCC_HIP(ctx, ensure(dv.c_cs, 8 * S));
  KCC_HIP(ctx, ensure(dv.c_ms, 8 * S));
  KCC_HIP(ctx, ensure(dv.c_mrc, 4 * S64));
  KCC_HIP(ctx, ensure(dv.c_crm, 4 * S64));
  KCC_HIP(ctx, ensure(dv.c_dperm, 4 * S));
  // the table copies stay all-zero between calls (clamp_prep zeroes what it reads); a
  // new or grown allocation, or a layout change, is zeroed before its first use
  const int64_t cs_ = kcc::clamp_c_cells((int64_t)S), hs = kcc::clamp_h_cells((int64_t)S);
  const size_t before[3] = {dv.c_C.bytes, dv.c_H2.bytes, dv.c_H3.bytes};
  // the spec ranks' per-slice counts: [rank_slices(S)][2][S] u32 (plain stores, nothing
  // to keep zero)
  KCC_HIP(ctx, ensure(dv.c_rank, 4 * (size_t)kcc::rank_words((int64_t)S)));
  if (dv.rank_arrive.bytes < 4 * (S64 / 64)) {  // every call leaves them zero
    KCC_HIP(ctx, ensure(dv.rank_arrive, 4 * (S64 / 64)));
    KCC_HIP(ctx, hipMemsetAsync(dv.rank_arrive.p, 0, dv.rank_arrive.bytes, dv.stream));
    KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  }
  KCC_HIP(ctx, ensure(dv.c_C, 8 * (size_t)kcc::C_COPIES * (size_t)cs_));
  KCC_HIP(ctx, ensure(dv.c_H2, 8 * (size_t)kcc::H2_COPIES * (size_t)hs));
  KCC_HIP(ctx, ensure(dv.c_H3, 8 * (size_t)kcc::H2_COPIES * (size_t)hs));
  KCC_HIP(ctx, ensure(dv.c_Crow, 8 * (size_t)cs_));
  if (kcc::clamp_binned((int64_t)S)) {  // node_prep's binned H2 / H3 records
    // the most passes (and record slots) any call of up to N rows makes
    const size_t passes = (size_t)((N + kcc::CLAMP_PASS_ROWS_MIN - 1) / kcc::CLAMP_PASS_ROWS_MIN);
    const size_t recs = (size_t)((N + kcc::CLAMP_PASS_ROWS_MAX - 1) / kcc::CLAMP_PASS_ROWS_MAX) *
                        2 * kcc::CLAMP_PASS_ROWS_MAX;  // >= passes(n) x 2 pass_rows(n) for any n <= N
    KCC_HIP(ctx, ensure(dv.c_rec, 8 * recs));
    KCC_HIP(ctx, ensure(dv.c_dir, 4 * (size_t)kcc::clamp_d_stride((int64_t)S) * passes));
  }
  if (dv.c_C.bytes != before[0] || dv.c_H2.bytes != before[1] || dv.c_H3.bytes != before[2] ||
      dv.c_stride != cs_ || dv.h_stride != hs)
    dv.clamp_dirty = true;
  dv.c_stride = cs_;
  dv.h_stride = hs;
  dv.d_stride = kcc::clamp_d_stride((int64_t)S);
  return KCC_OK;
}

// Zero the table copies when they are not known to be zero (before node_prep adds to them).
int clamp_clean(kcc_ctx* ctx, Dev& dv, hipStream_t s) {
  if (dv.fitq_dirty) {  // a new allocation of the fit queues (every launch leaves them zero)
    KCC_HIP(ctx, hipMemsetAsync(dv.fit_q.p, 0, dv.fit_q.bytes, s));
    dv.fitq_dirty = false;
  }
  if (!dv.clamp_dirty) return KCC_OK;
  KCC_HIP(ctx, hipMemsetAsync(dv.c_C.p, 0, dv.c_C.bytes, s));
  KCC_HIP(ctx, hipMemsetAsync(dv.c_H2.p, 0, dv.c_H2.bytes, s));
  KCC_HIP(ctx, hipMemsetAsync(dv.c_H3.p, 0, dv.c_H3.bytes, s));
  dv.clamp_dirty = false;
  return KCC_OK;
}

kcc::ClampWork clamp_of(Dev& dv) {
  kcc::ClampWork cw;
  cw.rank = as<uint32_t>(dv.c_rank);
  cw.bcnt = as<uint32_t>(dv.c_bcnt);
  cw.cs = as<uint64_t>(dv.c_cs);
  cw.ms = as<int64_t>(dv.c_ms);
  cw.mr_c = as<uint32_t>(dv.c_mrc);
  cw.cr_m = as<uint32_t>(dv.c_crm);
  cw.dperm = as<int32_t>(dv.c_dperm);
  cw.C = as<int64_t>(dv.c_C);
  cw.H2 = as<int64_t>(dv.c_H2);
  cw.H3 = as<int64_t>(dv.c_H3);
  cw.Crow = as<int64_t>(dv.c_Crow);
  cw.rec = as<uint64_t>(dv.c_rec);
  cw.dir = as<uint32_t>(dv.c_dir);
  cw.c_stride = dv.c_stride;
  cw.h_stride = dv.h_stride;
  cw.d_stride = dv.d_stride;
  cw.n_pass = 0;
  return cw;
}

// The spec-side workspace a call of S specs writes (host-side guard before any launch: a
// kernel writing past an allocation faults the device).
int check_spec_ws(kcc_ctx* ctx, Dev& dv, int64_t S) {
  const size_t S64 = (size_t)(S + 63) / 64 * 64;
  const bool ok = dv.c_rank.bytes >= 4 * (size_t)kcc::rank_words(S) &&
                  dv.c_bcnt.bytes >= 8 * (S64 / 64) && dv.c_mrc.bytes >= 4 * S64 &&
                  dv.rank_arrive.bytes >= 4 * (S64 / 64) &&
                  dv.c_crm.bytes >= 4 * S64 && dv.c_cs.bytes >= 8 * (size_t)S &&
                  dv.c_ms.bytes >= 8 * (size_t)S && dv.c_dperm.bytes >= 4 * (size_t)S &&
                  dv.srec.bytes >= sizeof(kcc::SpecRec) * (size_t)S &&
                  dv.sperm.bytes >= 4 * (size_t)S &&
                  dv.counters.bytes >= sizeof(unsigned long long) * kcc::CNT_N &&
                  dv.c_C.bytes >= 8 * (size_t)kcc::C_COPIES * (size_t)dv.c_stride &&
                  dv.c_stride >= kcc::clamp_c_cells(S);
  return ok ? KCC_OK : fail(ctx, KCC_EINVAL, "internal: spec workspace smaller than the call");
}

kcc::PlaceArgs place_args(Dev& dv, int64_t n_specs, const uint64_t* spec_cpu,
                          const int64_t* spec_mem, int64_t* partial) {
  return kcc::PlaceArgs{n_specs, spec_cpu, spec_mem, spec_prep_of(dv), clamp_of(dv), partial,
                        as<unsigned long long>(dv.counters), 0,
                        as<const unsigned long long>(dv.faults), 0};
}

int fit_prepare_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, const uint64_t* alloc_cpu,
                    const int64_t* alloc_mem, const int64_t* alloc_pods,
                    const int64_t* pod_count, const uint64_t* used_cpu,
                    const int64_t* used_mem, int64_t n_specs, const uint64_t* spec_cpu,
                    const int64_t* spec_mem, int64_t* partial, hipStream_t s) {
  ctx->host_stream_rows = -1;  // (kcc_fit_stream_rows: this call's device counters)
  if (n_nodes < 0 || n_specs < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_specs >= kcc::MAX_SPECS) return fail(ctx, KCC_EINVAL, "too many specs (max 2^26 - 1)");
  if (n_specs > 0 && (!spec_cpu || !spec_mem || !partial))
    return fail(ctx, KCC_EINVAL, "NULL spec array / partial");
  if (n_nodes > 0 && (!alloc_cpu || !alloc_mem || !alloc_pods || !pod_count || !used_cpu || !used_mem))
    return fail(ctx, KCC_EINVAL, "NULL node array");
  int rc = reserve_dev(ctx, dv, n_nodes, 0, n_specs);
  if (rc) return rc;
  dv.last_pairs = n_nodes * n_specs;
  dv.prep_nodes = n_nodes;
  dv.prep_specs = n_specs;
  if (n_specs == 0) return KCC_OK;
  if ((rc = check_spec_ws(ctx, dv, n_specs))) return rc;
  rc = clamp_clean(ctx, dv, s);
  if (rc) return rc;
  dv.clamp_dirty = true;  // until every kernel that leaves the tables zero is queued
  // spec_rank zeroes the counters and the coarse clamp table; spec_place zeroes
  // `partial` (no memset launches) and rides in the node_prep launch (node_prep reads
  // only the sorted arrays the ranks wrote)
  KCC_HIP(ctx, kcc::launch_spec_rank(kcc::rank_args(n_specs, spec_cpu, spec_mem, clamp_of(dv),
                                                    as<unsigned long long>(dv.counters),
                                                    as<uint32_t>(dv.rank_arrive)),
                                     s));
  const kcc::PlaceArgs pa = place_args(dv, n_specs, spec_cpu, spec_mem, partial);
  KCC_HIP(ctx, kcc::launch_node_prep(n_nodes, alloc_cpu, alloc_mem, alloc_pods, pod_count,
                                       used_cpu, used_mem, as<kcc::FitGroupA>(dv.fast_a),
                                       as<kcc::FitGroup>(dv.fast_b), as<kcc::SlowNode>(dv.slow),
                                       as<int64_t>(dv.slow_list), n_specs, clamp_of(dv),
                                       as<unsigned long long>(dv.counters), 0, 0,
                                       n_nodes, s, dv.fit_dense, &pa, nullptr));
  if (n_nodes == 0) {
    dv.clamp_dirty = false;
    return KCC_OK;
  }
  dv.stream_chunks = 1;
  KCC_HIP(ctx, kcc::launch_clamp_apply(n_specs, n_nodes, clamp_of(dv),
                                       as<unsigned long long>(dv.counters), partial, s));
  dv.clamp_dirty = false;
  return KCC_OK;
}

int fit_run_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, int64_t n_specs, int64_t* partial,
                hipStream_t s) {
  if (n_nodes != dv.prep_nodes || n_specs != dv.prep_specs)
    return fail(ctx, KCC_EINVAL, "fit_run sizes differ from the preceding fit_prepare");
  if (n_nodes == 0 || n_specs == 0) return KCC_OK;
  if (!partial) return fail(ctx, KCC_EINVAL, "NULL partial");
  KCC_HIP(ctx, kcc::launch_fit(n_nodes, as<kcc::FitGroupA>(dv.fast_a), as<kcc::FitGroup>(dv.fast_b),
                               as<kcc::SlowNode>(dv.slow),
                               as<int64_t>(dv.slow_list), n_specs, spec_prep_of(dv), partial,
                               as<unsigned long long>(dv.counters), as<uint32_t>(dv.fit_q), 0,
                               n_nodes, s, as<const unsigned long long>(dv.faults)));
  return KCC_OK;
}

int fit_partial_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, const uint64_t* alloc_cpu,
                    const int64_t* alloc_mem, const int64_t* alloc_pods,
                    const int64_t* pod_count, const uint64_t* used_cpu,
                    const int64_t* used_mem, int64_t n_specs, const uint64_t* spec_cpu,
                    const int64_t* spec_mem, int64_t* partial, hipStream_t s) {
  int rc = fit_prepare_dev(ctx, dv, n_nodes, alloc_cpu, alloc_mem, alloc_pods, pod_count,
                           used_cpu, used_mem, n_specs, spec_cpu, spec_mem, partial, s);
  if (rc) return rc;
  return fit_run_dev(ctx, dv, n_nodes, n_specs, partial, s);
}

int fit_finalize_dev(kcc_ctx* ctx, Dev& dv, int64_t n_specs, const int64_t* partial,
                     int64_t* totals, int32_t* spec_err, hipStream_t s) {
  if (n_specs < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_specs == 0) return KCC_OK;
  if (!partial || !totals || !spec_err) return fail(ctx, KCC_EINVAL, "NULL partial/totals/err");
  if (dv.sperm.bytes < sizeof(int32_t) * (size_t)n_specs)
    return fail(ctx, KCC_EINVAL, "finalize without a matching fit_partial");
  KCC_HIP(ctx, kcc::launch_fit_finalize(n_specs, partial, as<int32_t>(dv.sperm), totals,
                                        spec_err, as<const unsigned long long>(dv.faults), s));
  return KCC_OK;
}


// ---- pipelined reduce + fit (kcc_capacity_partial_async) ---------------------------

hipError_t prof_event(Dev& dv, hipEvent_t* ev) {
  if (!dv.prof_free.empty()) {
    *ev = dv.prof_free.back();
    dv.prof_free.pop_back();
    return hipSuccess;
  }
  // device-scope release only: a timing event between two kernels of one stream needs no
  // system-scope fence (with it, hipEventCreate's default, every record left a ~5.5 us gap
  // on the stream)
  return hipEventCreateWithFlags(ev, hipEventDisableSystemFence);
}

#ifndef KCC_NP_IN_REDUCE
#define KCC_NP_IN_REDUCE 1
#endif

// Chunk boundaries: node ranges of ~equal node count, multiples of CHUNK_ALIGN (a
// multiple of FIT_GROUP: the fit's node groups do not straddle two chunks); at least
// `min_nodes` nodes per chunk.
constexpr int64_t CHUNK_ALIGN = kcc::CLAMP_PASS_ROWS_MAX;  // whole node_prep passes
int plan_chunks(int64_t n_nodes, int want, int64_t min_nodes, std::vector<int64_t>& lo,
                std::vector<int64_t>& hi) {
  int k = want;
  if (k > kcc::FIT_MAX_CHUNKS) k = kcc::FIT_MAX_CHUNKS;
  while (k > 1 && n_nodes / k < min_nodes) --k;
  if (k < 1) k = 1;
  lo.assign(k, 0);
  hi.assign(k, 0);
  for (int c = 0; c < k; ++c) {
    lo[c] = c == 0 ? 0 : hi[c - 1];
    hi[c] = c == k - 1 ? n_nodes : (n_nodes * (c + 1) / k) / CHUNK_ALIGN * CHUNK_ALIGN;
    if (hi[c] < lo[c]) hi[c] = lo[c];
  }
  return k;
}

// Overlapping the reduce of chunk k with the fit of chunk k-1 measured SLOWER at C4
// (0.80 / 0.85 / 0.88 ms per step at 1 / 2 / 4 chunks): the fit keeps every SIMD's
// VALU issue ~90 % busy and the concurrent reduce's waves slow it by more than the
// reduce's own time.  Default: one chunk, everything on the caller's stream.
constexpr int KCC_DEFAULT_CHUNKS = 1;
constexpr int64_t KCC_MIN_CHUNK_NODES = 32768;

int capacity_partial_dev(kcc_ctx* ctx, Dev& dv, int64_t n_nodes, int64_t n_cont,
                         const int64_t* h_ptr, const int64_t* ptr, const uint64_t* cpu,
                         const int64_t* mem, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
                         const int64_t* alloc_pods, const int64_t* pod_count, uint64_t* used_cpu,
                         int64_t* used_mem, int64_t n_specs, const uint64_t* spec_cpu,
                         const int64_t* spec_mem, int64_t* partial, int n_chunks, hipStream_t s,
                         int64_t* totals = nullptr, int32_t* spec_err = nullptr) {
  ctx->host_stream_rows = -1;  // (kcc_fit_stream_rows: this call's device counters)
  if (n_nodes < 0 || n_cont < 0 || n_specs < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_nodes >= kcc::RED_MAX_NODES)
    return fail(ctx, KCC_EINVAL, "too many nodes per device (max 2^28 - 1)");
  if (n_specs >= kcc::MAX_SPECS) return fail(ctx, KCC_EINVAL, "too many specs (max 2^26 - 1)");
  if (n_nodes == 0 && n_cont != 0) return fail(ctx, KCC_EINVAL, "containers without nodes");
  if (n_nodes > 0 && (!ptr || !used_cpu || !used_mem || !alloc_cpu || !alloc_mem || !alloc_pods ||
                      !pod_count))
    return fail(ctx, KCC_EINVAL, "NULL node array");
  if (n_cont > 0 && (!cpu || !mem)) return fail(ctx, KCC_EINVAL, "NULL cpu_req/mem_req");
  if (!aligned16(cpu) || !aligned16(mem))
    return fail(ctx, KCC_EINVAL, "container arrays must be 16-byte aligned");
  if (n_specs > 0 && (!spec_cpu || !spec_mem || !partial))
    return fail(ctx, KCC_EINVAL, "NULL spec array / partial");
  std::vector<int64_t> lo, hi;
  const int k = plan_chunks(n_nodes, h_ptr ? (n_chunks > 0 ? n_chunks : KCC_DEFAULT_CHUNKS) : 1,
                            KCC_MIN_CHUNK_NODES, lo, hi);
  std::vector<int64_t> c0(k), c1(k);
  for (int c = 0; c < k; ++c) {
    if (k == 1) {
      c0[c] = 0;
      c1[c] = n_cont;
    } else {
      c0[c] = h_ptr[lo[c]];
      c1[c] = h_ptr[hi[c]];
      if (c0[c] < 0 || c1[c] < c0[c] || c1[c] > n_cont)
        return fail(ctx, KCC_EINVAL, "h_node_ptr is not a CSR of n_containers");
    }
  }
  int rc = reserve_dev(ctx, dv, n_nodes, n_cont, n_specs);
  if (rc) return rc;
  if (n_specs > 0 && (rc = check_spec_ws(ctx, dv, n_specs))) return rc;
  for (int c = 0; c < k; ++c)
    if (!dv.ev_red[c]) KCC_HIP(ctx, hipEventCreateWithFlags(&dv.ev_red[c], hipEventDisableTiming));
  dv.last_pairs = n_nodes * n_specs;
  dv.stream_chunks = k;
  dv.prep_nodes = -1;  // the split fit_run API must not reuse this call's workspace state
  dv.prep_specs = -1;
  // k > 1: the reduces run on the side stream, forked from s (they wait for everything
  // already queued on s: the previous call's fits still read used_* and the node
  // streams); k == 1: everything on s
  hipStream_t rs = k > 1 ? dv.side : s;
  if (k > 1) {
    KCC_HIP(ctx, hipEventRecord(dv.ev_fork, s));
    KCC_HIP(ctx, hipStreamWaitEvent(dv.side, dv.ev_fork, 0));
  }
  // k == 1: the spec ranks ride in the reduce launch (extra workgroups in front of the
  // reduce's: independent work) and spec_place in the node_prep launch (node_prep reads
  // only the arrays the ranks wrote): four launches per call — reduce + rank, node_prep +
  // place, fit, clamp_apply
  const bool fuse_place = n_specs > 0;
  const bool fuse_rank = k == 1 && fuse_place && n_nodes > 0 && n_cont > 0;
  // the clamp in the fit (one node chunk, S <= CLAMP_LDS_SPECS, not dense): no clamp_apply
  const bool nc = k == 1 && n_specs > 0 && n_specs <= kcc::CLAMP_LDS_SPECS && !dv.fit_dense &&
                  (dv.clamp_in_fit == 1 ||
                   (dv.clamp_in_fit < 0 && kcc::clamp_in_fit_auto(n_nodes, n_specs)));
  int32_t* const fast_cl = nc ? as<int32_t>(dv.fast_cl) : nullptr;
  dv.last_nc = nc;
  // the clamp in the fit needs no spec ranks (no clamp tables): the reduce launch carries
  // one workgroup that zeroes the counters, and spec_place counts the classes itself
  kcc::RankArgs ra = kcc::rank_args(n_specs, spec_cpu, spec_mem, clamp_of(dv),
                                    as<unsigned long long>(dv.counters),
                                    as<uint32_t>(dv.rank_arrive), nc);
  kcc::PlaceArgs pa = place_args(dv, n_specs, spec_cpu, spec_mem, partial);
  pa.no_ranks = nc ? 1 : 0;
  // the clamp in the fit with the ranks in the reduce launch: spec_place and node_prep's
  // work ride there too, behind the reduce's workgroups (kcc::NpArgs) — one launch fewer
  const bool np_fused = KCC_NP_IN_REDUCE && nc && fuse_rank;
  kcc::NpArgs np{};
  if (np_fused) {
    ra.done_flag = as<uint32_t>(dv.np_sync);
    np.n_place = (int32_t)((n_specs + 255) / 256);
    np.n_rows = (int32_t)((n_nodes + kcc::NP_ROWS_PER_WG - 1) / kcc::NP_ROWS_PER_WG);
    np.sync = as<uint32_t>(dv.np_sync);
    np.pa = pa;
    np.n = n_nodes;
    np.alloc_cpu = alloc_cpu;
    np.alloc_mem = alloc_mem;
    np.alloc_pods = alloc_pods;
    np.pod_count = pod_count;
    np.used_cpu = used_cpu;
    np.used_mem = used_mem;
    np.fast_a = as<kcc::FitGroupA>(dv.fast_a);
    np.fast_b = as<kcc::FitGroup>(dv.fast_b);
    np.slow = as<kcc::SlowNode>(dv.slow);
    np.slow_list = as<int64_t>(dv.slow_list);
    np.fast_cl = fast_cl;
    np.counters = as<unsigned long long>(dv.counters);
    np.bcnt = clamp_of(dv).bcnt;
    np.S = n_specs;
    np.faults = as<unsigned long long>(dv.faults);
  }
  if (n_specs > 0) {
    rc = clamp_clean(ctx, dv, s);
    if (rc) return rc;
    dv.clamp_dirty = true;  // until every kernel that leaves the tables zero is queued
    if (!fuse_rank) KCC_HIP(ctx, kcc::launch_spec_rank(ra, s));
  }
  for (int c = 0; c < k; ++c) {
    const int64_t n = hi[c] - lo[c];
    ProfPair pp{};
    if (dv.prof_on) {  // (the launch's own dispatch timestamps: no event packets around it)
      KCC_HIP(ctx, prof_event(dv, &pp.a));
      KCC_HIP(ctx, prof_event(dv, &pp.b));
    }
    KCC_HIP(ctx, kcc::launch_reduce(n, c0[c], c1[c] - c0[c], ptr + lo[c], cpu, mem, nullptr, nullptr,
                                    used_cpu + lo[c], used_mem + lo[c], nullptr, nullptr,
                                    as<uint64_t>(dv.red_tail),
                                    as<unsigned long long>(dv.faults), rs,
                                    fuse_rank ? &ra : nullptr, np_fused ? &np : nullptr,
                                    dv.prof_on ? pp.a : nullptr, dv.prof_on ? pp.b : nullptr));
    if (dv.prof_on) {
      pp.kind = 0;
      dv.prof_pending.push_back(pp);
    }
    if (k > 1) KCC_HIP(ctx, hipEventRecord(dv.ev_red[c], dv.side));
  }
  const bool fuse_fin = totals && n_nodes > 0;
  const kcc::FinArgs fin{as<int32_t>(dv.sperm), totals, spec_err, as<uint32_t>(dv.clamp_arrive),
                         as<const unsigned long long>(dv.faults)};
  for (int c = 0; c < k; ++c) {
    if (k > 1) KCC_HIP(ctx, hipStreamWaitEvent(s, dv.ev_red[c], 0));  // also joins the side stream
    const int64_t n = hi[c] - lo[c];
    const bool place_here = fuse_place && c == 0;
    if (n_specs == 0 || (n == 0 && !place_here)) continue;
    if (!np_fused)  // (else: in the reduce launch)
    KCC_HIP(ctx, kcc::launch_node_prep(n, alloc_cpu + lo[c], alloc_mem + lo[c], alloc_pods + lo[c],
                                       pod_count + lo[c], used_cpu + lo[c], used_mem + lo[c],
                                       as<kcc::FitGroupA>(dv.fast_a) + lo[c] / kcc::FIT_GROUP,
                                       as<kcc::FitGroup>(dv.fast_b) + lo[c] / kcc::FIT_GROUP,
                                       as<kcc::SlowNode>(dv.slow) + lo[c],
                                       as<int64_t>(dv.slow_list) + lo[c], n_specs, clamp_of(dv),
                                       as<unsigned long long>(dv.counters),
                                       c, lo[c], n_nodes, s, dv.fit_dense,
                                       place_here ? &pa : nullptr, fast_cl));
    if (n == 0) continue;
    ProfPair pp{};
    if (dv.prof_on) {
      KCC_HIP(ctx, prof_event(dv, &pp.a));
      KCC_HIP(ctx, prof_event(dv, &pp.b));
    }
    KCC_HIP(ctx, kcc::launch_fit(n, as<kcc::FitGroupA>(dv.fast_a) + lo[c] / kcc::FIT_GROUP,
                                 as<kcc::FitGroup>(dv.fast_b) + lo[c] / kcc::FIT_GROUP,
                                 as<kcc::SlowNode>(dv.slow) + lo[c],
                                 as<int64_t>(dv.slow_list) + lo[c], n_specs, spec_prep_of(dv),
                                 partial, as<unsigned long long>(dv.counters),
                                 as<uint32_t>(dv.fit_q), c, n_nodes, s,
                                 as<const unsigned long long>(dv.faults), fast_cl,
                                 dv.prof_on ? pp.a : nullptr, dv.prof_on ? pp.b : nullptr));
    if (dv.prof_on) {
      pp.kind = 1;
      dv.prof_pending.push_back(pp);
    }
  }
  // the pod-slot clamp of every chunk's fast rows, added back per spec; totals != nullptr:
  // the clamp launch's last workgroup also finalizes (no fit_finalize launch)
  if (n_specs > 0 && nc) {  // the fit applied the clamp: no clamp_apply, nothing dirty
    dv.clamp_dirty = false;
    if (totals) return fit_finalize_dev(ctx, dv, n_specs, partial, totals, spec_err, s);
    return KCC_OK;
  }
  if (n_specs > 0) {
    // (clamp_arrive is allocated and zeroed by reserve_dev; every launch leaves it zero)
    if (n_nodes > 0)
      KCC_HIP(ctx, kcc::launch_clamp_apply(n_specs, n_nodes, clamp_of(dv),
                                           as<unsigned long long>(dv.counters), partial, s,
                                           fuse_fin ? &fin : nullptr));
    dv.clamp_dirty = false;
    if (totals && !fuse_fin)
      return fit_finalize_dev(ctx, dv, n_specs, partial, totals, spec_err, s);
  }
  return KCC_OK;
}

// Host-array pipeline shared by kcc_fit / kcc_capacity: per device upload its node
// shard (and container shard), reduce (optional), fit_partial; all-reduce partials
// over RCCL when sharded; finalize on device 0; copy back.
int run_host(kcc_ctx* ctx, bool with_reduce, int64_t n_nodes, int64_t n_cont,
             const int64_t* node_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
             const uint64_t* alloc_cpu, const int64_t* alloc_mem, const int64_t* alloc_pods,
             const int64_t* pod_count, const uint64_t* used_cpu_in, const int64_t* used_mem_in,
             int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
             int64_t* totals, int32_t* spec_err) {
  if (n_nodes < 0 || n_specs < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_specs > 0 && (!spec_cpu || !spec_mem || !totals || !spec_err))
    return fail(ctx, KCC_EINVAL, "NULL spec array / output");
  if (n_nodes > 0 && (!alloc_cpu || !alloc_mem || !alloc_pods || !pod_count))
    return fail(ctx, KCC_EINVAL, "NULL node array");
  if (with_reduce) {
    int rc = check_csr(ctx, n_nodes, n_cont, node_ptr);
    if (rc) return rc;
    if (n_cont > 0 && (!cpu_req || !mem_req)) return fail(ctx, KCC_EINVAL, "NULL container array");
  } else if (n_nodes > 0 && (!used_cpu_in || !used_mem_in)) {
    return fail(ctx, KCC_EINVAL, "NULL used array");
  }
  if (n_specs == 0) return KCC_OK;
  const int nd = (int)ctx->devs.size();
  // node shards: one per device, or ctx->node_shards (kcc_set_node_shards) dealt
  // round-robin over the devices; a device's shards run one after the other on its
  // stream, each into its own slot of the device's partial buffer, and the slots are
  // summed on the device before the RCCL all-reduce over devices
  const int ns = ctx->node_shards > nd ? ctx->node_shards : nd;
  const int slots = (ns + nd - 1) / nd;
  std::vector<int64_t> lo, hi;
  shard_nodes(n_nodes, ns, lo, hi);
  std::vector<std::vector<int64_t>> rebased(ns);  // per shard: copies may still be in flight
  if (ctx->host_cnt_n < (size_t)ns * kcc::CNT_N) {
    if (ctx->host_cnt) (void)hipHostFree(ctx->host_cnt);
    ctx->host_cnt = nullptr;
    ctx->host_cnt_n = 0;
    KCC_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->host_cnt),
                               sizeof(unsigned long long) * (size_t)ns * kcc::CNT_N, hipHostMallocDefault));
    ctx->host_cnt_n = (size_t)ns * kcc::CNT_N;
  }
  ctx->host_stream_rows = -1;
  for (int d = 0; d < nd; ++d) {
    Dev& dv = ctx->devs[d];
    KCC_HIP(ctx, hipSetDevice(dv.device));
    KCC_HIP(ctx, ensure(dv.partial, sizeof(int64_t) * 2 * (size_t)n_specs * (size_t)slots));
  }
  for (int sh = 0; sh < ns; ++sh) {
    Dev& dv = ctx->devs[sh % nd];
    int64_t* part = as<int64_t>(dv.partial) + (size_t)(sh / nd) * 2 * (size_t)n_specs;
    KCC_HIP(ctx, hipSetDevice(dv.device));
    const int64_t n = hi[sh] - lo[sh];
    int rc;
    if ((rc = h2d(ctx, dv, dv.alloc_cpu, alloc_cpu + lo[sh], n))) return rc;
    if ((rc = h2d(ctx, dv, dv.alloc_mem, alloc_mem + lo[sh], n))) return rc;
    if ((rc = h2d(ctx, dv, dv.alloc_pods, alloc_pods + lo[sh], n))) return rc;
    if ((rc = h2d(ctx, dv, dv.pod_count, pod_count + lo[sh], n))) return rc;
    if ((rc = h2d(ctx, dv, dv.spec_cpu, spec_cpu, n_specs))) return rc;
    if ((rc = h2d(ctx, dv, dv.spec_mem, spec_mem, n_specs))) return rc;
    if (with_reduce) {
      // the shard's containers [c0, c1) with its CSR offsets rebased to 0
      const int64_t c0 = n > 0 ? node_ptr[lo[sh]] : 0, c1 = n > 0 ? node_ptr[hi[sh]] : 0;
      std::vector<int64_t>& rb = rebased[sh];
      rb.resize((size_t)n + 1);
      for (int64_t k = 0; k <= n; ++k) rb[k] = n > 0 ? node_ptr[lo[sh] + k] - c0 : 0;
      if ((rc = h2d(ctx, dv, dv.ptr, rb.data(), n + 1))) return rc;
      if ((rc = h2d(ctx, dv, dv.cpu, cpu_req + c0, c1 - c0))) return rc;
      if ((rc = h2d(ctx, dv, dv.mem, mem_req + c0, c1 - c0))) return rc;
      KCC_HIP(ctx, ensure(dv.used_cpu, 8 * (size_t)(n > 0 ? n : 1)));
      KCC_HIP(ctx, ensure(dv.used_mem, 8 * (size_t)(n > 0 ? n : 1)));
      if (n > 0) {
        rc = reduce_async_dev(ctx, dv, n, c1 - c0, as<int64_t>(dv.ptr), as<uint64_t>(dv.cpu),
                              as<int64_t>(dv.mem), nullptr, nullptr, as<uint64_t>(dv.used_cpu),
                              as<int64_t>(dv.used_mem), nullptr, nullptr, dv.stream);
        if (rc) return rc;
      }
    } else {
      if ((rc = h2d(ctx, dv, dv.used_cpu, used_cpu_in + lo[sh], n))) return rc;
      if ((rc = h2d(ctx, dv, dv.used_mem, used_mem_in + lo[sh], n))) return rc;
    }
    rc = fit_partial_dev(ctx, dv, n, as<uint64_t>(dv.alloc_cpu), as<int64_t>(dv.alloc_mem),
                         as<int64_t>(dv.alloc_pods), as<int64_t>(dv.pod_count),
                         as<uint64_t>(dv.used_cpu), as<int64_t>(dv.used_mem), n_specs,
                         as<uint64_t>(dv.spec_cpu), as<int64_t>(dv.spec_mem), part, dv.stream);
    if (rc) return rc;
    // exact-path pair count of this shard (the next shard's spec setup zeroes it)
    KCC_HIP(ctx, hipMemcpyAsync(ctx->host_cnt + (size_t)sh * kcc::CNT_N, dv.counters.p,
                                sizeof(unsigned long long) * kcc::CNT_N, hipMemcpyDeviceToHost,
                                dv.stream));
    if (sh >= nd)  // fold this slot into the device's slot 0 (wrapping int64 adds)
      KCC_HIP(ctx, kcc::launch_partial_add(2 * n_specs, as<int64_t>(dv.partial), part, dv.stream));
  }
  if (!ctx->comms.empty()) {
    // the context's first all-reduce proves itself (as bench.py's exchange does before it
    // is timed): every device's result must equal the host's wrapping sum of the devices'
    // partials (CC:138 summed over devices), else KCC_ERCCL.  Later calls are checked only
    // with kcc_set_allreduce_verify(ctx, 1) (two device-to-host copies and stream syncs
    // per device and call)
    const bool verify = !ctx->allreduce_verified || ctx->allreduce_verify_every;
    const size_t words = 2 * (size_t)n_specs;
    std::vector<uint64_t> expect, got;
    if (verify) {
      expect.assign(words, 0);
      got.resize(words);
      for (int d = 0; d < nd; ++d) {
        Dev& dv = ctx->devs[d];
        KCC_HIP(ctx, hipSetDevice(dv.device));
        KCC_HIP(ctx, hipMemcpyAsync(got.data(), dv.partial.p, 8 * words, hipMemcpyDeviceToHost,
                                    dv.stream));
        KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
        for (size_t i = 0; i < words; ++i) expect[i] += got[i];
      }
    }
    KCC_NCCL(ctx, ncclGroupStart());
    for (int d = 0; d < nd; ++d) {
      Dev& dv = ctx->devs[d];
      KCC_NCCL(ctx, ncclAllReduce(dv.partial.p, dv.partial.p, words, ncclInt64,
                                  ncclSum, ctx->comms[d], dv.stream));
    }
    KCC_NCCL(ctx, ncclGroupEnd());
#ifdef KCC_DIAG_INLIB_COMM
    // the drill (variant builds only): a corrupted all-reduce result on the last device
    if (std::getenv("KCC_DRILL_CORRUPT_ALLREDUCE")) {
      Dev& dv = ctx->devs[nd - 1];
      KCC_HIP(ctx, hipSetDevice(dv.device));
      KCC_HIP(ctx, hipMemsetAsync(dv.partial.p, 0x5a, 8, dv.stream));
    }
#endif
    if (verify) {
      for (int d = 0; d < nd; ++d) {
        Dev& dv = ctx->devs[d];
        KCC_HIP(ctx, hipSetDevice(dv.device));
        KCC_HIP(ctx, hipMemcpyAsync(got.data(), dv.partial.p, 8 * words, hipMemcpyDeviceToHost,
                                    dv.stream));
        KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
        for (size_t i = 0; i < words; ++i)
          if (got[i] != expect[i])
            return fail(ctx, KCC_ERCCL,
                        "in-library all-reduce verification failed on device " +
                            std::to_string(dv.device) + ": word " + std::to_string(i) + " is " +
                            std::to_string(got[i]) + ", the host sum of the devices' partials " +
                            std::to_string(expect[i]) + "; results not returned");
      }
      ctx->allreduce_verified = true;
    }
  }
  Dev& d0 = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(d0.device));
  KCC_HIP(ctx, ensure(d0.totals, 8 * (size_t)n_specs));
  KCC_HIP(ctx, ensure(d0.err, 4 * (size_t)n_specs));
  int rc = fit_finalize_dev(ctx, d0, n_specs, as<int64_t>(d0.partial), as<int64_t>(d0.totals),
                            as<int32_t>(d0.err), d0.stream);
  if (rc) return rc;
  KCC_HIP(ctx, hipMemcpyAsync(totals, d0.totals.p, 8 * (size_t)n_specs, hipMemcpyDeviceToHost,
                              d0.stream));
  KCC_HIP(ctx, hipMemcpyAsync(spec_err, d0.err.p, 4 * (size_t)n_specs, hipMemcpyDeviceToHost,
                              d0.stream));
  unsigned long long slow_pairs = 0;
  for (int d = 0; d < nd; ++d) {
    Dev& dv = ctx->devs[d];
    KCC_HIP(ctx, hipSetDevice(dv.device));
    KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  }
  int64_t streamed = 0;
  for (int sh = 0; sh < ns; ++sh) {
    slow_pairs += ctx->host_cnt[(size_t)sh * kcc::CNT_N + kcc::CNT_SLOW_PAIRS];
    streamed += (int64_t)ctx->host_cnt[(size_t)sh * kcc::CNT_N + kcc::CNT_STREAM];
  }
  ctx->host_stream_rows = streamed;
  const double pairs = (double)n_nodes * (double)n_specs;
  ctx->slow_frac = pairs > 0 ? (double)slow_pairs / pairs : 0.0;
  return check_faults(ctx);
}

}  // namespace

extern "C" {

int kcc_abi_version(void) { return KCC_ABI_VERSION; }

int kcc_set_allreduce_verify(kcc_ctx* ctx, int every_call) {
  if (!ctx) return KCC_EINVAL;
  ctx->allreduce_verify_every = every_call != 0;
  return KCC_OK;
}

// The knobs an experiment build was compiled with (csrc/Makefile `variant` passes them in
// KCC_VARIANT_FLAGS); the release library takes none (the Makefile refuses EXTRA there).
#ifdef KCC_VARIANT_BUILD
const char* kcc_build_info(void) { return "variant: " KCC_VARIANT_FLAGS; }
#else
const char* kcc_build_info(void) { return "release"; }
#endif

const char* kcc_create_error(void) { return g_create_error.c_str(); }

int kcc_create(kcc_ctx** out, int first_device, int n_gpus) {
  g_create_error.clear();
  if (!out) { g_create_error = "out is NULL"; return KCC_EINVAL; }
  *out = nullptr;
  if (n_gpus <= 0 || first_device < 0) {
    g_create_error = "n_gpus must be >= 1 and first_device >= 0 (there is no CPU backend)";
    return KCC_EINVAL;
  }
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    g_create_error = std::string("no HIP device: ") + hipGetErrorString(e);
    return KCC_ENODEV;
  }
  if (first_device + n_gpus > count) {
    g_create_error = "requested devices [" + std::to_string(first_device) + ", " +
                     std::to_string(first_device + n_gpus) + ") but only " +
                     std::to_string(count) + " visible";
    return KCC_ENODEV;
  }
  kcc_ctx* ctx = new kcc_ctx();
  ctx->devs.resize(n_gpus);
  std::vector<int> ids(n_gpus);
  for (int d = 0; d < n_gpus; ++d) {
    Dev& dv = ctx->devs[d];
    dv.device = first_device + d;
    ids[d] = dv.device;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, dv.device)) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      g_create_error = "device " + std::to_string(dv.device) + " is not gfx950 (" +
                       (e == hipSuccess ? std::string(prop.gcnArchName)
                                        : std::string(hipGetErrorString(e))) +
                       "): libkcc is built for MI355X only";
      kcc_destroy(ctx);
      return KCC_ENODEV;
    }
    if ((e = hipSetDevice(dv.device)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&dv.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&dv.side, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&dv.ev_fork, hipEventDisableTiming)) != hipSuccess) {
      g_create_error = std::string("stream creation failed: ") + hipGetErrorString(e);
      kcc_destroy(ctx);
      return KCC_EHIP;
    }
  }
#ifdef KCC_DIAG_INLIB_COMM
  const bool inlib_comm = true;  // (variant builds: one device goes through RCCL too)
#else
  const bool inlib_comm = n_gpus > 1;
#endif
  if (inlib_comm) {
    ctx->comms.resize(n_gpus);
    ncclResult_t r = ncclCommInitAll(ctx->comms.data(), n_gpus, ids.data());
    if (r != ncclSuccess) {
      ctx->comms.clear();
      g_create_error = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
      kcc_destroy(ctx);
      return KCC_ERCCL;
    }
  }
  *out = ctx;
  return KCC_OK;
}

void kcc_destroy(kcc_ctx* ctx) {
  if (!ctx) return;
  for (auto& c : ctx->comms) ncclCommDestroy(c);
  if (ctx->proc_comm) {
    (void)hipSetDevice(ctx->devs[0].device);
    (void)hipDeviceSynchronize();  // its all-reduces ran on caller streams
    ncclCommDestroy(ctx->proc_comm);
  }
  for (Dev& dv : ctx->devs) {
    (void)hipSetDevice(dv.device);
    if (dv.stream) (void)hipStreamSynchronize(dv.stream);
    if (dv.p2p_W > 0) {
      (void)hipDeviceSynchronize();  // exchanges ran on caller streams
      for (int p = 0; p < dv.p2p_W; ++p)
        if (p != dv.p2p_rank && dv.p2p_peer[p]) (void)hipIpcCloseMemHandle(dv.p2p_peer[p]);
      DevBuf* pb[] = {&dv.p2p_mbox, &dv.p2p_arrive};
      for (DevBuf* b : pb)
        if (b->p) (void)hipFree(b->p);
    }
    if (dv.clamp_arrive.p) (void)hipFree(dv.clamp_arrive.p);
    if (dv.np_sync.p) (void)hipFree(dv.np_sync.p);
    DevBuf* bufs[] = {&dv.c_rank, &dv.c_bcnt, &dv.c_cs, &dv.c_ms,
                      &dv.c_mrc, &dv.c_crm, &dv.c_dperm, &dv.c_C, &dv.c_H2, &dv.c_H3,
                      &dv.c_Crow, &dv.c_rec, &dv.c_dir,
                      &dv.red_tail,  &dv.faults, &dv.rank_arrive, &dv.fast_cl, &dv.slow_list, &dv.fast_a, &dv.fast_b, &dv.slow, &dv.srec,
                      &dv.sperm,     &dv.fit_q,
                      &dv.counters,  &dv.ptr,       &dv.cpu,       &dv.mem,       &dv.cpul,
                      &dv.meml,      &dv.used_cpu,  &dv.used_mem,  &dv.lim_cpu,   &dv.lim_mem,
                      &dv.alloc_cpu, &dv.alloc_mem, &dv.alloc_pods, &dv.pod_count, &dv.spec_cpu,
                      &dv.spec_mem,  &dv.partial,   &dv.totals,    &dv.err,
                      &dv.p_bytes,   &dv.p_off,     &dv.p_out,     &dv.p_st,      &dv.k_key,
                      &dv.kb_counts, &dv.kb_tot,    &dv.kb_sr,     &dv.kb_sv,     &dv.q_ptr,
                      &dv.kb_part,   &dv.kb_arrive,
                      &dv.kb_esc_n,  &dv.kb_esc_row, &dv.kb_esc_cpu, &dv.kb_esc_mem,
                      &dv.q_iptr,    &dv.q_icpu,    &dv.q_imem,    &dv.q_rst,     &dv.q_ocpu,
                      &dv.q_omem,    &dv.q_pcpu,    &dv.q_pmem};
    for (DevBuf* b : bufs)
      if (b->p) (void)hipFree(b->p);
    if (dv.stream) (void)hipStreamDestroy(dv.stream);
    if (dv.side) {
      (void)hipStreamSynchronize(dv.side);
      (void)hipStreamDestroy(dv.side);
    }
    if (dv.ev_fork) (void)hipEventDestroy(dv.ev_fork);
    for (hipEvent_t ev : dv.ev_red)
      if (ev) (void)hipEventDestroy(ev);
    for (const ProfPair& pp : dv.prof_pending) {
      (void)hipEventDestroy(pp.a);
      (void)hipEventDestroy(pp.b);
    }
    for (hipEvent_t ev : dv.prof_free) (void)hipEventDestroy(ev);
  }
  if (ctx->host_cnt) (void)hipHostFree(ctx->host_cnt);
  delete ctx;
}

const char* kcc_last_error(const kcc_ctx* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

int kcc_reserve(kcc_ctx* ctx, int64_t max_nodes, int64_t max_containers, int64_t max_specs) {
  if (!ctx) return KCC_EINVAL;
  if (max_nodes < 0 || max_containers < 0 || max_specs < 0)
    return fail(ctx, KCC_EINVAL, "negative size");
  return reserve_dev(ctx, ctx->devs[0], max_nodes, max_containers, max_specs);
}

int kcc_reduce_requests_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                              const int64_t* d_node_ptr, const uint64_t* d_cpu_req,
                              const int64_t* d_mem_req, const uint64_t* d_cpu_lim,
                              const int64_t* d_mem_lim, uint64_t* d_used_cpu,
                              int64_t* d_used_mem, uint64_t* d_lim_cpu, int64_t* d_lim_mem,
                              void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return reduce_async_dev(ctx, dv, n_nodes, n_containers, d_node_ptr, d_cpu_req, d_mem_req,
                          d_cpu_lim, d_mem_lim, d_used_cpu, d_used_mem, d_lim_cpu, d_lim_mem,
                          static_cast<hipStream_t>(stream));
}

int kcc_reduce_requests(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                        const int64_t* node_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
                        const uint64_t* cpu_lim, const int64_t* mem_lim, uint64_t* used_cpu,
                        int64_t* used_mem, uint64_t* lim_cpu, int64_t* lim_mem) {
  if (!ctx) return KCC_EINVAL;
  int rc = check_csr(ctx, n_nodes, n_containers, node_ptr);
  if (rc) return rc;
  if (n_nodes == 0) return KCC_OK;
  if (!used_cpu || !used_mem) return fail(ctx, KCC_EINVAL, "NULL output");
  if (n_containers > 0 && (!cpu_req || !mem_req)) return fail(ctx, KCC_EINVAL, "NULL container array");
  const bool lim = cpu_lim != nullptr || mem_lim != nullptr;
  if (lim && (!cpu_lim || !mem_lim || !lim_cpu || !lim_mem))
    return fail(ctx, KCC_EINVAL, "limits need cpu_lim, mem_lim, lim_cpu and lim_mem");
  // the reduce is cheap next to the fit: run it on the first device
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  if ((rc = h2d(ctx, dv, dv.ptr, node_ptr, n_nodes + 1))) return rc;
  if ((rc = h2d(ctx, dv, dv.cpu, cpu_req, n_containers))) return rc;
  if ((rc = h2d(ctx, dv, dv.mem, mem_req, n_containers))) return rc;
  if (lim) {
    if ((rc = h2d(ctx, dv, dv.cpul, cpu_lim, n_containers))) return rc;
    if ((rc = h2d(ctx, dv, dv.meml, mem_lim, n_containers))) return rc;
    KCC_HIP(ctx, ensure(dv.lim_cpu, 8 * (size_t)n_nodes));
    KCC_HIP(ctx, ensure(dv.lim_mem, 8 * (size_t)n_nodes));
  }
  KCC_HIP(ctx, ensure(dv.used_cpu, 8 * (size_t)n_nodes));
  KCC_HIP(ctx, ensure(dv.used_mem, 8 * (size_t)n_nodes));
  rc = reduce_async_dev(ctx, dv, n_nodes, n_containers, as<int64_t>(dv.ptr), as<uint64_t>(dv.cpu),
                        as<int64_t>(dv.mem), lim ? as<uint64_t>(dv.cpul) : nullptr,
                        lim ? as<int64_t>(dv.meml) : nullptr, as<uint64_t>(dv.used_cpu),
                        as<int64_t>(dv.used_mem), lim ? as<uint64_t>(dv.lim_cpu) : nullptr,
                        lim ? as<int64_t>(dv.lim_mem) : nullptr, dv.stream);
  if (rc) return rc;
  KCC_HIP(ctx, hipMemcpyAsync(used_cpu, dv.used_cpu.p, 8 * (size_t)n_nodes,
                              hipMemcpyDeviceToHost, dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(used_mem, dv.used_mem.p, 8 * (size_t)n_nodes,
                              hipMemcpyDeviceToHost, dv.stream));
  if (lim) {
    KCC_HIP(ctx, hipMemcpyAsync(lim_cpu, dv.lim_cpu.p, 8 * (size_t)n_nodes,
                                hipMemcpyDeviceToHost, dv.stream));
    KCC_HIP(ctx, hipMemcpyAsync(lim_mem, dv.lim_mem.p, 8 * (size_t)n_nodes,
                                hipMemcpyDeviceToHost, dv.stream));
  }
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return check_faults(ctx);
}

int kcc_fit(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
            const int64_t* alloc_pods, const int64_t* pod_count, const uint64_t* used_cpu,
            const int64_t* used_mem, int64_t n_specs, const uint64_t* spec_cpu,
            const int64_t* spec_mem, int64_t* totals, int32_t* spec_err) {
  if (!ctx) return KCC_EINVAL;
  return run_host(ctx, false, n_nodes, 0, nullptr, nullptr, nullptr, alloc_cpu, alloc_mem,
                  alloc_pods, pod_count, used_cpu, used_mem, n_specs, spec_cpu, spec_mem, totals,
                  spec_err);
}

int kcc_capacity(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers, const int64_t* node_ptr,
                 const uint64_t* cpu_req, const int64_t* mem_req, const uint64_t* alloc_cpu,
                 const int64_t* alloc_mem, const int64_t* alloc_pods, const int64_t* pod_count,
                 int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
                 int64_t* totals, int32_t* spec_err) {
  if (!ctx) return KCC_EINVAL;
  return run_host(ctx, true, n_nodes, n_containers, node_ptr, cpu_req, mem_req, alloc_cpu,
                  alloc_mem, alloc_pods, pod_count, nullptr, nullptr, n_specs, spec_cpu, spec_mem,
                  totals, spec_err);
}

int kcc_fit_partial_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                          const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                          const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                          const int64_t* d_used_mem, int64_t n_specs, const uint64_t* d_spec_cpu,
                          const int64_t* d_spec_mem, int64_t* d_partial, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return fit_partial_dev(ctx, dv, n_nodes, d_alloc_cpu, d_alloc_mem, d_alloc_pods, d_pod_count,
                         d_used_cpu, d_used_mem, n_specs, d_spec_cpu, d_spec_mem, d_partial,
                         static_cast<hipStream_t>(stream));
}

int kcc_fit_prepare_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                          const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                          const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                          const int64_t* d_used_mem, int64_t n_specs, const uint64_t* d_spec_cpu,
                          const int64_t* d_spec_mem, int64_t* d_partial, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return fit_prepare_dev(ctx, dv, n_nodes, d_alloc_cpu, d_alloc_mem, d_alloc_pods, d_pod_count,
                         d_used_cpu, d_used_mem, n_specs, d_spec_cpu, d_spec_mem, d_partial,
                         static_cast<hipStream_t>(stream));
}

int kcc_fit_run_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_specs, int64_t* d_partial,
                      void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return fit_run_dev(ctx, dv, n_nodes, n_specs, d_partial, static_cast<hipStream_t>(stream));
}

int kcc_fit_finalize_async(kcc_ctx* ctx, int64_t n_specs, const int64_t* d_partial,
                           int64_t* d_totals, int32_t* d_spec_err, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return fit_finalize_dev(ctx, dv, n_specs, d_partial, d_totals, d_spec_err,
                          static_cast<hipStream_t>(stream));
}

int kcc_fit_async(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* d_alloc_cpu,
                  const int64_t* d_alloc_mem, const int64_t* d_alloc_pods,
                  const int64_t* d_pod_count, const uint64_t* d_used_cpu,
                  const int64_t* d_used_mem, int64_t n_specs, const uint64_t* d_spec_cpu,
                  const int64_t* d_spec_mem, int64_t* d_totals, int32_t* d_spec_err,
                  void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, ensure(dv.partial, sizeof(int64_t) * 2 * (size_t)(n_specs > 0 ? n_specs : 1)));
  const hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = fit_partial_dev(ctx, dv, n_nodes, d_alloc_cpu, d_alloc_mem, d_alloc_pods, d_pod_count,
                           d_used_cpu, d_used_mem, n_specs, d_spec_cpu, d_spec_mem,
                           as<int64_t>(dv.partial), s);
  if (rc) return rc;
  return fit_finalize_dev(ctx, dv, n_specs, as<int64_t>(dv.partial), d_totals, d_spec_err, s);
}

int kcc_capacity_partial_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                               const int64_t* h_node_ptr, const int64_t* d_node_ptr,
                               const uint64_t* d_cpu_req, const int64_t* d_mem_req,
                               const uint64_t* d_alloc_cpu, const int64_t* d_alloc_mem,
                               const int64_t* d_alloc_pods, const int64_t* d_pod_count,
                               uint64_t* d_used_cpu, int64_t* d_used_mem, int64_t n_specs,
                               const uint64_t* d_spec_cpu, const int64_t* d_spec_mem,
                               int64_t* d_partial, int n_chunks, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return capacity_partial_dev(ctx, dv, n_nodes, n_containers, h_node_ptr, d_node_ptr, d_cpu_req,
                              d_mem_req, d_alloc_cpu, d_alloc_mem, d_alloc_pods, d_pod_count,
                              d_used_cpu, d_used_mem, n_specs, d_spec_cpu, d_spec_mem, d_partial,
                              n_chunks, static_cast<hipStream_t>(stream));
}

int kcc_capacity_async(kcc_ctx* ctx, int64_t n_nodes, int64_t n_containers,
                       const int64_t* h_node_ptr, const int64_t* d_node_ptr,
                       const uint64_t* d_cpu_req, const int64_t* d_mem_req,
                       const uint64_t* d_alloc_cpu, const int64_t* d_alloc_mem,
                       const int64_t* d_alloc_pods, const int64_t* d_pod_count,
                       uint64_t* d_used_cpu, int64_t* d_used_mem, int64_t n_specs,
                       const uint64_t* d_spec_cpu, const int64_t* d_spec_mem, int64_t* d_totals,
                       int32_t* d_spec_err, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  if (n_specs > 0 && (!d_totals || !d_spec_err)) return fail(ctx, KCC_EINVAL, "NULL totals/err");
  KCC_HIP(ctx, ensure(dv.partial, sizeof(int64_t) * 2 * (size_t)(n_specs > 0 ? n_specs : 1)));
  return capacity_partial_dev(ctx, dv, n_nodes, n_containers, h_node_ptr, d_node_ptr, d_cpu_req,
                              d_mem_req, d_alloc_cpu, d_alloc_mem, d_alloc_pods, d_pod_count,
                              d_used_cpu, d_used_mem, n_specs, d_spec_cpu, d_spec_mem,
                              as<int64_t>(dv.partial), 1, static_cast<hipStream_t>(stream),
                              d_totals, d_spec_err);
}

int kcc_profile_enable(kcc_ctx* ctx, int on) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, hipDeviceSynchronize());
  for (const ProfPair& pp : dv.prof_pending) {
    dv.prof_free.push_back(pp.a);
    dv.prof_free.push_back(pp.b);
  }
  dv.prof_pending.clear();
  dv.prof_on = on != 0;
  dv.prof_ms[0] = dv.prof_ms[1] = 0.0;
  dv.prof_n[0] = dv.prof_n[1] = 0;
  return KCC_OK;
}

int kcc_profile_read(kcc_ctx* ctx, double* reduce_ms, int64_t* reduce_launches, double* fit_ms,
                     int64_t* fit_launches) {
  if (!ctx) return KCC_EINVAL;
  if (!reduce_ms || !reduce_launches || !fit_ms || !fit_launches)
    return fail(ctx, KCC_EINVAL, "NULL output");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  for (const ProfPair& pp : dv.prof_pending) {
    KCC_HIP(ctx, hipEventSynchronize(pp.b));
    float ms = 0.0f;
    KCC_HIP(ctx, hipEventElapsedTime(&ms, pp.a, pp.b));
    dv.prof_ms[pp.kind] += ms;
    dv.prof_n[pp.kind] += 1;
    dv.prof_free.push_back(pp.a);
    dv.prof_free.push_back(pp.b);
  }
  dv.prof_pending.clear();
  *reduce_ms = dv.prof_ms[0];
  *reduce_launches = dv.prof_n[0];
  *fit_ms = dv.prof_ms[1];
  *fit_launches = dv.prof_n[1];
  return KCC_OK;
}

double kcc_last_slow_fraction(const kcc_ctx* ctx) { return ctx ? ctx->slow_frac : -1.0; }

int kcc_fit_slow_pairs(kcc_ctx* ctx, int64_t* slow_pairs, int64_t* pairs) {
  if (!ctx || !slow_pairs || !pairs) return ctx ? fail(ctx, KCC_EINVAL, "NULL output") : KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, hipDeviceSynchronize());
  unsigned long long c = 0;
  if (dv.counters.p) KCC_HIP(ctx, hipMemcpy(&c, dv.counters.p, sizeof(c), hipMemcpyDeviceToHost));
  *slow_pairs = (int64_t)c;
  *pairs = dv.last_pairs;
  return KCC_OK;
}

int kcc_set_fit_dense(kcc_ctx* ctx, int dense) {
  if (!ctx) return KCC_EINVAL;
  for (Dev& dv : ctx->devs) dv.fit_dense = dense != 0;
  return KCC_OK;
}

int kcc_clamp_in_fit_used(kcc_ctx* ctx, int* used) {
  if (!ctx || !used) return KCC_EINVAL;
  *used = 0;
  for (const Dev& dv : ctx->devs) *used |= dv.last_nc ? 1 : 0;
  return KCC_OK;
}

int kcc_set_clamp_in_fit(kcc_ctx* ctx, int mode) {
  if (!ctx) return KCC_EINVAL;
  if (mode < -1 || mode > 1) return fail(ctx, KCC_EINVAL, "mode: -1 (by size), 0 or 1");
  for (Dev& dv : ctx->devs) dv.clamp_in_fit = mode;
  return KCC_OK;
}

int kcc_fit_stream_rows(kcc_ctx* ctx, int64_t* streamed) {
  if (!ctx || !streamed) return ctx ? fail(ctx, KCC_EINVAL, "NULL output") : KCC_EINVAL;
  if (ctx->host_stream_rows >= 0) {  // the last fit was kcc_fit / kcc_capacity: every shard
    *streamed = ctx->host_stream_rows;
    return KCC_OK;
  }
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, hipDeviceSynchronize());
  unsigned long long c[kcc::CNT_N] = {};
  if (dv.counters.p)
    KCC_HIP(ctx, hipMemcpy(c, dv.counters.p, sizeof(c), hipMemcpyDeviceToHost));
  int64_t t = 0;
  for (int k = 0; k < dv.stream_chunks && k < kcc::FIT_MAX_CHUNKS; ++k) t += (int64_t)c[kcc::CNT_STREAM + k];
  *streamed = t;
  return KCC_OK;
}

int kcc_reduce_faults(kcc_ctx* ctx, int64_t* faults) {
  if (!ctx || !faults) return ctx ? fail(ctx, KCC_EINVAL, "NULL output") : KCC_EINVAL;
  int64_t t = 0;
  for (Dev& dv : ctx->devs) {
    if (!dv.faults.p) continue;
    KCC_HIP(ctx, hipSetDevice(dv.device));
    KCC_HIP(ctx, hipDeviceSynchronize());
    unsigned long long f = 0;
    KCC_HIP(ctx, hipMemcpy(&f, as<unsigned long long>(dv.faults) + kcc::FAULT_RED, sizeof(f),
                           hipMemcpyDeviceToHost));
    t += (int64_t)f;
  }
  *faults = t;
  return KCC_OK;
}

int kcc_clear_faults(kcc_ctx* ctx) {
  if (!ctx) return KCC_EINVAL;
  for (Dev& dv : ctx->devs) {
    KCC_HIP(ctx, hipSetDevice(dv.device));
    KCC_HIP(ctx, hipDeviceSynchronize());
    if (dv.faults.p) KCC_HIP(ctx, hipMemset(dv.faults.p, 0, dv.faults.bytes));
    // a wait that gave up left its record published: every tag back to free
    if (dv.red_tail.p) KCC_HIP(ctx, hipMemset(dv.red_tail.p, 0, dv.red_tail.bytes));
    // and every counter a launch leaves zero: a gather part that gave up can have
    // published its ready count after the last part reset it
    for (DevBuf* b : {&dv.kb_arrive, &dv.rank_arrive, &dv.fit_q, &dv.clamp_arrive})
      if (b->p) KCC_HIP(ctx, hipMemset(b->p, 0, b->bytes));
    KCC_HIP(ctx, hipDeviceSynchronize());
  }
  return KCC_OK;
}

int kcc_set_node_shards(kcc_ctx* ctx, int n_shards) {
  if (!ctx) return KCC_EINVAL;
  if (n_shards < 0) return fail(ctx, KCC_EINVAL, "n_shards must be >= 0");
  ctx->node_shards = n_shards;
  return KCC_OK;
}

// ---- one rank of a multi-process run (one process per GPU) --------------------------

int kcc_comm_unique_id(uint8_t* id) {
  if (!id) return KCC_EINVAL;
  static_assert(sizeof(ncclUniqueId) == KCC_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return KCC_ERCCL;
  std::memcpy(id, &u, sizeof(u));
  return KCC_OK;
}

int kcc_comm_init(kcc_ctx* ctx, const uint8_t* id, int n_ranks, int rank) {
  if (!ctx) return KCC_EINVAL;
  if (!id || n_ranks < 1 || rank < 0 || rank >= n_ranks)
    return fail(ctx, KCC_EINVAL, "need an id, n_ranks >= 1 and 0 <= rank < n_ranks");
  if (ctx->devs.size() != 1)
    return fail(ctx, KCC_EINVAL, "a multi-process rank drives exactly one device");
  if (ctx->proc_comm) return fail(ctx, KCC_EINVAL, "communicator already initialised");
  KCC_HIP(ctx, hipSetDevice(ctx->devs[0].device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  KCC_NCCL(ctx, ncclCommInitRank(&ctx->proc_comm, n_ranks, u, rank));
  ctx->proc_ranks = n_ranks;
  ctx->proc_rank = rank;
  return KCC_OK;
}

int kcc_allreduce_partial_async(kcc_ctx* ctx, int64_t n_specs, int64_t* d_partial, void* stream) {
  if (!ctx) return KCC_EINVAL;
  if (n_specs < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (!ctx->proc_comm) return fail(ctx, KCC_EINVAL, "no communicator (kcc_comm_init)");
  if (n_specs == 0) return KCC_OK;
  if (!d_partial) return fail(ctx, KCC_EINVAL, "NULL partial");
  KCC_HIP(ctx, hipSetDevice(ctx->devs[0].device));
  KCC_NCCL(ctx, ncclAllReduce(d_partial, d_partial, 2 * (size_t)n_specs, ncclInt64, ncclSum,
                              ctx->proc_comm, static_cast<hipStream_t>(stream)));
  return KCC_OK;
}

// ---- one-shot exchange over xGMI peer memory (kcc_p2p_*) ---------------------------

int kcc_p2p_export(kcc_ctx* ctx, int n_ranks, int64_t max_specs, uint8_t* handle) {
  if (!ctx) return KCC_EINVAL;
  if (!handle || n_ranks < 1 || n_ranks > kcc::P2P_MAX_RANKS || max_specs < 1 ||
      max_specs > KCC_P2P_MAX_SPECS)
    return fail(ctx, KCC_EINVAL, "need a handle buffer, 1 <= n_ranks <= 8, 1 <= max_specs <= 2^20");
  if (ctx->devs.size() != 1)
    return fail(ctx, KCC_EINVAL, "a multi-process rank drives exactly one device");
  Dev& dv = ctx->devs[0];
  if (dv.p2p_W > 0) return fail(ctx, KCC_EINVAL, "mailbox already exported");
  KCC_HIP(ctx, hipSetDevice(dv.device));
  const size_t bytes = kcc::p2p_mbox_bytes(n_ranks, max_specs);
  {
    int rc = faults_ws(ctx, dv, dv.stream);
    if (rc) return rc;
  }
  KCC_HIP(ctx, ensure_uncached(dv.p2p_mbox, bytes));
  KCC_HIP(ctx, ensure(dv.p2p_arrive, 64));
  KCC_HIP(ctx, hipMemset(dv.p2p_mbox.p, 0, bytes));  // flags 0: no epoch seen
  KCC_HIP(ctx, hipMemset(dv.p2p_arrive.p, 0, 64));   // no arrivals, epoch 0 pushed
  KCC_HIP(ctx, hipDeviceSynchronize());
  static_assert(sizeof(hipIpcMemHandle_t) == KCC_P2P_HANDLE_BYTES, "IPC handle size");
  hipIpcMemHandle_t h;
  KCC_HIP(ctx, hipIpcGetMemHandle(&h, dv.p2p_mbox.p));
  std::memcpy(handle, &h, sizeof(h));
  dv.p2p_W = n_ranks;
  dv.p2p_smax = max_specs;
  return KCC_OK;
}

int kcc_p2p_open(kcc_ctx* ctx, int rank, const uint8_t* handles) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  if (dv.p2p_W == 0) return fail(ctx, KCC_EINVAL, "kcc_p2p_export first");
  if (dv.p2p_ready) return fail(ctx, KCC_EINVAL, "peers already opened");
  if (!handles || rank < 0 || rank >= dv.p2p_W) return fail(ctx, KCC_EINVAL, "need handles and 0 <= rank < n_ranks");
  KCC_HIP(ctx, hipSetDevice(dv.device));
  for (int p = 0; p < dv.p2p_W; ++p) {
    if (p == rank) {
      dv.p2p_peer[p] = static_cast<unsigned char*>(dv.p2p_mbox.p);
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles + (size_t)p * KCC_P2P_HANDLE_BYTES, sizeof(h));
    void* ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      for (int q = 0; q < p; ++q)
        if (q != rank && dv.p2p_peer[q]) (void)hipIpcCloseMemHandle(dv.p2p_peer[q]);
      for (auto& q : dv.p2p_peer) q = nullptr;
      return fail(ctx, KCC_EHIP, std::string("hipIpcOpenMemHandle(rank ") + std::to_string(p) +
                                     "): " + hipGetErrorString(e));
    }
    dv.p2p_peer[p] = static_cast<unsigned char*>(ptr);
  }
  dv.p2p_rank = rank;
  dv.p2p_ready = true;
  return KCC_OK;
}

int kcc_exchange_finalize_async(kcc_ctx* ctx, int64_t n_specs, const int64_t* d_partial,
                                int64_t* d_totals, int32_t* d_spec_err, void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  if (!dv.p2p_ready) return fail(ctx, KCC_EINVAL, "no peers (kcc_p2p_export + kcc_p2p_open)");
  if (n_specs < 0 || n_specs > dv.p2p_smax)
    return fail(ctx, KCC_EINVAL, "n_specs outside [0, the mailbox's max_specs]");
  if (n_specs == 0) return KCC_OK;
  if (!d_partial || !d_totals || !d_spec_err) return fail(ctx, KCC_EINVAL, "NULL partial/totals/err");
  if (dv.sperm.bytes < sizeof(int32_t) * (size_t)n_specs)
    return fail(ctx, KCC_EINVAL, "exchange without a matching fit_partial");
  KCC_HIP(ctx, hipSetDevice(dv.device));
  kcc::P2PArgs a{};
  a.S = n_specs;
  a.smax = dv.p2p_smax;
  a.W = dv.p2p_W;
  a.rank = dv.p2p_rank;
  a.epoch = as<uint64_t>(dv.p2p_arrive) + 1;  // (word 0: the arrival counter)
  a.partial = d_partial;
  for (int p = 0; p < dv.p2p_W; ++p) a.mbox[p] = dv.p2p_peer[p];
  a.perm = as<int32_t>(dv.sperm);
  a.totals = d_totals;
  a.spec_err = d_spec_err;
  a.arrive = as<uint32_t>(dv.p2p_arrive);
  a.faults = as<unsigned long long>(dv.faults);
  KCC_HIP(ctx, kcc::launch_exchange_finalize(a, static_cast<hipStream_t>(stream)));
  return KCC_OK;
}

int kcc_p2p_faults(kcc_ctx* ctx, int64_t* faults) {
  if (!ctx || !faults) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  *faults = 0;
  if (!dv.faults.p) return KCC_OK;
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, hipDeviceSynchronize());
  unsigned long long f = 0;
  KCC_HIP(ctx, hipMemcpy(&f, as<unsigned long long>(dv.faults) + kcc::FAULT_P2P, sizeof(f),
                         hipMemcpyDeviceToHost));
  *faults = (int64_t)f;
  return KCC_OK;
}

}  // extern "C"


// ---- quantity-string parse --------------------------------------

namespace {

int parse_async_dev(kcc_ctx* ctx, int mode, int64_t n, const char* bytes, int64_t n_bytes,
                    const int64_t* offsets, int64_t* out, int8_t* status, hipStream_t s) {
  if (n < 0 || n_bytes < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n == 0) return KCC_OK;
  if (!offsets || !out || !status || (n_bytes > 0 && !bytes))
    return fail(ctx, KCC_EINVAL, "NULL bytes/offsets/out/status");
  if ((reinterpret_cast<uintptr_t>(bytes) & 3u) != 0)
    return fail(ctx, KCC_EINVAL, "bytes must be 4-byte aligned");
  KCC_HIP(ctx, kcc::launch_parse(mode, n, reinterpret_cast<const uint8_t*>(bytes), n_bytes,
                                 offsets, out, status, s));
  return KCC_OK;
}

int parse_host(kcc_ctx* ctx, int mode, int64_t n, const char* bytes, int64_t n_bytes,
               const int64_t* offsets, int64_t* out, int8_t* status) {
  if (!ctx) return KCC_EINVAL;
  if (n < 0 || n_bytes < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n == 0) return KCC_OK;
  if (!offsets || !out || !status || (n_bytes > 0 && !bytes))
    return fail(ctx, KCC_EINVAL, "NULL bytes/offsets/out/status");
  if (offsets[0] < 0 || offsets[n] > n_bytes)
    return fail(ctx, KCC_EINVAL, "offsets outside [0, n_bytes]");
  for (int64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return fail(ctx, KCC_EINVAL, "offsets are not non-decreasing");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  int rc;
  if ((rc = h2d(ctx, dv, dv.p_bytes, bytes, n_bytes))) return rc;
  if ((rc = h2d(ctx, dv, dv.p_off, offsets, n + 1))) return rc;
  KCC_HIP(ctx, ensure(dv.p_out, 8 * (size_t)n));
  KCC_HIP(ctx, ensure(dv.p_st, (size_t)n));
  rc = parse_async_dev(ctx, mode, n, as<char>(dv.p_bytes), n_bytes, as<int64_t>(dv.p_off),
                       as<int64_t>(dv.p_out), as<int8_t>(dv.p_st), dv.stream);
  if (rc) return rc;
  KCC_HIP(ctx, hipMemcpyAsync(out, dv.p_out.p, 8 * (size_t)n, hipMemcpyDeviceToHost, dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(status, dv.p_st.p, (size_t)n, hipMemcpyDeviceToHost, dv.stream));
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return KCC_OK;
}

}  // namespace

int kcc_parse_cpu_millis(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                         const int64_t* offsets, uint64_t* out, int8_t* status) {
  return parse_host(ctx, kcc::PARSE_MODE_CPU_MILLIS, n, bytes, n_bytes, offsets,
                    reinterpret_cast<int64_t*>(out), status);
}

int kcc_parse_bytes(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                    const int64_t* offsets, int64_t* out, int8_t* status) {
  return parse_host(ctx, kcc::PARSE_MODE_BYTES, n, bytes, n_bytes, offsets, out, status);
}

int kcc_parse_quantity(kcc_ctx* ctx, int64_t n, const char* bytes, int64_t n_bytes,
                       const int64_t* offsets, int64_t* out, int8_t* status) {
  return parse_host(ctx, kcc::PARSE_MODE_QUANTITY, n, bytes, n_bytes, offsets, out, status);
}

int kcc_parse_quantity_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                             const int64_t* d_offsets, int64_t* d_out, int8_t* d_status,
                             void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return parse_async_dev(ctx, kcc::PARSE_MODE_QUANTITY, n, d_bytes, n_bytes, d_offsets, d_out,
                         d_status, static_cast<hipStream_t>(stream));
}

int kcc_parse_cpu_millis_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                               const int64_t* d_offsets, uint64_t* d_out, int8_t* d_status,
                               void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return parse_async_dev(ctx, kcc::PARSE_MODE_CPU_MILLIS, n, d_bytes, n_bytes, d_offsets,
                         reinterpret_cast<int64_t*>(d_out), d_status,
                         static_cast<hipStream_t>(stream));
}

int kcc_parse_bytes_async(kcc_ctx* ctx, int64_t n, const char* d_bytes, int64_t n_bytes,
                          const int64_t* d_offsets, int64_t* d_out, int8_t* d_status,
                          void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return parse_async_dev(ctx, kcc::PARSE_MODE_BYTES, n, d_bytes, n_bytes, d_offsets, d_out,
                         d_status, static_cast<hipStream_t>(stream));
}


// ---- list-order (keyed) reduce ------------------------------------

namespace {

// Workspace of the bucketed keyed reduce (grows on demand); nullptr when the keys do not
// fit the bucketed path (the kernels then fall back to device atomics).
int keyed_work(kcc_ctx* ctx, Dev& dv, int64_t n_keys, int64_t n, int na, kcc::KeyedWork& kw,
               const kcc::KeyedWork** out) {
  *out = nullptr;
  if (!kcc::keyed_bucketed(n_keys, n)) return KCC_OK;
  {
    int rc = faults_ws(ctx, dv, dv.stream);  // (the gather's bounded wait reports here)
    if (rc) return rc;
  }
  const size_t nb = (size_t)kcc::keyed_buckets(n_keys);
  const size_t m = (size_t)(n > 0 ? n : 1);
  KCC_HIP(ctx, ensure(dv.kb_counts, 4 * (size_t)kcc::keyed_counts_words(n_keys, n)));
  KCC_HIP(ctx, ensure(dv.kb_tot, 4 * nb));
  KCC_HIP(ctx, ensure(dv.kb_sr, 8 * (size_t)kcc::keyed_sr_slots(n)));
  KCC_HIP(ctx, ensure(dv.kb_part, 8 * (size_t)kcc::keyed_part_words(n_keys, na > 2 ? 2 : na)));
  if (dv.kb_arrive.bytes < 8 * nb) {  // [arrivals | published parts]: every gather leaves them zero
    KCC_HIP(ctx, ensure(dv.kb_arrive, 8 * nb));
    KCC_HIP(ctx, hipMemsetAsync(dv.kb_arrive.p, 0, dv.kb_arrive.bytes, dv.stream));
    KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  }
  if (na > 2) KCC_HIP(ctx, ensure(dv.kb_sv, 8 * (size_t)(na - 2) * m));
  if (na >= 2) {
    const size_t ne = (size_t)(n > 0 ? n : 1);
    if (!dv.kb_esc_n.p) {  // [0] list length, [1] kb_escape's arrivals: zero between calls
      KCC_HIP(ctx, ensure(dv.kb_esc_n, 16));
      KCC_HIP(ctx, hipMemsetAsync(dv.kb_esc_n.p, 0, 16, dv.stream));
      KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
    }
    KCC_HIP(ctx, ensure(dv.kb_esc_row, 4 * ne));
    KCC_HIP(ctx, ensure(dv.kb_esc_cpu, 8 * ne));
    KCC_HIP(ctx, ensure(dv.kb_esc_mem, 8 * ne));
  }
  kw.counts = as<uint32_t>(dv.kb_counts);
  kw.tot = as<uint32_t>(dv.kb_tot);
  kw.sr = as<uint64_t>(dv.kb_sr);
  kw.sv = na > 2 ? as<uint64_t>(dv.kb_sv) : nullptr;
  kw.esc_n = na >= 2 ? as<uint32_t>(dv.kb_esc_n) : nullptr;
  kw.esc_row = na >= 2 ? as<int32_t>(dv.kb_esc_row) : nullptr;
  kw.esc_cpu = na >= 2 ? as<uint64_t>(dv.kb_esc_cpu) : nullptr;
  kw.esc_mem = na >= 2 ? as<uint64_t>(dv.kb_esc_mem) : nullptr;
  kw.part_acc = as<uint64_t>(dv.kb_part);
  kw.arrive = as<uint32_t>(dv.kb_arrive);
  kw.faults = as<unsigned long long>(dv.faults);
  *out = &kw;
  return KCC_OK;
}

int keyed_async_dev(kcc_ctx* ctx, int64_t n_keys, int64_t n, const int32_t* key,
                    const uint64_t* cpu, const int64_t* mem, const uint64_t* cpul,
                    const int64_t* meml, uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                    int64_t* lim_mem, hipStream_t s) {
  if (n_keys < 0 || n < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_keys > 0x7fffffff) return fail(ctx, KCC_EINVAL, "more than 2^31 - 1 keys");
  if (n_keys > 0 && (!used_cpu || !used_mem)) return fail(ctx, KCC_EINVAL, "NULL output");
  if (n > 0 && (!key || !cpu || !mem)) return fail(ctx, KCC_EINVAL, "NULL key/cpu_req/mem_req");
  const bool lim = cpul != nullptr || meml != nullptr;
  if (lim && (!cpul || !meml || (n_keys > 0 && (!lim_cpu || !lim_mem))))
    return fail(ctx, KCC_EINVAL, "limits need cpu_lim, mem_lim, lim_cpu and lim_mem");
  if (!aligned16(key) || !aligned16(cpu) || !aligned16(mem) ||
      (lim && (!aligned16(cpul) || !aligned16(meml))))
    return fail(ctx, KCC_EINVAL, "key and container arrays must be 16-byte aligned");
  Dev& dv = ctx->devs[0];
  kcc::KeyedWork kw{};
  const kcc::KeyedWork* kwp = nullptr;
  int rc = keyed_work(ctx, dv, n_keys, n, lim ? 4 : 2, kw, &kwp);
  if (rc) return rc;
  KCC_HIP(ctx, kcc::launch_reduce_keyed(n_keys, n, key, cpu, mem, lim ? cpul : nullptr,
                                        lim ? meml : nullptr, used_cpu, used_mem,
                                        lim ? lim_cpu : nullptr, lim ? lim_mem : nullptr, kwp, s));
  return KCC_OK;
}

}  // namespace

extern "C" {

int kcc_reduce_requests_keyed_async(kcc_ctx* ctx, int64_t n_keys, int64_t n_containers,
                                    const int32_t* d_key, const uint64_t* d_cpu_req,
                                    const int64_t* d_mem_req, const uint64_t* d_cpu_lim,
                                    const int64_t* d_mem_lim, uint64_t* d_used_cpu,
                                    int64_t* d_used_mem, uint64_t* d_lim_cpu, int64_t* d_lim_mem,
                                    void* stream) {
  if (!ctx) return KCC_EINVAL;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  return keyed_async_dev(ctx, n_keys, n_containers, d_key, d_cpu_req, d_mem_req, d_cpu_lim,
                         d_mem_lim, d_used_cpu, d_used_mem, d_lim_cpu, d_lim_mem,
                         static_cast<hipStream_t>(stream));
}

int kcc_reduce_requests_keyed(kcc_ctx* ctx, int64_t n_keys, int64_t n_containers,
                              const int32_t* key, const uint64_t* cpu_req, const int64_t* mem_req,
                              const uint64_t* cpu_lim, const int64_t* mem_lim,
                              uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                              int64_t* lim_mem) {
  if (!ctx) return KCC_EINVAL;
  if (n_keys < 0 || n_containers < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_keys > 0 && (!used_cpu || !used_mem)) return fail(ctx, KCC_EINVAL, "NULL output");
  if (n_containers > 0 && (!key || !cpu_req || !mem_req))
    return fail(ctx, KCC_EINVAL, "NULL key/cpu_req/mem_req");
  const bool lim = cpu_lim != nullptr || mem_lim != nullptr;
  if (lim && (!cpu_lim || !mem_lim || (n_keys > 0 && (!lim_cpu || !lim_mem))))
    return fail(ctx, KCC_EINVAL, "limits need cpu_lim, mem_lim, lim_cpu and lim_mem");
  if (n_keys == 0) return KCC_OK;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  int rc;
  if ((rc = h2d(ctx, dv, dv.k_key, key, n_containers))) return rc;
  if ((rc = h2d(ctx, dv, dv.cpu, cpu_req, n_containers))) return rc;
  if ((rc = h2d(ctx, dv, dv.mem, mem_req, n_containers))) return rc;
  if (lim) {
    if ((rc = h2d(ctx, dv, dv.cpul, cpu_lim, n_containers))) return rc;
    if ((rc = h2d(ctx, dv, dv.meml, mem_lim, n_containers))) return rc;
    KCC_HIP(ctx, ensure(dv.lim_cpu, 8 * (size_t)n_keys));
    KCC_HIP(ctx, ensure(dv.lim_mem, 8 * (size_t)n_keys));
  }
  KCC_HIP(ctx, ensure(dv.used_cpu, 8 * (size_t)n_keys));
  KCC_HIP(ctx, ensure(dv.used_mem, 8 * (size_t)n_keys));
  rc = keyed_async_dev(ctx, n_keys, n_containers, as<int32_t>(dv.k_key), as<uint64_t>(dv.cpu),
                       as<int64_t>(dv.mem), lim ? as<uint64_t>(dv.cpul) : nullptr,
                       lim ? as<int64_t>(dv.meml) : nullptr, as<uint64_t>(dv.used_cpu),
                       as<int64_t>(dv.used_mem), lim ? as<uint64_t>(dv.lim_cpu) : nullptr,
                       lim ? as<int64_t>(dv.lim_mem) : nullptr, dv.stream);
  if (rc) return rc;
  KCC_HIP(ctx, hipMemcpyAsync(used_cpu, dv.used_cpu.p, 8 * (size_t)n_keys, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(used_mem, dv.used_mem.p, 8 * (size_t)n_keys, hipMemcpyDeviceToHost,
                              dv.stream));
  if (lim) {
    KCC_HIP(ctx, hipMemcpyAsync(lim_cpu, dv.lim_cpu.p, 8 * (size_t)n_keys,
                                hipMemcpyDeviceToHost, dv.stream));
    KCC_HIP(ctx, hipMemcpyAsync(lim_mem, dv.lim_mem.p, 8 * (size_t)n_keys,
                                hipMemcpyDeviceToHost, dv.stream));
  }
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return check_faults(ctx);
}

int kcc_count_by_key_async(kcc_ctx* ctx, int64_t n_keys, int64_t n, const int32_t* d_key,
                           int64_t* d_count, void* stream) {
  if (!ctx) return KCC_EINVAL;
  if (n_keys < 0 || n < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_keys > 0x7fffffff) return fail(ctx, KCC_EINVAL, "more than 2^31 - 1 keys");
  if ((n_keys > 0 && !d_count) || (n > 0 && !d_key)) return fail(ctx, KCC_EINVAL, "NULL key/count");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  kcc::KeyedWork kw{};
  const kcc::KeyedWork* kwp = nullptr;
  int rc = keyed_work(ctx, dv, n_keys, n, 0, kw, &kwp);
  if (rc) return rc;
  KCC_HIP(ctx, kcc::launch_count_keyed(n_keys, n, d_key, d_count, kwp,
                                       static_cast<hipStream_t>(stream)));
  return KCC_OK;
}

int kcc_count_by_key(kcc_ctx* ctx, int64_t n_keys, int64_t n, const int32_t* key, int64_t* count) {
  if (!ctx) return KCC_EINVAL;
  if (n_keys < 0 || n < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if ((n_keys > 0 && !count) || (n > 0 && !key)) return fail(ctx, KCC_EINVAL, "NULL key/count");
  if (n_keys == 0) return KCC_OK;
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  int rc;
  if ((rc = h2d(ctx, dv, dv.k_key, key, n))) return rc;
  KCC_HIP(ctx, ensure(dv.pod_count, 8 * (size_t)n_keys));
  kcc::KeyedWork kw{};
  const kcc::KeyedWork* kwp = nullptr;
  if ((rc = keyed_work(ctx, dv, n_keys, n, 0, kw, &kwp))) return rc;
  KCC_HIP(ctx, kcc::launch_count_keyed(n_keys, n, as<int32_t>(dv.k_key), as<int64_t>(dv.pod_count),
                                       kwp, dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(count, dv.pod_count.p, 8 * (size_t)n_keys, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return check_faults(ctx);
}

}  // extern "C"


// ---- per-row q of one spec -----------------------------------------

extern "C" int kcc_fit_rows(kcc_ctx* ctx, int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, uint64_t spec_cpu, int64_t spec_mem,
                            int64_t* q, int32_t* row_err) {
  if (!ctx) return KCC_EINVAL;
  if (n_nodes < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_nodes == 0) return KCC_OK;
  if (!alloc_cpu || !alloc_mem || !alloc_pods || !pod_count || !used_cpu || !used_mem || !q ||
      !row_err)
    return fail(ctx, KCC_EINVAL, "NULL node array / output");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  int rc;
  if ((rc = h2d(ctx, dv, dv.alloc_cpu, alloc_cpu, n_nodes))) return rc;
  if ((rc = h2d(ctx, dv, dv.alloc_mem, alloc_mem, n_nodes))) return rc;
  if ((rc = h2d(ctx, dv, dv.alloc_pods, alloc_pods, n_nodes))) return rc;
  if ((rc = h2d(ctx, dv, dv.pod_count, pod_count, n_nodes))) return rc;
  if ((rc = h2d(ctx, dv, dv.used_cpu, used_cpu, n_nodes))) return rc;
  if ((rc = h2d(ctx, dv, dv.used_mem, used_mem, n_nodes))) return rc;
  KCC_HIP(ctx, ensure(dv.totals, 8 * (size_t)n_nodes));
  KCC_HIP(ctx, ensure(dv.err, 4 * (size_t)n_nodes));
  KCC_HIP(ctx, kcc::launch_fit_rows(n_nodes, as<uint64_t>(dv.alloc_cpu), as<int64_t>(dv.alloc_mem),
                                    as<int64_t>(dv.alloc_pods), as<int64_t>(dv.pod_count),
                                    as<uint64_t>(dv.used_cpu), as<int64_t>(dv.used_mem), spec_cpu,
                                    spec_mem, as<int64_t>(dv.totals), as<int32_t>(dv.err),
                                    dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(q, dv.totals.p, 8 * (size_t)n_nodes, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(row_err, dv.err.p, 4 * (size_t)n_nodes, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return KCC_OK;
}


// ---- opt-in scheduler request model (kcc_pods.hip) ------------------

namespace {

// Host-side checks shared by the two host-array entry points.
int check_pods(kcc_ctx* ctx, int64_t n_pods, int64_t n_cont, int64_t n_init,
               const int64_t* pod_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
               const int64_t* init_ptr, const uint64_t* init_cpu, const int64_t* init_mem,
               const uint8_t* restartable) {
  int rc = check_csr(ctx, n_pods, n_cont, pod_ptr);
  if (rc) return rc;
  if (n_cont > 0 && (!cpu_req || !mem_req)) return fail(ctx, KCC_EINVAL, "NULL cpu_req/mem_req");
  if (!init_ptr) {
    if (n_init != 0 || init_cpu || init_mem || restartable)
      return fail(ctx, KCC_EINVAL, "init container arrays without init_ptr");
    return KCC_OK;
  }
  if ((rc = check_csr(ctx, n_pods, n_init, init_ptr))) return rc;
  if (n_init > 0 && (!init_cpu || !init_mem)) return fail(ctx, KCC_EINVAL, "NULL init_cpu/init_mem");
  return KCC_OK;
}

// Stages the pod-level inputs and enqueues the per-pod kernel; pod outputs in q_pcpu/q_pmem.
int pods_stage_run(kcc_ctx* ctx, Dev& dv, int64_t n_pods, int64_t n_cont, int64_t n_init,
                   const int64_t* pod_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
                   const int64_t* init_ptr, const uint64_t* init_cpu, const int64_t* init_mem,
                   const uint8_t* restartable, const uint64_t* ovh_cpu, const int64_t* ovh_mem) {
  int rc;
  if ((rc = h2d(ctx, dv, dv.q_ptr, pod_ptr, n_pods + 1))) return rc;
  if ((rc = h2d(ctx, dv, dv.cpu, cpu_req, n_cont))) return rc;
  if ((rc = h2d(ctx, dv, dv.mem, mem_req, n_cont))) return rc;
  if (init_ptr) {
    if ((rc = h2d(ctx, dv, dv.q_iptr, init_ptr, n_pods + 1))) return rc;
    if ((rc = h2d(ctx, dv, dv.q_icpu, init_cpu, n_init))) return rc;
    if ((rc = h2d(ctx, dv, dv.q_imem, init_mem, n_init))) return rc;
    if (restartable && (rc = h2d(ctx, dv, dv.q_rst, restartable, n_init))) return rc;
  }
  if (ovh_cpu && (rc = h2d(ctx, dv, dv.q_ocpu, ovh_cpu, n_pods))) return rc;
  if (ovh_mem && (rc = h2d(ctx, dv, dv.q_omem, ovh_mem, n_pods))) return rc;
  KCC_HIP(ctx, ensure(dv.q_pcpu, 8 * (size_t)n_pods));
  KCC_HIP(ctx, ensure(dv.q_pmem, 8 * (size_t)n_pods));
  KCC_HIP(ctx, kcc::launch_pod_requests(
                   n_pods, n_cont, init_ptr ? n_init : 0, as<int64_t>(dv.q_ptr),
                   as<uint64_t>(dv.cpu), as<int64_t>(dv.mem),
                   init_ptr ? as<int64_t>(dv.q_iptr) : nullptr,
                   init_ptr ? as<uint64_t>(dv.q_icpu) : nullptr,
                   init_ptr ? as<int64_t>(dv.q_imem) : nullptr,
                   init_ptr && restartable ? as<uint8_t>(dv.q_rst) : nullptr,
                   ovh_cpu ? as<uint64_t>(dv.q_ocpu) : nullptr,
                   ovh_mem ? as<int64_t>(dv.q_omem) : nullptr, as<uint64_t>(dv.q_pcpu),
                   as<int64_t>(dv.q_pmem), dv.stream));
  return KCC_OK;
}

}  // namespace

extern "C" {

int kcc_pod_requests_async(kcc_ctx* ctx, int64_t n_pods, int64_t n_containers, int64_t n_init,
                           const int64_t* d_pod_ptr, const uint64_t* d_cpu_req,
                           const int64_t* d_mem_req, const int64_t* d_init_ptr,
                           const uint64_t* d_init_cpu, const int64_t* d_init_mem,
                           const uint8_t* d_restartable, const uint64_t* d_ovh_cpu,
                           const int64_t* d_ovh_mem, uint64_t* d_pod_cpu, int64_t* d_pod_mem,
                           void* stream) {
  if (!ctx) return KCC_EINVAL;
  if (n_pods < 0 || n_containers < 0 || n_init < 0) return fail(ctx, KCC_EINVAL, "negative size");
  if (n_pods == 0) return KCC_OK;
  if (!d_pod_ptr || !d_pod_cpu || !d_pod_mem) return fail(ctx, KCC_EINVAL, "NULL pod_ptr/output");
  if (n_containers > 0 && (!d_cpu_req || !d_mem_req))
    return fail(ctx, KCC_EINVAL, "NULL cpu_req/mem_req");
  if (d_init_ptr && n_init > 0 && (!d_init_cpu || !d_init_mem))
    return fail(ctx, KCC_EINVAL, "NULL init_cpu/init_mem");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  KCC_HIP(ctx, kcc::launch_pod_requests(n_pods, n_containers, d_init_ptr ? n_init : 0, d_pod_ptr,
                                        d_cpu_req, d_mem_req, d_init_ptr, d_init_cpu, d_init_mem,
                                        d_init_ptr ? d_restartable : nullptr, d_ovh_cpu,
                                        d_ovh_mem, d_pod_cpu, d_pod_mem,
                                        static_cast<hipStream_t>(stream)));
  return KCC_OK;
}

int kcc_pod_requests(kcc_ctx* ctx, int64_t n_pods, int64_t n_containers, int64_t n_init,
                     const int64_t* pod_ptr, const uint64_t* cpu_req, const int64_t* mem_req,
                     const int64_t* init_ptr, const uint64_t* init_cpu, const int64_t* init_mem,
                     const uint8_t* restartable, const uint64_t* ovh_cpu,
                     const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem) {
  if (!ctx) return KCC_EINVAL;
  if (n_init < 0) return fail(ctx, KCC_EINVAL, "negative size");
  int rc = check_pods(ctx, n_pods, n_containers, n_init, pod_ptr, cpu_req, mem_req, init_ptr,
                      init_cpu, init_mem, restartable);
  if (rc) return rc;
  if (n_pods == 0) return KCC_OK;
  if (!pod_cpu || !pod_mem) return fail(ctx, KCC_EINVAL, "NULL output");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  if ((rc = pods_stage_run(ctx, dv, n_pods, n_containers, n_init, pod_ptr, cpu_req, mem_req,
                           init_ptr, init_cpu, init_mem, restartable, ovh_cpu, ovh_mem)))
    return rc;
  KCC_HIP(ctx, hipMemcpyAsync(pod_cpu, dv.q_pcpu.p, 8 * (size_t)n_pods, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(pod_mem, dv.q_pmem.p, 8 * (size_t)n_pods, hipMemcpyDeviceToHost,
                              dv.stream));
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return KCC_OK;
}

int kcc_reduce_requests_pods(kcc_ctx* ctx, int64_t n_nodes, int64_t n_pods,
                             int64_t n_containers, int64_t n_init, const int64_t* node_pod_ptr,
                             const int64_t* pod_ptr, const uint64_t* cpu_req,
                             const int64_t* mem_req, const int64_t* init_ptr,
                             const uint64_t* init_cpu, const int64_t* init_mem,
                             const uint8_t* restartable, const uint64_t* ovh_cpu,
                             const int64_t* ovh_mem, uint64_t* used_cpu, int64_t* used_mem) {
  if (!ctx) return KCC_EINVAL;
  if (n_init < 0) return fail(ctx, KCC_EINVAL, "negative size");
  int rc = check_csr(ctx, n_nodes, n_pods, node_pod_ptr);
  if (rc) return rc;
  if ((rc = check_pods(ctx, n_pods, n_containers, n_init, pod_ptr, cpu_req, mem_req, init_ptr,
                       init_cpu, init_mem, restartable)))
    return rc;
  if (n_nodes == 0) return KCC_OK;
  if (!used_cpu || !used_mem) return fail(ctx, KCC_EINVAL, "NULL output");
  Dev& dv = ctx->devs[0];
  KCC_HIP(ctx, hipSetDevice(dv.device));
  if ((rc = h2d(ctx, dv, dv.ptr, node_pod_ptr, n_nodes + 1))) return rc;
  if (n_pods > 0 &&
      (rc = pods_stage_run(ctx, dv, n_pods, n_containers, n_init, pod_ptr, cpu_req, mem_req,
                           init_ptr, init_cpu, init_mem, restartable, ovh_cpu, ovh_mem)))
    return rc;
  KCC_HIP(ctx, ensure(dv.q_pcpu, 8 * (size_t)(n_pods > 0 ? n_pods : 1)));
  KCC_HIP(ctx, ensure(dv.q_pmem, 8 * (size_t)(n_pods > 0 ? n_pods : 1)));
  KCC_HIP(ctx, ensure(dv.used_cpu, 8 * (size_t)n_nodes));
  KCC_HIP(ctx, ensure(dv.used_mem, 8 * (size_t)n_nodes));
  // the pods of each node are the "containers" of the ordinary segmented reduce
  rc = reduce_async_dev(ctx, dv, n_nodes, n_pods, as<int64_t>(dv.ptr), as<uint64_t>(dv.q_pcpu),
                        as<int64_t>(dv.q_pmem), nullptr, nullptr, as<uint64_t>(dv.used_cpu),
                        as<int64_t>(dv.used_mem), nullptr, nullptr, dv.stream);
  if (rc) return rc;
  KCC_HIP(ctx, hipMemcpyAsync(used_cpu, dv.used_cpu.p, 8 * (size_t)n_nodes,
                              hipMemcpyDeviceToHost, dv.stream));
  KCC_HIP(ctx, hipMemcpyAsync(used_mem, dv.used_mem.p, 8 * (size_t)n_nodes,
                              hipMemcpyDeviceToHost, dv.stream));
  KCC_HIP(ctx, hipStreamSynchronize(dv.stream));
  return check_faults(ctx);
}

}  // extern "C"
