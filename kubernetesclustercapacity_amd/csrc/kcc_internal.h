// kcc_internal.h — launch interface between the C-ABI layer (kcc_abi.cpp) and the
// gfx950 kernels (kcc_kernels.hip).  Internal: not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic knobs produce wrong results by design (no stores, loads only), add stamp
// stores, or make every bounded wait give up (the fault-path test build): only experiment
// builds (csrc/Makefile `variant` / `faultdiag`, which define KCC_VARIANT_BUILD and write a
// separate .so) may set them.  The tuning choices are constants here: the variants that
// lost their A/B were deleted (DESIGN.md §10 lists them with their numbers and commits).
#if !defined(KCC_VARIANT_BUILD) &&                                                       \
    (defined(KCC_DIAG_RED_NOSTORE) || defined(KCC_DIAG_RED_LOADONLY) ||                  \
     defined(KCC_TIMELINE) || defined(KCC_DIAG_RED_GIVEUP) || defined(KCC_DIAG_P2P_GIVEUP) || \
     defined(KCC_DIAG_INLIB_COMM) || defined(KCC_DIAG_GA_NOATOM) ||                     \
     defined(KCC_DIAG_NP_NOSYNC) || defined(KCC_DIAG_NP_NOSC1))
#error "a diagnostic KCC_* knob in a release build: use `make variant` (KCC_VARIANT_BUILD)"
#endif

namespace kcc {

struct RankArgs;   // below: spec ranks, run as extra workgroups of a reduce launch
struct NpArgs;     // below: node prep (clamp in the fit) behind a reduce launch's workgroups

// ---- (a) segmented request reduce -------------------------------------------
// One wavefront owns a contiguous range of reduce_range() containers and walks it in
// tiles of RED_TILE (RED_IPL containers per lane: two 16-B loads per lane per array).
// The launch is self-contained (no marking pass, no zeroing, no atomics): a wave finds
// the node owning its first container by a 64-ary search of the CSR offsets, stores
// every node that ends inside its range, and a node cut by range boundaries is
// assembled by the wave where it ends from the pieces its predecessors publish
// (decoupled look-back over per-wave tail records: each record is published at most once
// per launch and consumed by exactly one wave, which clears its tag — every tag is 0
// between launches, so nothing in the launch depends on host state and a captured graph
// replays correctly).
// tiles in flight ahead of the one being reduced (1-6 measured equal: ping-pong)
constexpr int RED_PREFETCH = 1;
// containers per lane per tile: 8 halves the per-tile work (scan, node walk, stores) per
// container against 4, at 125 VGPRs (4 waves per SIMD instead of 6): C4 reduce 136.4 ->
// 131.1 us, 8-way shard 20.2 -> 19.5 us (A/B in one process, outputs identical)
constexpr int RED_IPL = 8;
constexpr int RED_TILE = 64 * RED_IPL;  // 512
constexpr int RED_WAVES_PER_BLOCK = 4;
// the reduce stores through 32-bit buffer offsets (8 B per node, < 2^31)
constexpr int64_t RED_MAX_NODES = (int64_t)1 << 28;
// per-wave tail record: the NA values of the node open at the range end, then the tag
constexpr int RED_TAIL_WORDS = 8;  // 64 B: one line per wave
constexpr int RED_TAIL_TAG = 7;
constexpr uint64_t RED_TAG_READY = 1;  // published (0: free; the consumer clears it)

// Device fault words (one 64-B line per device, zero until a wait gives up; sticky until
// kcc_clear_faults): the reduce's look-back waits and the exchange's flag waits that gave
// up.  Every finalize reads them and marks every spec KCC_SPEC_FAULT while either is set,
// and the synchronous entry points return KCC_EFAULT.
enum { FAULT_RED = 0, FAULT_P2P = 1, FAULT_WORDS = 8 };
constexpr int32_t SPEC_ERR_DIV0 = 1;   // include/kcc.h KCC_SPEC_DIVZERO
constexpr int32_t SPEC_ERR_FAULT = 2;  // include/kcc.h KCC_SPEC_FAULT
// The fault travels with the data: a fit launched while its device is faulted adds
// SPEC_FAULT_MARK to every spec's div-by-zero count in partial[S..2S), once per spec, so
// every consumer of the partial — this device's finalize, the p2p exchange, an RCCL or
// torch.distributed all-reduce summed into another rank's finalize, the in-library device
// fold — sees a count >= SPEC_FAULT_MARK and marks the spec KCC_SPEC_FAULT.  Real counts
// are < 2^28 per device (one per node row); the marks of up to 2^14 launches x ranks sum
// without wrapping.
constexpr uint64_t SPEC_FAULT_MARK = 1ull << 48;

// Containers per wave range: whole tiles, sized so the waves fill the device's resident
// wave slots (occupancy API) in KCC_RED_ROUNDS rounds: one round of equal, long ranges
// leaves no half-empty second round (9672 waves of 4096 containers at C4 ran 1.6 rounds
// of 6144 resident waves).  Small inputs get one tile per wave.  `limits` selects the
// 4-array kernel (more registers, fewer resident waves).
// reserve_waves: resident wave slots left to other work of the same launch (the spec
// rank workgroups in front of the reduce's)
int32_t reduce_range(int64_t n_containers, bool limits, int64_t reserve_waves = 0);
inline int64_t reduce_n_waves(int64_t n_containers, bool limits, int64_t reserve_waves = 0) {
  const int64_t r = reduce_range(n_containers, limits, reserve_waves);
  return (n_containers + r - 1) / r;
}
// tail records a launch may need: an upper bound of reduce_n_waves (one range per
// resident wave slot at most)
int64_t reduce_tail_records();

// One reduce launch: nodes [0, n_nodes) of `ptr` (the caller offsets ptr and the
// per-node outputs for a node range) and containers [c0, c_end); the offsets in ptr and
// the container arrays stay absolute (ptr[0] == c0), so a node range of one CSR is
// reduced without rebasing anything.  Every output of [0, n_nodes) is written.
struct RedArgs {
  int64_t n_nodes, c0, c_end;
  int32_t range;
  const int64_t* ptr;
  const uint64_t* in[4];
  uint64_t* out[4];
  uint64_t* tail;                  // [reduce_tail_records()][RED_TAIL_WORDS], tags 0
  unsigned long long* faults;      // the device's fault words (FAULT_RED: look-back give-ups)
  int32_t ranks_last;              // the spec ranks' workgroups behind the reduce's (else in front)
};
// rank != nullptr (with rank->n_blocks > 0): the spec ranks run as that many extra
// workgroups beside the reduce's (independent work, one launch fewer per step): behind them
// on long reduces (>= KCC_RED_RANKS_LAST_MIN containers: they take the slots of the first
// waves to finish; C4 step 0.3059 -> 0.3030 ms), in front on short ones (the 8-way C4 rank:
// behind, they lengthened its 23 us reduce by 3 us).
hipError_t launch_reduce(int64_t n_nodes, int64_t c0, int64_t n_containers, const int64_t* node_ptr,
                         const uint64_t* cpu_req, const int64_t* mem_req,
                         const uint64_t* cpu_lim, const int64_t* mem_lim,
                         uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu, int64_t* lim_mem,
                         uint64_t* tail, unsigned long long* faults, hipStream_t s,
                         const RankArgs* rank = nullptr, const NpArgs* np = nullptr,
                         hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
// (ev_start / ev_stop, kcc_profile_*: the kernel's own dispatch timestamps, hipExtLaunchKernel —
// event packets around the launch also timed the dispatch, ~3 us per launch)

// ---- (b) fit -----------------------------------------------------------------
// Node streams of the fit kernel: groups of FIT_GROUP nodes, field-major inside the
// group.  The per-node values arrive through the scalar cache and feed the VALU as
// SGPR operands.  The fast loops sum min(findMin(qc, qm), P) — the pod-slot clamp
// itself (CC:134-136) is added back per spec by the clamp correction (ClampWork).
// Rows outside the fast-path bounds, and the padding of the last group, hold all-zero
// fields (they contribute exactly 0) and are listed in slow_list for the exact path.
//
// FitGroupA — class-A spec waves: the integers themselves, which the
// VALU reads as IEEE denormals (an integer k < 2^23 is the f32 bit pattern of
// k * 2^-149, k < 2^52 the f64 pattern of k * 2^-1074).
constexpr int FIT_GROUP = 8;
struct __attribute__((aligned(32))) FitGroupA {
  uint64_t fm[FIT_GROUP];  // free memory (bytes), < 2^50
  uint32_t fc[FIT_GROUP];  // free CPU (millicores), < 2^23
  uint32_t P[FIT_GROUP];   // max(allocatable pods, 0), <= 2^20
};
static_assert(sizeof(FitGroupA) == 128, "FitGroupA must be 128 B");
// FitGroup — class-B spec waves (memory request < 2^18): f64 values for the biased
// FMA path; written by node_prep only when such specs exist.
constexpr double FIT_BIAS = 4503599627370496.0;  // 2^52: integers in [2^52, 2^53) have ulp 1
struct __attribute__((aligned(32))) FitGroup {
  double fc[FIT_GROUP];  // free CPU (millicores), exact in f64
  double fm[FIT_GROUP];  // free memory (bytes), exact in f64
  double Pb[FIT_GROUP];  // 2^52 + max(allocatable pods, 0) (<= 2^20: exact)
};
static_assert(sizeof(FitGroup) == 192, "FitGroup must be 192 B");
__host__ __device__ inline int64_t fit_groups(int64_t n_nodes) { return (n_nodes + FIT_GROUP - 1) / FIT_GROUP; }

// Raw per-node values for the exact path (fc/fm are 0 where the reference's
// `alloc <= used` branch yields 0, i.e. no division happens).
struct __attribute__((aligned(32))) SlowNode {
  uint64_t fc;
  int64_t fm;
  int64_t P;
  int64_t cl;
};
static_assert(sizeof(SlowNode) == 32, "SlowNode must be 32 B");

// One 48-B record per spec, in the kernel's internal (partitioned) order: class A
// first, then B, then the exact-path specs (so at most two wavefronts mix classes;
// a wave runs the most general class among its lanes).
enum SpecClass : int32_t { SPEC_A = 0, SPEC_B = 1, SPEC_EXACT = 2 };
struct __attribute__((aligned(16))) SpecRec {
  uint64_t c;    // cpu request (millicores)
  int64_t m;     // memory request (bytes)
  double rc;     // smallest f64 >= 1/c (classes A, B)
  double rm;     // smallest f64 >= 1/m (classes A, B)
  float rcf;     // smallest f32 >= 1/c (class A)
  int32_t cls;   // SpecClass
  int64_t pad;
};
static_assert(sizeof(SpecRec) == 48, "SpecRec must be 48 B");

struct SpecPrep {
  SpecRec* rec;    // by internal position
  int32_t* perm;   // internal index -> caller index
};

// Clamp correction.  On the fast paths the fit kernel sums
// min(findMin(qc, qm), P) and leaves out the pod-slot clamp of CC:134-136; the clamp is
// added back per spec as  partial[s] -= D_s,  D_s = Σ_i w_i [x_is >= P_i],  w_i = P_i - cl_i
// (the pod count; for P_i <= 0 rows, clamped for every spec, w_i = -cl_i).  For P_i >= 1,
// x_is >= P_i  <=>  c_s <= U_i = fc_i / P_i  and  m_s <= V_i = fm_i / P_i  (integer
// quotients): a 2-D dominance sum.  The nN normal specs (classes A and B) get an x-rank by
// (c, index) and a y-rank by (m, index) (permutations of 0..nN-1); row i dominates exactly
// the specs with x < L_i = #{c <= U_i} and y < b_i = #{m <= V_i}.  Both axes are cut into
// blocks of 64 ranks (T = ceil(nN / 64)):
//   - coarse: C[L_i >> 6][b_i >> 6] += w_i, a (T+2) x (T+2) table (P <= 0 rows in cell
//     [T+1][T+1]); spec s collects Σ_{GX > x_s>>6, GY > y_s>>6} C;
//   - x-group: the rows with L_i >> 6 == g, r = L_i & 63 > 0, in H2[g][k][r] with
//     k = #{specs of x-group g with y < b_i}; spec s (x-group g) collects
//     Σ_{k > kpos_s, r > x_s & 63} H2[g][k][r], kpos_s = #{specs of x-group g, y < y_s};
//   - y-block: the rows with b_i >> 6 == Y, r = b_i & 63 > 0, L_i >> 6 > 0, in H3[Y][j][r]
//     with j = #{specs of y-block Y whose x-group < L_i >> 6}; spec s collects
//     Σ_{j > jpos_s, r > y_s & 63} H3[Y][j][r], jpos_s = #{specs of y-block Y, x < x_s}.
// All tables are O(S) (the tables of round 1 grew as S^2/64: 270 MB at S = 16384).  C has
// one copy per XCD, H2/H3 two (node_prep's atomics spread over more cache lines); every
// copy is zero between calls: clamp_prep zeroes what it reads.
struct ClampWork {
  uint32_t* rank;    // [rank_words(S)] by caller index: x-ranks [0, S), y-ranks [S, 2S),
                     // then each slice's share of the x-rank and the y-rank
  uint32_t* bcnt;    // [ceil(S/64)][2] class A / class B specs per block of 64 (caller order)
  uint64_t* cs;      // [S] normal specs' cpu requests by x-rank (ascending)
  int64_t* ms;       // [S] memory requests by y-rank (ascending)
  uint32_t* mr_c;    // [64 * T] y-rank by x-rank (padding 0xffffffff)
  uint32_t* cr_m;    // [64 * T] x-rank by y-rank (padding 0xffffffff)
  int32_t* dperm;    // [S] x-rank -> internal position
  int64_t* C;        // [C_COPIES][c_stride]: (T+2) x (T+2), cell GX * (T+2) + GY
  int64_t* H2;       // [H2_COPIES][h_stride]: T x 65 x 64, cell (g * 65 + k) * 64 + r
  int64_t* H3;       // [H2_COPIES][h_stride]: T x 65 x 64, cell (Y * 65 + j) * 64 + r
  int64_t* Crow;     // [c_stride]: C summed over the copies, suffix sums along GY
  // binned form of H2 / H3 (clamp_binned(S)): node_prep writes each pass's
  // (cell, w) records sorted by bin (x-group g: bin g; y-block Y: bin T + Y) into the
  // pass's own slot range, and the bins' starts into dir; clamp_apply's workgroup for a
  // bin sums that bin's records of every pass into LDS.  No global atomics.
  uint64_t* rec;     // [n_pass][pass_recs]: cell | (int32 w) << 32
  uint32_t* dir;     // [n_pass][d_stride]: a pass's bin starts (exclusive prefix) + its total
  int64_t c_stride;  // cells per C copy (clamp_c_cells(S) of the workspace)
  int64_t h_stride;  // cells per H2 / H3 copy (clamp_h_cells(S))
  int64_t d_stride;  // clamp_d_stride(S) of the workspace
  int64_t n_pass;    // passes of the call's node rows (set by launch_clamp_apply)
  int64_t pass_recs; // record slots per pass: 2 x clamp_pass_rows (set by launch_clamp_apply)
};
// specs per call
constexpr int64_t MAX_SPECS = (int64_t)1 << 26;
__host__ __device__ inline int64_t clamp_c_cells(int64_t S) { return (S / 64 + 3) * (S / 64 + 3); }
inline int64_t clamp_h_cells(int64_t S) { return (S / 64 + 1) * 65 * 64; }
// copies of the coarse table: node_prep flushes its LDS-summed table once per workgroup
// (S <= 4096), so two spread the flushes enough; clamp_apply's x-group workgroups read
// every copy (C4 8-way shard, fit prepare + run: 8 copies 60.4 us, 2: 58.2, 1: 58.5; C5's
// global-memory atomics need more than one: 544.8 / 545.5 / 557.8 us)
constexpr int C_COPIES = 2;
constexpr int H2_COPIES = 2;
// binned H2 / H3 (ClampWork::rec): node_prep's passes of clamp_pass_rows(n) rows (1 or 4
// per thread) emit at most one record of each table per row; up to CLAMP_BIN_T_MAX
// x-groups (S <= 16384), larger S adds to the H2 / H3 copies with device atomics
constexpr int CLAMP_PASS_ROWS_MIN = 1024;
constexpr int CLAMP_PASS_ROWS_MAX = 4096;  // chunks of a pipelined call are multiples of it
// Rows per node_prep pass for a call of n_nodes rows: 4096 when such passes still fill
// the chip (one node_prep workgroup per CU), else 1024 — 4x the workgroups on small
// shards (C4's 8-way shard: 123 instead of 31).  Fewer, larger passes keep clamp_apply's
// heavy bins cheap: a bin's records are read pass by pass, and at C4 one bin held 34k
// records (12.9 us to consume over 245 passes, 28.5 us over 977).
inline int64_t clamp_pass_rows(int64_t n_nodes) {
  return n_nodes >= (int64_t)200 * CLAMP_PASS_ROWS_MAX ? CLAMP_PASS_ROWS_MAX : CLAMP_PASS_ROWS_MIN;
}
constexpr int64_t CLAMP_BIN_T_MAX = 256;
__host__ __device__ inline bool clamp_binned(int64_t S) { return (S + 63) / 64 <= CLAMP_BIN_T_MAX; }
inline int64_t clamp_d_stride(int64_t S) { return 2 * ((S + 63) / 64) + 1; }
inline int64_t clamp_passes(int64_t n_nodes) {
  const int64_t pr = clamp_pass_rows(n_nodes);
  return (n_nodes + pr - 1) / pr;
}
// up to this many specs node_prep's search and count tables live in LDS; larger S
// searches the same tables in global memory
constexpr int64_t CLAMP_LDS_SPECS = 4096;

// Spec ranks (spec_rank): the x-rank by (c, index) and the y-rank by (m, index) of every
// normal spec, by sort and search: workgroup (query block of RANK_L, slice of RANK_L
// candidates), rank_slices(S)^2 workgroups; each sorts its slice's keys in registers and LDS
// and finds each query's count below it by binary search.  Each slice stores its x and y
// counts (rank[S + (slice * 2 + r) * S + i], write-through) and adds to its query block's
// arrival counter; the last slice to arrive (the counter's returned value) sums the
// slices and writes the sorted arrays itself — cs[x] = c, ms[y] = m, mr_c[x] = y,
// cr_m[y] = x — and rank[i] = x, rank[S + i] = y, then resets the counter.  The slice-0 workgroups store
// the class-A / class-B counts of each block of 64 queries (bcnt).  The rank workgroups
// also zero the counters (all but CNT_SPECS_A / CNT_SPECS_B, set by spec_place) and the
// coarse clamp table's cells: the first launch of a step, ahead of every reader.
constexpr int64_t RANK_L = 1024;         // candidates per slice: 16 KiB of 16-B keys
constexpr int64_t RANK_FULL_MAX = 4096;  // up to this S the ranks count (above: sort + search)
__host__ __device__ inline int64_t rank_slices(int64_t S) { return (S + RANK_L - 1) / RANK_L; }
// u32 words of ClampWork::rank for S specs: the x- and y-ranks, then the slices' counts
__host__ __device__ inline int64_t rank_words(int64_t S) { return 2 * S + 2 * S * rank_slices(S); }
struct RankArgs {
  int64_t S;
  const uint64_t* c_in;
  const int64_t* m_in;
  uint32_t* part;      // ClampWork::rank
  uint32_t* arrive;    // [rank_slices(S)] per query block: slices arrived (zero between calls)
  uint32_t* bcnt;      // ClampWork::bcnt
  uint64_t* cs;        // ClampWork::cs / ms / mr_c / cr_m
  int64_t* ms;
  uint32_t* mr_c;
  uint32_t* cr_m;
  int64_t* C;          // ClampWork::C: cells [0, c_cells) of each copy are zeroed
  int64_t c_stride, c_cells;
  unsigned long long* counters;
  int32_t n_blocks;    // 256-thread workgroups: rank_slices(S)^2 (0: none)
  // 1: the clamp in the fit needs no ranks — one workgroup that zeroes the counters and
  // writes the block class counts (bcnt) alone (PlaceArgs::no_ranks)
  int32_t zero_only;
  // zero_only with node prep in the same launch (NpArgs): the counters and bcnt written
  // through (sc1), then *done_flag = 1 for the node-prep workgroups
  uint32_t* done_flag;      // NpArgs::sync (the epoch at NP_EPOCH, the flag at NP_DONE)
};
RankArgs rank_args(int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
                   const ClampWork& cw, unsigned long long* counters, uint32_t* arrive,
                   bool zero_only = false);
hipError_t launch_spec_rank(const RankArgs& ra, hipStream_t s);

// spec_place's work (one thread per spec), run as extra workgroups in front of the
// node_prep launch (node_prep reads only the arrays spec_rank wrote, and not the padding
// spec_place writes): the stable 3-way partition position, the
// SpecRec / perm there, dperm, mr_c / cr_m's padding, partial[0..2S) zeroed,
// CNT_SPECS_A / CNT_SPECS_B set.
struct PlaceArgs {
  int64_t S;
  const uint64_t* c_in;
  const int64_t* m_in;
  SpecPrep sp;
  ClampWork cw;
  int64_t* partial;
  unsigned long long* counters;
  int32_t n_blocks;  // workgroups of the launch's block size (0: none)
  const unsigned long long* faults;  // set: partial[S + i] starts at SPEC_FAULT_MARK
  // 1 (the clamp in the fit, S <= CLAMP_LDS_SPECS): no spec ranks ran (only bcnt was
  // written): nothing rank-indexed is read or written
  int32_t no_ranks;
};


// Node prep of the clamp in the fit (one node chunk, S <= CLAMP_LDS_SPECS) as workgroups
// behind a reduce launch's (KCC_NP_IN_REDUCE): n_place workgroups of spec_place (after the
// zero_only rank workgroup's flag), then n_rows workgroups of 1024 rows each (node_prep's
// clamp-in-fit work, after every reduce wave has signalled).  The reduce's node sums go
// out write-through (sc1) and each reduce wave adds 1 to sync[16] when done (its stores
// performed); the node-prep workgroups read them at agent scope.  The last of them resets
// the sync words.  Dispatch order makes the waits safe: on every XCD all the reduce's
// workgroups are dispatched before any node-prep workgroup, and no reduce wave waits on
// one.  Every wait is bounded; a give-up counts in faults[FAULT_RED].
struct NpArgs {
  int32_t n_place, n_rows;  // workgroups (256 threads)
  uint32_t* sync;           // NP_EPOCH, NP_DONE, NP_ARRIVE, NP_FLAGS (reduce_tail_records() words)
  // set by launch_reduce: the reduce's CSR offsets, first container, range and wave count
  const int64_t* ptr;
  int64_t c0;
  int32_t range, red_waves;
  PlaceArgs pa;
  int64_t n;                // rows
  const uint64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int64_t* alloc_pods;
  const int64_t* pod_count;
  const uint64_t* used_cpu;
  const int64_t* used_mem;
  FitGroupA* fast_a;
  FitGroup* fast_b;
  SlowNode* slow;
  int64_t* slow_list;
  int32_t* fast_cl;
  unsigned long long* counters;
  const uint32_t* bcnt;
  int64_t S;
  unsigned long long* faults;
};
constexpr int NP_ROWS_PER_WG = 1024;  // 256 threads x 4 rows
// NpArgs::sync (uint32 words, 64-B lines): [NP_EPOCH] the last launch's epoch (a launch's
// epoch E is one past it; its last node-prep workgroup to finish publishes E), [NP_DONE]
// the spec ranks' done flag (= E), [NP_ARRIVE] the node-prep arrivals (zero between
// launches), then [NP_FLAGS + w] reduce wave w's flag (= E once its node sums are stored).
// Epoch flags need no reset, and a node-prep workgroup waits for the waves that store its
// rows alone: one counter of every wave's arrival took the ~3200 same-address atomics of
// the 8-way C4 rank serially (~25 ns apiece, 80 us)
constexpr int NP_EPOCH = 0, NP_DONE = 16, NP_ARRIVE = 32, NP_FLAGS = 64;

// counters (CNT_*): exact-path (node, spec) pairs, class-B specs, and per node chunk
// of a pipelined call (kcc_capacity_partial_async) the rows in that chunk's slow_list.
// spec_rank zeroes the counters, spec_place sets the class counts and zeroes
// partial[0..2S); node_prep appends to slow_list and the fit streams.
constexpr int FIT_MAX_CHUNKS = 16;
enum {
  CNT_SLOW_PAIRS = 0,  // (node, spec) pairs evaluated on the exact path
  CNT_SPECS_A = 1,     // class-A specs (internal positions [0, nA))
  CNT_SPECS_B = 2,     // class-B specs (internal positions [nA, nA + nB))
  CNT_CLAMP_ALL = 3,   // clamp in the fit: Σ (max(P, 0) - clamp) of the rows clamped for
                       // every spec (P <= 0), subtracted from every normal spec by the fit
  CNT_SLOW_ROWS = 4,   // + chunk: rows in that node chunk's slow_list
  CNT_STREAM = 4 + FIT_MAX_CHUNKS,  // + chunk: node rows in that chunk's fit stream (x 8)
  CNT_N = 4 + 2 * FIT_MAX_CHUNKS
};
// The clamp correction after every node_prep of the call (n_nodes: the call's rows, for
// the binned records' pass count): partial[s] -= D_s for the normal specs of clamp-free
// waves; leaves the table copies zero.
// fin != nullptr (one rank, the call's last kernel): the launch's last workgroup to finish
// (an arrival counter, zero between launches) also finalizes — totals[perm[i]] = err ? 0 :
// partial[i], spec_err[perm[i]] = err — instead of a fit_finalize launch.
struct FinArgs {
  const int32_t* perm;
  int64_t* totals;
  int32_t* spec_err;
  uint32_t* arrive;
  const unsigned long long* faults;  // the device's fault words: set -> KCC_SPEC_FAULT
};
hipError_t launch_clamp_apply(int64_t n_specs, int64_t n_nodes, ClampWork cw,
                              const unsigned long long* counters, int64_t* partial, hipStream_t s,
                              const FinArgs* fin = nullptr);
int64_t clamp_apply_blocks(int64_t n_specs);  // clamp_apply_kernel's grid
// the spec ranks' workgroups of a fused reduce launch go behind the reduce's workgroups on
// launches of at least this many containers, in front of them on shorter ones
constexpr int64_t RED_RANKS_LAST_MIN = (int64_t)16 << 20;

// The fit's node stream (FitGroupA / FitGroup records) holds the rows that can contribute
// to the fast sum Σ min(findMin(qc, qm), P): fast-bound rows with free CPU, free memory
// and P >= 1 (every other row adds exactly 0 there: qc = 0 or qm = 0 makes x = 0, and
// P <= 0 rows are the clamp correction's), compacted per workgroup pass into
// counters[CNT_STREAM + chunk] rows (padded to whole groups).  dense: stream every row (the
// round-1 layout's cost: zero fields for the rows that add nothing).  row0: the launch's
// first row within the call (a multiple of CLAMP_PASS_ROWS_MAX; the binned records'
// passes), call_nodes: the call's rows (its pass size, clamp_pass_rows).
// Needs the sorted spec arrays (spec_rank's) on the stream before it.  place != nullptr:
// spec_place runs as extra workgroups of this launch (place->n_blocks is set here).
hipError_t launch_node_prep(int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, FitGroupA* fast_a, FitGroup* fast_b,
                            SlowNode* slow, int64_t* slow_list, int64_t n_specs, ClampWork cw,
                            unsigned long long* counters, int chunk, int64_t row0,
                            int64_t call_nodes, hipStream_t s, bool dense = false,
                            const PlaceArgs* place = nullptr, int32_t* fast_cl = nullptr);
// Clamp in the fit (fast_cl != nullptr; one node chunk, S <= CLAMP_LDS_SPECS, not dense):
// node_prep streams each row's clamp value (allocatable pods - pod count, CC:135) beside
// its FitGroupA (fast_cl[row position]) and builds no clamp tables; the fit computes the
// reference's x >= P ? clamp : x itself (5 VALU per node x wave instead of 3) and
// subtracts counters[CNT_CLAMP_ALL] from every normal spec; no clamp_apply launch.  The
// choice for small shards, where clamp_apply's fixed cost exceeds the fit's extra issue.
// node rows x specs at most: the C4 8-way (5.1e8) and 4-way (1.0e9) shards
constexpr int64_t CLAMP_IN_FIT_PAIRS = 1100000000LL;
inline bool clamp_in_fit_auto(int64_t n_nodes, int64_t n_specs) {
  return n_specs <= CLAMP_LDS_SPECS && n_nodes * n_specs <= CLAMP_IN_FIT_PAIRS;
}

// partial[0..S) += Σ_i q(i,s), partial[S..2S) += #div-by-zero rows (internal order).
hipError_t launch_fit(int64_t n_nodes, const FitGroupA* fast_a, const FitGroup* fast_b,
                      const SlowNode* slow,
                      const int64_t* slow_list, int64_t n_specs, SpecPrep sp, int64_t* partial,
                      unsigned long long* counters, uint32_t* queue, int chunk,
                      int64_t grid_nodes, hipStream_t s, const unsigned long long* faults,
                      const int32_t* fast_cl = nullptr, hipEvent_t ev_start = nullptr,
                      hipEvent_t ev_stop = nullptr);
// the fit's work queues: fit_queue_words(S) uint32 (a 64-B line per spec column of 256 and
// sub-queue), zero before the first launch (each launch leaves them zero)
constexpr int64_t FIT_QSUBS_MAX = 32;
inline int64_t fit_queue_words(int64_t S) { return (S + 255) / 256 * FIT_QSUBS_MAX * 16; }

// totals[perm[i]] = err ? 0 : partial[i], spec_err[perm[i]] = err (KCC_SPEC_DIVZERO when
// partial[S + i] != 0; KCC_SPEC_FAULT for every spec while a fault word is set)
hipError_t launch_fit_finalize(int64_t n_specs, const int64_t* partial,
                               const int32_t* perm, int64_t* totals, int32_t* spec_err,
                               const unsigned long long* faults, hipStream_t s);
// dst[k] += src[k] (wrapping int64), k < n: folds one node shard's partial vector into
// another on the same device (the host-array entry points with more shards than devices)
hipError_t launch_partial_add(int64_t n, int64_t* dst, const int64_t* src, hipStream_t s);

// ---- one-shot exchange of the per-spec partials over xGMI peer memory (kcc_p2p_*) -----
// One process per GPU, W <= P2P_MAX_RANKS.  Every rank owns a mailbox in its own HBM,
// exported as an IPC handle and mapped by every peer:
//   flags [2][W][8] u64 (parity, sender: one 64-B line each; the sender's epoch),
//   data  [2][W][2 smax] i64 (parity, sender: the sender's partial — sums, then div-by-zero
//         counts).
// exchange_finalize_kernel (one launch per step, replacing the RCCL all-reduce and
// fit_finalize): thread i pushes spec i's two partial words into every mailbox (remote
// stores over xGMI, its own included), the launch's last workgroup to finish pushing
// (arrival counter) publishes the epoch into every mailbox's flag of this sender (system
// scope, after every pushing thread's system-scope fence), every workgroup waits for all
// W flags of this epoch in its own mailbox, then sums the W vectors and finalizes
// (totals[perm[i]], spec_err[perm[i]]).  Parity = epoch & 1: a rank can only push epoch
// e + 2 after every peer pushed e + 1, i.e. after every peer's launch for e read its data.
// The epoch lives in device memory (the last workgroup to push advances it), so every
// launch — a replay of a captured graph included — uses the next one.
constexpr int P2P_MAX_RANKS = 8;
__host__ __device__ inline size_t p2p_flag_words(int W) { return (size_t)2 * W * 8; }
inline size_t p2p_mbox_bytes(int W, int64_t smax) {
  return 8 * (p2p_flag_words(W) + (size_t)2 * W * 2 * (size_t)smax);
}
struct P2PArgs {
  int64_t S, smax;
  int32_t W, rank;
  uint64_t* epoch;                        // this rank's last pushed epoch (device word, 0 at
                                          // export; the launch pushes *epoch + 1)
  const int64_t* partial;                 // [2S] this rank's (internal order)
  unsigned char* mbox[P2P_MAX_RANKS];     // rank p's mailbox (this rank's own at [rank])
  const int32_t* perm;                    // internal -> caller index (this rank's fit)
  int64_t* totals;
  int32_t* spec_err;
  uint32_t* arrive;                       // this rank's push arrivals (zero between launches)
  unsigned long long* faults;             // the device's fault words (FAULT_P2P: flag waits
                                          // that gave up; a workgroup that gave up marks its
                                          // specs KCC_SPEC_FAULT)
};
hipError_t launch_exchange_finalize(const P2PArgs& a, hipStream_t s);

// ---- quantity-string parse (kcc_parse.hip) ------------------------
enum ParseMode : int { PARSE_MODE_CPU_MILLIS = 0, PARSE_MODE_BYTES = 1, PARSE_MODE_QUANTITY = 2 };
// per-string status (include/kcc.h KCC_PARSE_*)
enum ParseStatus : int8_t {
  PARSE_OK = 1,           // value as the reference computes it
  PARSE_ERR = 0,          // the reference reports an error and uses 0
  PARSE_UNSUPPORTED = -1, // outside the device parser's exact domain (value 0)
  PARSE_BADOFF = -2       // offsets outside [0, n_bytes] or decreasing (value 0)
};
int64_t parse_grid(int64_t n);
// string i = bytes[offsets[i], offsets[i+1]); bytes 4-byte aligned
hipError_t launch_parse(int mode, int64_t n, const uint8_t* bytes, int64_t n_bytes,
                        const int64_t* offsets, int64_t* out, int8_t* status, hipStream_t s);

// ---- keyed (list-order) reduce (kcc_keyed.hip) --------------------
// Bucketed path: rows in buckets of KB_ROWS, containers in tiles of about KB_TILE.
constexpr int KB_SHIFT = 12;  // 4096 rows per bucket: ~1 KB runs per tile and array
constexpr int KB_ROWS = 1 << KB_SHIFT;
// containers per scatter workgroup (about; keyed_tile cuts whole rounds): at C4 65536
// (3 rounds, 768 tiles) took the keyed call 0.392 -> 0.340 and 0.395 -> 0.372 ms on two
// boxes against 32768 (5 rounds); 131072 equal, 262144 slower
constexpr int KB_TILE = 65536;
constexpr int64_t KB_NB_MAX = 4096;  // buckets (LDS cursors): n_keys <= 16M rows
struct KeyedWork {
  uint32_t* counts;   // [keyed_tiles(n) * keyed_buckets(n_keys)] (one-sweep path: the tiles'
                      // bucket starts, u16 entries in blocks of 32 buckets, kcc_keyed.hip kb_tab_at)
  uint32_t* tot;      // [keyed_buckets(n_keys)]
  uint64_t* sr;       // [n] scattered 8-B records: row within the bucket, low 20 cpu
                      // bits, memory / 64 (kcc_keyed.hip kb_record)
  uint64_t* sv;       // [n][2] the limit values, element-major (NA = 4 only)
  uint32_t* esc_n;    // escape list: what the records cannot hold (cpu >= 2^20: its high
  int32_t* esc_row;   // [n]   bits; memory not a multiple of 64 in [0, 2^38): all of it)
  uint64_t* esc_cpu;  // [n]
  uint64_t* esc_mem;  // [n]
  // one-sweep path (kb_sweep + kb_gather): a bucket group's records are gathered by
  // keyed_sweep_parts(nb) workgroups; parts > 1 sum through part_acc: every part but the
  // last to arrive (arrive[b]) publishes its rows and counts itself (arrive[groups + b]),
  // the last adds them and writes the group's outputs
  uint64_t* part_acc; // [groups][parts][NACC][KB_GA_ROWS]
  uint32_t* arrive;   // [2 x groups]: arrivals, then the published parts (zero between calls)
  unsigned long long* faults;  // the device's fault words (a gather wait that gave up)
};
// One-sweep keyed reduce (NA = 0 counts, 2 requests): each tile of KB_SW_TILE containers
// is counting-sorted by bucket in LDS and written contiguously into its own region of sr
// (whole lines), with the bucket starts in its table row — no global histogram pass, no
// scan, keys read once.  kb_gather then sums bucket b's segments of every tile into LDS
// rows.  The four-kernel bucketed path (kb_hist / kb_scan / kb_scatter / kb_accum) serves
// only the calls with limits (NA = 4).
constexpr int KB_SW_THREADS = 1024;
constexpr int KB_SW_PER = 8;  // containers per thread (the next tile's loads in registers)
constexpr int64_t KB_SW_TILE = (int64_t)KB_SW_THREADS * KB_SW_PER;  // 8192
// containers per sweep tile: KB_SW_TILE, or (beyond one round of one tile per CU) cut so
// the tiles make whole rounds (C4: 2418 tiles = 9.4 rounds -> 2560 of 15472 = 10); a
// tile's records keep the KB_SW_TILE stride in the staging buffer
int64_t keyed_sweep_tile(int64_t n);
int64_t keyed_sweep_tiles(int64_t n);
int keyed_sweep_parts(int64_t nb);
// sizes of the KeyedWork arrays for a call (either path): u32 words of counts, u64
// record slots of sr, u64 words of part_acc
int64_t keyed_counts_words(int64_t n_keys, int64_t n);
int64_t keyed_sr_slots(int64_t n);
int64_t keyed_part_words(int64_t n_keys, int na);
int64_t keyed_tile(int64_t n);   // containers per scatter workgroup (whole CU rounds)
int64_t keyed_tiles(int64_t n);
int64_t keyed_buckets(int64_t n_keys);
bool keyed_bucketed(int64_t n_keys, int64_t n);
// Writes every per-key output (zero where no container), adding every container with
// 0 <= key < n_keys (wrapping sums are order-independent).  kw == nullptr or too many keys:
// memsets + device atomics.  key/value arrays 16-B aligned.
hipError_t launch_reduce_keyed(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* cpu,
                               const int64_t* mem, const uint64_t* cpul, const int64_t* meml,
                               uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                               int64_t* lim_mem, const KeyedWork* kw, hipStream_t s);
// count[k] = #{i : key[i] == k}
hipError_t launch_count_keyed(int64_t n_keys, int64_t n, const int32_t* key, int64_t* count,
                              const KeyedWork* kw, hipStream_t s);

// ---- per-row q of one spec (kcc_rows.hip) -------------------------
hipError_t launch_fit_rows(int64_t n, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
                           const int64_t* alloc_pods, const int64_t* pod_count,
                           const uint64_t* used_cpu, const int64_t* used_mem, uint64_t spec_cpu,
                           int64_t spec_mem, int64_t* q, int32_t* err, hipStream_t s);

// ---- opt-in scheduler request model (kcc_pods.hip) ---------------
hipError_t launch_pod_requests(int64_t n_pods, int64_t n_cont, int64_t n_init,
                               const int64_t* pod_ptr, const uint64_t* cpu_req,
                               const int64_t* mem_req, const int64_t* init_ptr,
                               const uint64_t* init_cpu, const int64_t* init_mem,
                               const uint8_t* restartable, const uint64_t* ovh_cpu,
                               const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem,
                               hipStream_t s);

}  // namespace kcc
