// kcc_kernels.hip — gfx950 kernels of the capacity engine.
//
// Hot path of AshutoshNirkhe/KubernetesClusterCapacity, src/KubeAPI/ClusterCapacity.go (CC):
//   (a) reduce_kernel: the per-container request sums of getPodCPUMemoryRequestsLimits
//       (CC:276-294, adds at CC:290-293), as a segmented int64 reduction over a CSR
//       container list (one segment per node).
//   (b) fit_kernel: main's per-node fit (CC:119-136, findMin CC:159-164) and the
//       total (CC:138), for a batch of S specs (nodes x specs), reduced per spec.
// Both are integer work: no MFMA (no contraction), HBM-bound (a) / VALU-bound (b).
// Results are bit-exact to Go's uint64/int64 wrapping arithmetic.

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "kcc_internal.h"

namespace kcc {

namespace {

// Diagnostic timeline (KCC_TIMELINE builds only): per-workgroup wall-clock stamps
// (s_memrealtime, 100 MHz) of the small kernels' phases, read by kcc_debug_timeline.
#ifdef KCC_TIMELINE
__device__ uint64_t kcc_tl[8192][8];
#define KCC_TL(slot, k) \
  do { if (threadIdx.x == 0) kcc_tl[(slot)][(k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define KCC_TLV(slot, k, v) \
  do { if (threadIdx.x == 0) kcc_tl[(slot)][(k)] = (v); } while (0)
#else
#define KCC_TL(slot, k) do { } while (0)
#define KCC_TLV(slot, k, v) do { } while (0)
#endif

// 64-bit add into LDS (ds_add_u64) through a pointer the compiler cannot prove is LDS
typedef __attribute__((address_space(3))) unsigned long long lds_ull;
__device__ __forceinline__ void lds_add_u64(unsigned long long* p, uint64_t v) {
  __hip_atomic_fetch_add((lds_ull*)p, (unsigned long long)v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ unsigned long long atomic_add_u64(uint64_t* p, uint64_t v) {
  return atomicAdd(reinterpret_cast<unsigned long long*>(p),
                   static_cast<unsigned long long>(v));
}

// A fault word of the device is set (a reduce look-back or exchange flag wait gave up):
// the step's results are not trustworthy and every finalize marks every spec.
__device__ __forceinline__ bool device_faulted(const unsigned long long* f) {
  if (!f) return false;
  return (__hip_atomic_load(f + FAULT_RED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
          __hip_atomic_load(f + FAULT_P2P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
}

// ----------------------------------------------------------------------------
// (a) segmented reduce
// ----------------------------------------------------------------------------

// DPP controls (gfx9 family): row_shr:n, row_bcast:15/31, wave_shr:1.
constexpr int DPP_ROW_SHR = 0x110;
constexpr int DPP_ROW_BCAST15 = 0x142;
constexpr int DPP_ROW_BCAST31 = 0x143;
constexpr int DPP_WAVE_SHR1 = 0x138;

template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, CTRL, ROW_MASK, BANK_MASK, false);
  const uint32_t hi =
      __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), CTRL, ROW_MASK, BANK_MASK, false);
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive prefix sum of a 64-bit value over the 64 lanes, wrapping mod 2^64 —
// all VALU (DPP row shifts within 16-lane rows, then row broadcasts), no LDS.
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
  v += dpp_u64<DPP_ROW_SHR + 1, 0xf, 0xf>(v);
  v += dpp_u64<DPP_ROW_SHR + 2, 0xf, 0xf>(v);
  v += dpp_u64<DPP_ROW_SHR + 4, 0xf, 0xf>(v);
  v += dpp_u64<DPP_ROW_SHR + 8, 0xf, 0xf>(v);
  v += dpp_u64<DPP_ROW_BCAST15, 0xa, 0xf>(v);
  v += dpp_u64<DPP_ROW_BCAST31, 0xc, 0xf>(v);
  return v;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int l) {
  return (int64_t)readlane_u64((uint64_t)v, l);
}

// 32-bit version (every lane sum below 2^32; also packed fields that never carry)
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_SHR + 1, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_SHR + 2, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_SHR + 4, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_SHR + 8, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_BCAST15, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0u, v, DPP_ROW_BCAST31, 0xc, 0xf, false);
  return v;
}

// Two inclusive 64-bit prefix sums over the 64 lanes at once (wrapping): per DPP step one
// v_add_co_u32_dpp + v_addc_co_u32_dpp per value (the neighbour's operand read through
// DPP; out-of-row lanes read 0 (bound_ctrl), rows masked off keep their value), the two
// scans interleaved so every DPP read is >= 2 wait states after the write it reads.
// 12 VALU per value instead of 30 (zeroed DPP move targets, moves, 64-bit add).
// (C4 reduce 136.5 -> 134.3 us against the compiler's scan, A/B in one process, outputs
// identical)
// gfx950 (as gfx942) needs 2 wait states between a VALU write of VCC and a VALU read of it
// (LLVM puts an s_nop 1 between v_sub_co_u32 and v_subb_co_u32): one after each low half.
#define KCC_SCAN2_STEP(ctl)                                 \
  "v_add_co_u32_dpp %0, vcc, %0, %0 " ctl "\n\t"            \
  "s_nop 1\n\t"                                             \
  "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc " ctl "\n\t"      \
  "v_add_co_u32_dpp %2, vcc, %2, %2 " ctl "\n\t"            \
  "s_nop 1\n\t"                                             \
  "v_addc_co_u32_dpp %3, vcc, %3, %3, vcc " ctl "\n\t"
__device__ __forceinline__ void wave_incl_scan2_u64(uint64_t& a, uint64_t& b) {
  uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32), bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
  asm volatile("s_nop 1\n\t"
               KCC_SCAN2_STEP("row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0")
               KCC_SCAN2_STEP("row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:0")
               KCC_SCAN2_STEP("row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:0")
               KCC_SCAN2_STEP("row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:0")
               KCC_SCAN2_STEP("row_bcast:15 row_mask:0xa bank_mask:0xf")
               KCC_SCAN2_STEP("row_bcast:31 row_mask:0xc bank_mask:0xf")
               "s_nop 1"
               : "+v"(al), "+v"(ah), "+v"(bl), "+v"(bh)
               :
               : "vcc");
  a = (uint64_t)ah << 32 | al;
  b = (uint64_t)bh << 32 | bl;
}

// CSR offset of node j relative to the wave range start, clamped into int32.
__device__ __forceinline__ int32_t rel_clamp(int64_t raw, int64_t wb) {
  const int64_t v = raw - wb;  // any range is < 2^28 (reduce_range)
  constexpr int64_t HI = (int64_t)1 << 30;
  return (int32_t)(v < -1 ? -1 : (v > HI ? HI : v));
}
__device__ __forceinline__ int64_t ptr_at(const int64_t* __restrict__ ptr, int64_t j,
                                          int64_t n_nodes) {
  return ptr[j < n_nodes ? j : n_nodes];
}
__device__ __forceinline__ int32_t rel_ptr(const int64_t* __restrict__ ptr, int64_t j,
                                           int64_t n_nodes, int64_t wb) {  // NOLINT
  return rel_clamp(ptr_at(ptr, j, n_nodes), wb);
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));


// Container loads use the default cache policy.  Measured (round 3, one process, outputs
// identical): C4 reduce default 130.5 us, nt 181.8, sc1 183.5, nt sc1 181.5; the 8-way
// shard 19.5 / 32.3 / 25.2 / 32.2 us: the 16-B lane loads of a wave coalesce in L1, which
// every non-default policy bypasses

// RED_IPL consecutive 64-bit values of one array for this lane: RED_IPL / 2 16-B
// range-checked buffer loads (outside the descriptor's range they read 0), so the
// prefetch is branch-free and never waits where it is issued.
// The lane offset (voff) is loop-invariant and the tile offset goes in soffset, so no
// address VGPR is recomputed per tile (a recomputed address register that the
// allocator shares with an in-flight load's destination forces a vmcnt(0) wait).
__device__ __forceinline__ void load_quad(__amdgpu_buffer_rsrc_t r, int32_t voff, int32_t soff,
                                          uint64_t (&x)[RED_IPL]) {
#pragma unroll
  for (int h = 0; h < RED_IPL / 2; ++h) {
    const u64x2 v = __builtin_bit_cast(
        u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16 * h, soff, 0));
    x[2 * h] = v.x;
    x[2 * h + 1] = v.y;
  }
}

// One wavefront walks a contiguous range of `range` containers in tiles of
// RED_TILE = 256 (4 per lane, coalesced SoA buffer loads, next tile prefetched).
// Start: the node owning the range's first container (the last node whose CSR offset is
// <= it) by a 64-ary search of the offsets — one wave-wide load per level (3 levels at
// 125k nodes, 4 at 1M), issued after the first tiles' data loads, whose latency it hides.
// Per tile and array:
//   1. the tile-local inclusive prefix sum of the 256 values: a 4-item running sum per
//      lane, one DPP inclusive scan (64-bit, all VALU) of the lane totals, written to
//      a per-wave LDS strip pre[0..255];
//   2. nodes are visited in aligned blocks of 64 (lane l <-> node 64*blk + l), so the
//      block's CSR end offsets are one coalesced 512-B load, held in a register (eA),
//      with the next block's reloaded at every tile end (eNr; L2 hits, but at a fixed
//      distance from its use, so no tile drains the data prefetch); a node's start is the previous lane's end
//      (DPP shift; lane 0 takes the previous block's last end).  The nodes ending in
//      this tile are a contiguous run of lanes starting at node cur (the node holding
//      the tile's first item); each gets sum = pre[end-1] - pre[start-1], or
//      pre[end-1] + carry when it began in an earlier tile (carry = its running sum so
//      far, wave-uniform), in wrapping uint64 arithmetic, so the differences are exact;
//      when the run reaches lane 63 the block is complete and the pass continues with
//      the next block in the same tile;
//   3. the sums stay in registers (res, one per lane = per node of the block) and a
//      completed block is written with ONE coalesced 512-B store per array: stores
//      count in vmcnt like loads, so a store per tile would put its completion latency
//      in front of the next tile's data wait.
// End: every node that ends in the range is stored by this wave (empty ones included;
// wave 0 starts at node 0, so the empty nodes ahead of the first container too), except
// node0 when it began in an earlier range: the wave publishes its tail record (the
// piece of the node open at its range end, `carry`) and then, if node0 began earlier and
// ended here, sums the tail records of the waves from the one holding node0's first
// container up to its own and stores node0 (decoupled look-back: each wave publishes
// before it waits, so waits never chain; a wave waits only for lower-indexed waves,
// dispatched before it).  No atomics, nothing to zero between launches.
// The tile-local prefix strip: position p (lane p / RED_IPL's item p % RED_IPL) at
// strip_at(p) of the wave's strip: pair-major — item pair h of every lane together, so the
// lanes' 16-B stores are 16 B apart (conflict-free; lane-major, 64 B apart, is 4-way)
__device__ __forceinline__ int32_t strip_at(int32_t p) {
  static_assert(RED_IPL == 8, "pair-major strip");
  return ((p & 6) << 6) + ((p >> 3) << 1) + (p & 1);
}
constexpr uint32_t RED_OOB_OFFSET = 0x7ffffff0u;  // > any output's range (n_nodes < 2^28)
[[maybe_unused]] constexpr uint32_t RED_SPIN_MAX = 1u << 18;       // look-back polls before a wait gives up
// node-prep polls: s_sleep units (64 clocks) between them (4 and 1 measured equal, round 5)
#define KCC_NP_SLEEP 20
[[maybe_unused]] constexpr uint32_t NP_SPIN_MAX = 1u << 22;  // polls before a wait gives up (~2 s)
// Look-back publication: tagged words.  Each 64-bit value of the piece travels as two
// 64-bit words {tag:32 | half:32}, stored by 2 x NA lanes as relaxed agent-scope atomics;
// the consumer polls the words until every tag matches and assembles the halves.  Every
// word is single-copy atomic and validates itself, so no ordering between the stores is
// needed at all — exact under the HIP memory model, without fences or a vmcnt(0) drain.
// (Measured and deleted, DESIGN.md §10: a release / acquire tag word, 2.3x slower at C4 —
// every publishing wave wrote back its XCD's L2; round 3's relaxed stores + vmcnt(0) + tag.)
constexpr uint64_t RED_WORD_TAG = 0x4B43C0DEull << 32;  // upper half of a published word
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// The rank bodies' few workgroup words live right after their 16 * RANK_L bytes of keys in
// the caller's LDS buffer (RANK_LDS_WORDS u64 in all), not in __shared__ variables of their
// own: those would add to every launch that carries them (the reduce's 32 KiB strips + 24 B
// held a CU to 4 of its workgroups, where 5 fit in 160 KiB)
constexpr int RANK_LDS_WORDS = 2 * RANK_L + 4;
__device__ __forceinline__ uint32_t* rank_small(uint64_t* lds) {
  return reinterpret_cast<uint32_t*>(lds + 2 * RANK_L);  // [0] last, [4..7] per-wave counts
}

__device__ void spec_rank_body(const RankArgs& ra, int64_t blk, uint64_t* lds);
__device__ void spec_place_body(const PlaceArgs& pa, int64_t blk);

// The wave's sum of a 64-bit value (wrapping), wave-uniform.
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  v = wave_incl_scan_u64(v);
  return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, 63);
}

__device__ void np_body(const NpArgs& np, int32_t j, uint32_t* scratch);

// NPM: node prep behind the reduce's workgroups (NpArgs): the node sums written through
// (sc1) and every wave's completion counted
#ifdef KCC_DIAG_NP_NOSYNC  // timing diagnostics only (wrong results): node prep does not wait
constexpr bool KCC_NP_NOSYNC = true;
#else
constexpr bool KCC_NP_NOSYNC = false;
#endif
#ifdef KCC_DIAG_NP_NOSC1  // timing diagnostics only: the node sums stored plainly
constexpr bool KCC_NP_NOSC1 = true;
#else
constexpr bool KCC_NP_NOSC1 = false;
#endif
template <int NA, bool NPM>
__global__ __launch_bounds__(256) void reduce_kernel(RedArgs a, RankArgs ra, NpArgs np) {
  __shared__ __attribute__((aligned(16))) uint64_t pre_s[RED_WAVES_PER_BLOCK][NA][RED_TILE];
  static_assert(sizeof(pre_s) >= 8 * RANK_LDS_WORDS, "the rank workgroups stage RANK_L 16-B keys");
  const int32_t npb = NPM ? np.n_place + np.n_rows : 0;  // the last workgroups
  if constexpr (NPM) {
    if ((int32_t)blockIdx.x >= (int32_t)gridDim.x - npb) {
      np_body(np, (int32_t)blockIdx.x - ((int32_t)gridDim.x - npb), reinterpret_cast<uint32_t*>(&pre_s[0][0][0]));
      return;
    }
  }
  // the spec ranks' workgroups: behind the reduce's (RedArgs::ranks_last; dispatched as its
  // first waves retire, they run in the reduce's tail) or in front of them
  const int32_t rank0 = a.ranks_last ? (int32_t)gridDim.x - npb - ra.n_blocks : 0;  // first rank block
  const int32_t red0 = a.ranks_last ? 0 : ra.n_blocks;                              // first reduce block
  if constexpr (NA == 2) {  // (launch_reduce: the ranks ride the 2-array reduce only)
    if (ra.n_blocks > 0 && (int32_t)blockIdx.x >= rank0 && (int32_t)blockIdx.x < rank0 + ra.n_blocks) {
      // the rank workgroups' waves issue ahead of the reduce's waves on their CUs (the
      // arbiter serves the oldest wave first, and the ranks, dispatched last, gate node
      // prep): 2-way C4 rank step 168.4 -> 165.2 / 168.5 -> 165.6 us, 4-way 88.1 -> 87.6,
      // C4 and the 8-way rank equal (round 6, profiles/r06t_ab_rank_prio.txt)
      __builtin_amdgcn_s_setprio(3);
      spec_rank_body(ra, (int32_t)blockIdx.x - rank0, &pre_s[0][0][0]);
      return;
    }
  }
  const int lane = threadIdx.x & 63;
  const int64_t n_nodes = a.n_nodes, c0 = a.c0, n_cont = a.c_end;
  const int32_t range = a.range;
  const int64_t* __restrict__ ptr = a.ptr;
  // wave index made provably uniform (T20: no waterfall loops around the buffer ops).
  // Range order = dispatch order: a wave's look-back predecessors are dispatched before it
  const int32_t w = __builtin_amdgcn_readfirstlane((int32_t)((blockIdx.x - red0) *
                                                             RED_WAVES_PER_BLOCK +
                                                             (threadIdx.x >> 6)));
  // containers [c0, n_cont): absolute indices, like the offsets in ptr (node indices
  // are local to the launch)
  const int64_t wb = c0 + (int64_t)w * range;
  if (wb >= n_cont) return;  // wave-uniform; no block-level barrier in this kernel
  // NPM: this launch's epoch (the node-prep workgroups publish it only after every storing
  // wave's flag); the wave's stores performed, then its flag
  const uint32_t epoch = NPM ? __hip_atomic_load(np.sync + NP_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
  auto red_signal = [&]() {
    if constexpr (NPM && !KCC_NP_NOSYNC) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if ((threadIdx.x & 63) == 0)
        __hip_atomic_store(np.sync + NP_FLAGS + w, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  KCC_TL(4096 + (blockIdx.x - red0) % 4096, 0);
  const int32_t len = (int32_t)(n_cont - wb < range ? n_cont - wb : range);
  __builtin_assume(len >= 1);  // (wb < n_cont: the tile loop runs, its first loads need no guard)
  uint64_t (*pre)[RED_TILE] = pre_s[threadIdx.x >> 6];
  const uint64_t* in[4] = {a.in[0], a.in[1], a.in[2], a.in[3]};
  uint64_t* out[4] = {a.out[0], a.out[1], a.out[2], a.out[3]};
  __amdgpu_buffer_rsrc_t rs[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k)  // whole 16-B pairs only: an odd last item is fixed up below
    rs[k] = __builtin_amdgcn_make_buffer_rsrc((void*)(in[k] + wb), (short)0,
                                              (int)((len & ~1) * 8), 0x00020000);
  // a ring of RED_PREFETCH + 1 tiles in registers: RED_PREFETCH in flight while one is
  // reduced (static ring indices: the tile loop below is unrolled over the ring).
  // The first tiles' loads go out first: they depend on the range alone, while the node
  // search below is a chain of dependent loads
  constexpr int RING = RED_PREFETCH + 1;
  uint64_t xs[RING][NA][RED_IPL];
#pragma unroll
  for (int u = 0; u < RED_PREFETCH; ++u)
#pragma unroll
    for (int k = 0; k < NA; ++k) load_quad(rs[k], lane * 8 * RED_IPL, u * RED_TILE * 8, xs[u][k]);
  __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink them below the search)

  // node0: the last node j < n_nodes with ptr[j] <= wb (ptr[0] == c0 <= wb; wave 0 takes
  // node 0 itself, so the empty nodes ahead of the first container are its to store).
  // Invariant: ptr[lo] <= wb, and hi == n_nodes or ptr[hi] > wb.
  int64_t node0 = 0, p0 = c0;  // p0 = ptr[node0]
  if (w > 0) {
    int64_t lo = 0, hi = n_nodes;
    while (hi - lo > 1) {
      const int64_t step = (hi - lo + 63) >> 6;
      const int64_t idx = lo + (int64_t)lane * step;
      const int64_t v = idx < hi ? ptr[idx] : INT64_MAX;
      const unsigned long long bl = __ballot(v <= wb);  // lane 0 (idx = lo) always
      const int h = 63 - __builtin_clzll(bl);
      p0 = readlane_i64(v, h);
      lo += (int64_t)h * step;
      hi = lo + step < hi ? lo + step : hi;
    }
    node0 = lo;
  }
  const bool first_open = p0 < wb;                      // node0 began in an earlier range
  const int64_t own_lo = node0 + (first_open ? 1 : 0);  // first node stored by the flushes
  int64_t cur = node0;  // node holding the current tile's first item
  // start of node cur relative to wb (<= 0 for node0): when it is < len at the range end,
  // node cur continues into the next range and its piece here is published
  int32_t open_start = p0 - wb < -1 ? -1 : (int32_t)(p0 - wb);
  uint64_t carry[NA];   // node cur's running sum over the earlier tiles of this range
  uint64_t res[NA];     // sums of block blk's nodes (lane l <-> node 64*blk + l)
  uint64_t head[NA];    // node0's piece in this range, when first_open (wave-uniform)
#pragma unroll
  for (int k = 0; k < NA; ++k) carry[k] = res[k] = head[k] = 0;

  int64_t blk = node0 >> 6;
  int32_t eA = rel_ptr(ptr, 64 * blk + 1 + lane, n_nodes, wb);  // end of node 64*blk + l
  int32_t sA0 = rel_ptr(ptr, 64 * blk, n_nodes, wb);            // end of node 64*blk - 1
  int64_t eNr = ptr_at(ptr, 64 * blk + 65 + lane, n_nodes);     // next block (raw, in flight)
  bool have_next = true;  // eNr holds block blk + 1's ends
  // a completed block's sums awaiting their store (lane l <-> node 64*pend_blk + l)
  uint64_t resF[NA];
  bool pend = false;
  int64_t pend_blk = 0;  // wave-uniform
  auto flush_pending = [&]() {  // rare path only (see issue_pending)
    const int64_t pend_j = 64 * pend_blk + lane;
    if (pend_j >= own_lo) {
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        if constexpr (NPM && !KCC_NP_NOSC1) __hip_atomic_store(out[k] + pend_j, resF[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else out[k][pend_j] = resF[k];
      }
    }
    pend = false;
  };
  // Output descriptors: a store at an offset past the end is dropped by the hardware,
  // which lets every tile issue its pending-block stores unconditionally.
  __amdgpu_buffer_rsrc_t ro[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k)
    ro[k] = __builtin_amdgcn_make_buffer_rsrc((void*)out[k], (short)0, (int)(n_nodes * 8),
                                              0x00020000);
  // The pending block's stores, issued right before a tile's prefetch loads: vmcnt is
  // an in-order count, so a store makes every later load's wait include its
  // acknowledgement; issued alongside the prefetch it completes with it.  A fixed
  // number of them every tile (out of range when nothing is pending) keeps the count
  // static, so the compiler's waits do not assume the stores absent.
  auto issue_pending = [&]() {
    const int64_t pend_j = 64 * pend_blk + lane;
    const uint32_t voff = (pend && pend_j >= own_lo) ? (uint32_t)(pend_j * 8) : RED_OOB_OFFSET;
#pragma unroll
    for (int k = 0; k < NA; ++k)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, resF[k]), ro[k],
                                            (int)voff, 0, NPM && !KCC_NP_NOSC1 ? 16 : 0);  // (16: sc1)
    pend = false;
  };

  auto tile = [&](uint64_t (&x)[NA][RED_IPL], uint64_t (&nx)[NA][RED_IPL], const int32_t tb) {
#ifndef KCC_DIAG_RED_NOSTORE
    issue_pending();
#endif
#pragma unroll
    for (int k = 0; k < NA; ++k)
      load_quad(rs[k], lane * 8 * RED_IPL, (tb + RED_PREFETCH * RED_TILE) * 8, nx[k]);
#ifdef KCC_DIAG_RED_LOADONLY
#pragma unroll
    for (int k = 0; k < NA; ++k)
#pragma unroll
      for (int i = 0; i < RED_IPL; ++i) carry[k] += x[k][i];
    return;
#endif
    const int32_t p0l = tb + RED_IPL * lane;  // relative position of this lane's first item
    if ((len & 1) && p0l <= len - 1 && len - 1 < p0l + RED_IPL) {  // odd tail: last item alone
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        const uint64_t v = in[k][wb + len - 1];
#pragma unroll
        for (int i = 0; i < RED_IPL; ++i)  // static indices only (no scratch)
          if (p0l + i == len - 1) x[k][i] = v;
      }
    }

    // --- 1. tile-local inclusive prefix sums -> LDS -----------------------------
    // the lane's 4-item total, scanned in place; the lane's items' prefixes then walk
    // back from it (x0 is dead once the total is formed: fewer live registers)
    // the lane's in-lane inclusive prefixes in place; after the scan, each item's prefix is
    // the lane's exclusive base plus its in-lane prefix: 64-bit adds only (one
    // v_lshl_add_u64 each; round 5 walked back from the lane's inclusive prefix with 64-bit
    // subtracts, v_sub_co + v_subb each: 83 -> 73 VALU per tile, C4 130.8 -> 130.6 us, the
    // 8-way shard 20.1 -> 19.9 us, profiles/r06d_ab_reduce_fwd_*.txt)
    uint64_t tot[NA], P[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
#pragma unroll
      for (int i = 1; i < RED_IPL; ++i) x[k][i] += x[k][i - 1];
      P[k] = x[k][RED_IPL - 1];
    }
#pragma unroll
    for (int k = 0; k < NA; k += 2) wave_incl_scan2_u64(P[k], P[k + 1]);
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      uint64_t pp[RED_IPL];  // the lane's items' inclusive prefixes
      const uint64_t base = P[k] - x[k][RED_IPL - 1];
#pragma unroll
      for (int i = 0; i < RED_IPL - 1; ++i) pp[i] = base + x[k][i];
      pp[RED_IPL - 1] = P[k];
      u64x2* dst = reinterpret_cast<u64x2*>(&pre[k][0]);  // pair h at strip_at(8 lane + 2 h)
#pragma unroll
      for (int h = 0; h < RED_IPL / 2; ++h) dst[h * 64 + lane] = u64x2{pp[2 * h], pp[2 * h + 1]};
      tot[k] = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(P[k] >> 32), 63) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((uint32_t)P[k], 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // --- 2./3. nodes ending in this tile, block by block ----------------------------
    const int32_t eN_rel = rel_clamp(eNr, wb);  // next block's ends (previous tile's load)
    const int32_t lim = tb + RED_TILE < len ? tb + RED_TILE : len;
    int32_t last_end = -1;  // end of the last node that ended in this tile (-1: none)
    for (;;) {
      int32_t s = __builtin_amdgcn_update_dpp(0, eA, DPP_WAVE_SHR1, 0xf, 0xf, false);
      if (lane == 0) s = sA0;
      // node 64 blk + lane ends in this tile: lanes [cur - 64 blk, n_nodes - 64 blk) (cur
      // lies in block blk or at its end) whose end is within the tile
      const int64_t jb = 64 * blk, nrem = n_nodes - jb;
      const int32_t lo_l = (int32_t)(cur - jb), hi_l = nrem < 64 ? (int32_t)nrem : 64;
      const bool act = lane >= lo_l && lane < hi_l && eA <= lim;
      // branch-free: both prefixes read at positions clamped into the strip, the sum
      // selected (s <= tb only for node cur, which began in an earlier tile)
      const int32_t ie = min(max(eA - 1 - tb, 0), RED_TILE - 1);
      const int32_t is = min(max(s - 1 - tb, 0), RED_TILE - 1);
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        const uint64_t pe = pre[k][strip_at(ie)], ps = pre[k][strip_at(is)];
        const uint64_t startp = s > tb ? ps : (0ull - carry[k]);
        const uint64_t sum = eA > s ? pe - startp : 0ull;
        res[k] = act ? sum : res[k];
      }
      const unsigned long long bal = __ballot(act);
      if (!bal) break;
      if (first_open && cur == node0 && ((bal >> (node0 & 63)) & 1ull)) {  // node0 ends here
#pragma unroll
        for (int k = 0; k < NA; ++k) head[k] = readlane_u64(res[k], (int)(node0 & 63));
      }
      const int hi = 63 - __builtin_clzll(bal);  // the run is lanes [cur - 64*blk, hi]
      last_end = __builtin_amdgcn_readlane(eA, hi);
      cur = 64 * blk + hi + 1;
      if (hi != 63) break;
      // block complete.  The next block's ends were loaded at the end of the previous
      // tile (a second block completing in the same tile loads its ends here).  This
      // block's sums move to the pending buffer, stored at the top of the next tile.
      const int32_t e_next =
          have_next ? eN_rel : rel_ptr(ptr, 64 * blk + 65 + lane, n_nodes, wb);
      have_next = false;
      if (pend) flush_pending();  // two blocks in one tile (runs of tiny nodes): now
#pragma unroll
      for (int k = 0; k < NA; ++k) resF[k] = res[k];
      pend = true;
      pend_blk = blk;
      sA0 = last_end;
      eA = e_next;
      ++blk;
    }
    eNr = ptr_at(ptr, 64 * blk + 65 + lane, n_nodes);  // next block's ends (usually L2 hits)
    have_next = true;
    if (last_end >= 0) open_start = last_end;
    if (last_end > tb) {  // node cur is open at the tile end: its sum so far
#pragma unroll
      for (int k = 0; k < NA; ++k)
        carry[k] = tot[k] - pre[k][strip_at(last_end - 1 - tb)];
    } else if (last_end == tb) {  // only empty nodes ended, at the tile's start (wave 0's
#pragma unroll                    // leading empty nodes): cur starts here
      for (int k = 0; k < NA; ++k) carry[k] = tot[k];
    } else {
#pragma unroll
      for (int k = 0; k < NA; ++k) carry[k] += tot[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  for (int32_t tb = 0; tb < len; tb += RING * RED_TILE) {
#pragma unroll
    for (int u = 0; u < RING; ++u)
      if (tb + u * RED_TILE < len) tile(xs[u], xs[(u + RED_PREFETCH) % RING], tb + u * RED_TILE);
  }
#if defined(KCC_DIAG_RED_LOADONLY) || defined(KCC_DIAG_RED_NOSTORE)
  if (carry[0] == 0x123456789ull) out[0][0] = carry[NA - 1] ^ res[0];
#endif
#ifndef KCC_DIAG_RED_NOSTORE
  issue_pending();
#endif
  // the partly finished block: nodes [max(own_lo, 64*blk), cur)
  {
    const int64_t j = 64 * blk + lane;
    if (j >= own_lo && j < cur) {
#ifndef KCC_DIAG_RED_NOSTORE
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        if constexpr (NPM && !KCC_NP_NOSC1) __hip_atomic_store(out[k] + j, res[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else out[k][j] = res[k];
      }
#endif
    }
  }
  // publish: node cur continues into the next range (it began before the range end);
  // its piece here is `carry`.  Exactly one later wave consumes the record (the wave where
  // node cur ends: it looks back over every range the node spans) and frees it, so every
  // record is free (all zero) between launches; nothing is published for a node that
  // starts at the next range (no consumer).
  uint64_t* const rec = a.tail + (int64_t)w * RED_TAIL_WORDS;
  const bool publish = wb + len < n_cont && open_start < len;
  static_assert(2 * NA <= RED_TAIL_WORDS, "two tagged words per value");
  if (publish && lane < 2 * NA) {  // lane j: half (j & 1) of value j >> 1
    uint64_t v = carry[0];
#pragma unroll
    for (int k = 1; k < NA; ++k) v = (lane >> 1) == k ? carry[k] : v;
    const uint64_t word = RED_WORD_TAG | ((lane & 1) ? v >> 32 : v & 0xffffffffull);
    __hip_atomic_store(rec + lane, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // look-back: node0 began in an earlier range and ended in this one
  if (first_open && cur > node0) {
    uint64_t acc[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] = head[k];
    const int64_t ws = (p0 - c0) / range;  // the wave holding node0's first container
    for (int64_t b0 = ws; b0 < w; b0 += 64) {
      const int64_t wi = b0 + lane;
      uint64_t v[NA];
#pragma unroll
      for (int k = 0; k < NA; ++k) v[k] = 0;
      if (wi < w) {
        uint64_t* r = a.tail + wi * RED_TAIL_WORDS;
        bool seen = true;
        uint64_t wd[2 * NA];
        uint32_t spins = 0;
        for (;;) {
          bool all = true;
#pragma unroll
          for (int j = 0; j < 2 * NA; ++j) {
            wd[j] = __hip_atomic_load(r + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            all = all && (wd[j] >> 32) == (RED_WORD_TAG >> 32);
          }
#ifdef KCC_DIAG_RED_GIVEUP  // fault-path test builds only: every wait gives up at once
          all = false;
          spins = RED_SPIN_MAX;
#endif
          if (all) break;
          if (++spins >= RED_SPIN_MAX) {  // never on a healthy device: count it, go on
            atomicAdd(&a.faults[FAULT_RED], 1ull);
            seen = false;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int k = 0; k < NA; ++k) v[k] = (wd[2 * k] & 0xffffffffull) | (wd[2 * k + 1] << 32);
        // consumed: free the record for the next launch (a wait that gave up leaves it:
        // the context is faulted until kcc_clear_faults re-zeroes the records)
        if (seen) {
#pragma unroll
          for (int j = 0; j < 2 * NA; ++j)
            __hip_atomic_store(r + j, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#pragma unroll
      for (int k = 0; k < NA; ++k) acc[k] += wave_sum_u64(v[k]);
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        if constexpr (NPM && !KCC_NP_NOSC1) __hip_atomic_store(out[k] + node0, acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else out[k][node0] = acc[k];
      }
    }
  }
  red_signal();
  KCC_TL(4096 + (blockIdx.x - red0) % 4096, 1);
}

// ----------------------------------------------------------------------------
// (b) fit
// ----------------------------------------------------------------------------

// Fast-path bounds (see DESIGN.md "Fit fast path: exactness argument").
constexpr uint64_t FAST_FC_MAX = 1ull << 23;    // free CPU < 2^23 (f32 quotient exact)
constexpr int64_t FAST_FM_MAX = 1ll << 50;      // 0 <= free mem < 2^50 (f64 quotient exact)
constexpr int64_t FAST_P_ABS = 1ll << 20;       // |allocatable pods| <= 2^20
constexpr int64_t FAST_CL_ABS = 1ll << 20;      // |allocPods - podCount| <= 2^20
constexpr uint64_t FAST_C_MAX = 1ull << 51;     // 1 <= spec cpu < 2^51
constexpr int64_t FAST_M_MAX = 1ll << 51;       // 1 <= spec mem < 2^51

// ---- node prep behind the reduce (NpArgs, the clamp in the fit) ---------------------
// thread 0 waits until *w == epoch (bounded: a give-up counts as a reduce fault), then the
// workgroup goes on.  Polls ~0.5 us apart (each is an uncached load of one line)
__device__ void np_wait(const uint32_t* w, uint32_t epoch, unsigned long long* faults) {
  if (threadIdx.x == 0) {
    uint32_t spins = 0;
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      if (++spins >= NP_SPIN_MAX) {
        atomicAdd(&faults[FAULT_RED], 1ull);
        break;
      }
      __builtin_amdgcn_s_sleep(KCC_NP_SLEEP);
    }
  }
  __syncthreads();
}

// rows [i0, i1): wave 0 waits for the flags of the reduce waves that store their sums — the
// wave where a node's last container lies, the one before a range boundary for an empty
// node there: waves [(ptr[i0] - c0) / range - 1, (ptr[i1] - c0) / range] (every storing
// wave is in some workgroup's window) — then the workgroup goes on
__device__ void np_wait_rows(const NpArgs& np, int64_t i0, int64_t i1, uint32_t epoch) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int64_t r = np.range;
    int64_t wlo = (np.ptr[i0] - np.c0) / r - 1, whi = (np.ptr[i1] - np.c0) / r;
    wlo = wlo < 0 ? 0 : wlo;
    whi = whi > np.red_waves - 1 ? np.red_waves - 1 : whi;
    for (int64_t b = wlo; b <= whi; b += 64) {
      const int64_t wi = b + lane;
      uint32_t spins = 0;
      while (__ballot(wi <= whi && __hip_atomic_load(np.sync + NP_FLAGS + wi, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) != epoch)) {
        if (++spins >= NP_SPIN_MAX) {
          if (lane == 0) atomicAdd(&np.faults[FAULT_RED], 1ull);
          break;
        }
        __builtin_amdgcn_s_sleep(KCC_NP_SLEEP);
      }
    }
  }
  __syncthreads();
}

// 1024 rows (thread t: rows i0 + t + 256 q): node_prep's clamp-in-fit work (NC, one node
// chunk; see node_prep_kernel): the free capacity, the slow rows, the node stream (one
// stream position per workgroup, the rows padded to whole groups), the clamp values, and
// the rows clamped for every spec
__device__ void np_rows(const NpArgs& np, int32_t rb, uint32_t* scratch) {
  constexpr int SUB = NP_ROWS_PER_WG / 256;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t n = np.n, i0 = (int64_t)rb * NP_ROWS_PER_WG;
  KCC_TL(rb % 1024, 2);
  // the inputs this launch does not write go out first
  uint64_t ac[SUB];
  int64_t am[SUB], aP[SUB], pc[SUB];
#pragma unroll
  for (int q = 0; q < SUB; ++q) {
    const int64_t i = i0 + q * 256 + tid;
    const bool valid = i < n;
    ac[q] = valid ? np.alloc_cpu[i] : 0;
    am[q] = valid ? np.alloc_mem[i] : 0;
    aP[q] = valid ? np.alloc_pods[i] : 0;
    pc[q] = valid ? np.pod_count[i] : 0;
  }
  const uint32_t epoch = __hip_atomic_load(np.sync + NP_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  np_wait(np.sync + NP_DONE, epoch, np.faults);  // the counters zeroed, the class counts written
  KCC_TL(rb % 1024, 6);
  uint64_t cls_n = 0;  // class A | class B << 32
  {
    const unsigned long long* bc = reinterpret_cast<const unsigned long long*>(np.bcnt);
    for (int64_t b = lane; b < (np.S + 63) / 64; b += 64)
      cls_n += __hip_atomic_load(bc + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cls_n = readlane_u64(wave_incl_scan_u64(cls_n), 63);
  }
  const bool want_b = (cls_n >> 32) != 0;
  const int64_t nN = (int64_t)(uint32_t)cls_n + (int64_t)(cls_n >> 32);
  const bool slow_all = nN < np.S;
  if (!KCC_NP_NOSYNC) np_wait_rows(np, i0, i0 + NP_ROWS_PER_WG < n ? i0 + NP_ROWS_PER_WG : n, epoch);  // the rows' sums stored
  KCC_TL(rb % 1024, 3);
  uint64_t uc[SUB];
  int64_t um[SUB];
#pragma unroll
  for (int q = 0; q < SUB; ++q) {
    const int64_t i = i0 + q * 256 + tid;
    const bool valid = i < n;
    uc[q] = valid ? __hip_atomic_load(np.used_cpu + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    um[q] = valid ? __hip_atomic_load(np.used_mem + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  }
  uint64_t r_fm[SUB];
  uint32_t r_fc[SUB];
  int32_t r_P[SUB], r_cl[SUB];
  unsigned long long sbal[SUB];
  uint64_t always_sum = 0;
#pragma unroll
  for (int q = 0; q < SUB; ++q) {
    const int64_t i = i0 + q * 256 + tid;
    const bool valid = i < n;
    bool ok = false;
    r_fm[q] = 0;
    r_fc[q] = 0;
    r_P[q] = 0;
    r_cl[q] = 0;
    if (valid) {
      const uint64_t fc = ac[q] > uc[q] ? ac[q] - uc[q] : 0;                                      // CC:119-123
      const int64_t fm = am[q] > um[q] ? (int64_t)((uint64_t)am[q] - (uint64_t)um[q]) : 0;       // CC:125-129
      const int64_t P = aP[q];
      const int64_t cl = (int64_t)((uint64_t)P - (uint64_t)pc[q]);                               // CC:135
      ok = fc < FAST_FC_MAX && fm >= 0 && fm < FAST_FM_MAX && P >= -FAST_P_ABS && P <= FAST_P_ABS &&
           cl >= -FAST_CL_ABS && cl <= FAST_CL_ABS;
      if (ok) {
        r_fm[q] = (uint64_t)fm;
        r_fc[q] = (uint32_t)fc;
        r_P[q] = (int32_t)P;
        r_cl[q] = (int32_t)cl;
        if (nN > 0 && P <= 0) always_sum += (uint64_t)(0 - cl);  // x >= P for every spec: w = Penc - cl
      }
      if (slow_all || !ok) {
        SlowNode sn;
        sn.fc = fc;
        sn.fm = fm;
        sn.P = P;
        sn.cl = cl;
        np.slow[i] = sn;
      }
    }
    const unsigned long long bl = __ballot(valid && !ok);
    if (bl) {
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(&np.counters[CNT_SLOW_ROWS], (unsigned long long)__popcll(bl));
      base = __shfl(base, 0);
      if (valid && !ok) np.slow_list[base + __popcll(bl & ((1ull << lane) - 1ull))] = i;
    }
    sbal[q] = __ballot(r_fc[q] > 0 && r_fm[q] > 0 && r_P[q] > 0);  // 0 unless ok
  }
  KCC_TL(rb % 1024, 4);
  {  // rows clamped for every spec: one wave-summed add (one per workgroup: equal, round 5)
    uint64_t v = always_sum;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if (lane == 0 && v) atomicAdd(&np.counters[CNT_CLAMP_ALL], (unsigned long long)v);
  }
  // the workgroup's stream position: one returning atomic, rows padded to whole groups
  uint32_t* np_wc = scratch;                                       // [4]
  unsigned long long* np_base = reinterpret_cast<unsigned long long*>(scratch + 8);
  uint32_t wave_streamed = 0;
#pragma unroll
  for (int q = 0; q < SUB; ++q) wave_streamed += (uint32_t)__popcll(sbal[q]);
  if (lane == 0) np_wc[wv] = wave_streamed;
  __syncthreads();
  const uint32_t tot = np_wc[0] + np_wc[1] + np_wc[2] + np_wc[3];
  if (tid == 0) {
    const uint32_t padded = (tot + FIT_GROUP - 1) / FIT_GROUP * FIT_GROUP;
    *np_base = padded ? atomicAdd(&np.counters[CNT_STREAM], (unsigned long long)padded) : 0ull;
  }
  __syncthreads();
  KCC_TL(rb % 1024, 5);
  uint32_t before = 0;
  for (int u = 0; u < wv; ++u) before += np_wc[u];
  const uint64_t base = *np_base;
  auto put = [&](uint64_t pos, uint64_t fmv, uint32_t fcv, uint32_t Pv, int32_t clv) {
    const int kk = (int)(pos % FIT_GROUP);
    np.fast_cl[pos] = clv;
    FitGroupA& g = np.fast_a[pos / FIT_GROUP];
    g.fm[kk] = fmv;
    g.fc[kk] = fcv;
    g.P[kk] = Pv;
    if (want_b) {
      FitGroup& gb = np.fast_b[pos / FIT_GROUP];
      gb.fc[kk] = (double)fcv;             // exact
      gb.fm[kk] = (double)fmv;             // exact (< 2^50)
      gb.Pb[kk] = FIT_BIAS + (double)Pv;   // exact (P <= 2^20)
    }
  };
  uint32_t done = 0;
#pragma unroll
  for (int q = 0; q < SUB; ++q) {
    if ((sbal[q] >> lane) & 1ull)
      put(base + before + done + (uint32_t)__popcll(sbal[q] & ((1ull << lane) - 1ull)), r_fm[q], r_fc[q],
          (uint32_t)r_P[q], r_cl[q]);
    done += (uint32_t)__popcll(sbal[q]);
  }
  const uint32_t pad = (tot + FIT_GROUP - 1) / FIT_GROUP * FIT_GROUP - tot;
  if ((uint32_t)tid < pad) put(base + tot + tid, 0ull, 0u, 0u, 0);  // the last group's padding
  KCC_TL(rb % 1024, 1);
}

__device__ void np_body(const NpArgs& np, int32_t j, uint32_t* scratch) {
  if (j < np.n_place) {  // spec_place, after the class counts
    np_wait(np.sync + NP_DONE,
            __hip_atomic_load(np.sync + NP_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u, np.faults);
    spec_place_body(np.pa, j);
  } else {
    np_rows(np, j - np.n_place, scratch);
  }
  // the last node-prep workgroup to finish publishes the epoch: every storing reduce wave
  // (each in some row workgroup's window), the rank workgroup and every node-prep workgroup
  // have read it by then
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t total = (uint32_t)(np.n_place + np.n_rows);
    if (__hip_atomic_fetch_add(np.sync + NP_ARRIVE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1u) {
      const uint32_t e = __hip_atomic_load(np.sync + NP_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(np.sync + NP_ARRIVE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(np.sync + NP_EPOCH, e + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
constexpr int64_t CLASS_A_M_MIN = 1ll << 18;    // class A: spec mem >= 2^18, so fm/m < 2^32

__device__ __forceinline__ int32_t spec_class(uint64_t c, int64_t m) {
  if (c < 1 || c >= FAST_C_MAX || m < 1 || m >= FAST_M_MAX) return SPEC_EXACT;
  return m >= CLASS_A_M_MIN ? SPEC_A : SPEC_B;
}

// Smallest f64 >= 1/v (1 <= v < 2^51, exact in f64): the fit's quotients never
// undershoot.
__device__ __forceinline__ double recip_up_f64(uint64_t v) {
  const double vd = (double)v;
  double r = 1.0 / vd;                                   // correctly rounded
  if (fma(r, vd, -1.0) < 0.0) r = __longlong_as_double(__double_as_longlong(r) + 1);  // next up
  return r;
}

// ---- clamp-correction helpers (see ClampWork in kcc_internal.h) ----

__device__ __forceinline__ int64_t clamp_n_normal(const unsigned long long* counters) {
  return (int64_t)(counters[CNT_SPECS_A] + counters[CNT_SPECS_B]);
}
// normal specs whose wavefront has no exact-path lane (the exact path applies the clamp
// itself): all of them, or all but a last wave shared with exact-path specs
__device__ __forceinline__ int64_t clamp_n_pure(int64_t nN, int64_t S) {
  return (nN % 64 == 0 || nN == S) ? nN : nN / 64 * 64;
}

// Slot of entry k (rank k < 4096 of a sorted ascending search table): the BFS
// (Eytzinger) order of the perfect binary tree over entries 0..4094 — slot 1 the root,
// slots 2i and 2i + 1 its children — and entry 4095 in slot 0.  A search walks
// i -> 2i + (a[i] <= v) for 12 levels (one compare and one shift-add per level, no index
// arithmetic), and i - 4096 = #{k < 4095 : a[k] <= v}; slot 0 adds the last entry.  The
// top levels' probes are shared by many lanes (LDS broadcast), the deeper ones spread
// over the banks (a sorted layout's probes, 2^j entries apart, sat in one bank).
__host__ __device__ inline uint32_t np_slot(uint32_t k) {
  if (k == 4095u) return 0u;
  const uint32_t t = (uint32_t)__builtin_ctz(k + 1u);
  return (1u << (11u - t)) + ((k + 1u) >> (t + 1u));
}
// the 64 x 64 member masks mk[g][Y]: Y XOR g, so a row (fixed g) and a column (fixed Y)
// of 32 lanes both hit 32 distinct bank pairs (ds_read_b64)
__device__ __forceinline__ uint32_t mk_at(uint32_t g, uint32_t Y) { return g * 64u + (Y ^ (g & 31u)); }

// #{k < n : a[k] <= v} for a sorted ascending (binary search, n <= 2^31)
template <class T>
__device__ __forceinline__ uint32_t upper_bound_count(const T* __restrict__ a, int64_t n, T v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return (uint32_t)lo;
}

// #{l < 64 : a[l] < v} over one unsorted block of 64 entries (16-B aligned, padding >=
// every v): the counts from global memory (S > CLAMP_LDS_SPECS), 64 compares
// #{entries of a[0..lim) below v} (lim <= 64; the group's padding is not read: spec_place,
// which writes it, may run in the same launch)
__device__ __forceinline__ uint32_t count_lt64(const uint32_t* __restrict__ a, uint32_t v, uint32_t lim) {
  const uint4* q = reinterpret_cast<const uint4*>(a);
  uint32_t n = 0;
#pragma unroll 4
  for (uint32_t u = 0; u < 16; ++u) {
    const uint4 w = q[u];
    n += (w.x < v && 4 * u + 0 < lim ? 1u : 0u) + (w.y < v && 4 * u + 1 < lim ? 1u : 0u) +
         (w.z < v && 4 * u + 2 < lim ? 1u : 0u) + (w.w < v && 4 * u + 3 < lim ? 1u : 0u);
  }
  return n;
}

// Per-node free capacity (CC:119-135 operands).  Rows that fit the fast-path
// bounds get exact FitGroupA fields (and FitGroup fields when class-B specs exist);
// the others get all-zero fields (contribute exactly 0 on the fast paths) and are
// appended to slow_list for the exact path.  Covers the padding of the last group too
// (zero fields, not listed).  SlowNode records are written for the slow rows, and for
// every row when exact-path specs exist (their waves walk all rows).  Clamp correction:
// each fast row with P >= 1 that dominates some spec adds its weight to at most one
// cell each of C, H2 and H3; rows with P <= 0 to C[T+1][T+1] (ClampWork).  C is summed
// in LDS (S <= CLAMP_LDS_SPECS) and added to its copy once per workgroup; H2 / H3 leave as
// binned records (clamp_binned(S)) — no scattered device atomics on the common path.
#define KCC_NODE_PREP_BLOCK 1024
static_assert(CLAMP_PASS_ROWS_MIN == KCC_NODE_PREP_BLOCK, "a pass is 1, 2 or 4 rows per thread");
static_assert(2 * CLAMP_PASS_ROWS_MAX <= 0xffff, "record ranks packed in 16 bits");
__device__ __forceinline__ void np_atomic(int64_t* p, int64_t w) {
  atomic_add_u64(reinterpret_cast<uint64_t*>(p), (uint64_t)w);
}
static_assert(CLAMP_LDS_SPECS % KCC_NODE_PREP_BLOCK == 0, "node_prep table fill");
// workgroups at most (one resident round; each fills its LDS tables once)
constexpr int64_t NODE_PREP_GRID = 1024;
constexpr int NP_C_CELLS = (int)((CLAMP_LDS_SPECS / 64 + 2) * (CLAMP_LDS_SPECS / 64 + 2));
// dynamic LDS: the search tables (cs u32, ms i64, 2 x u16) and the private C table (C summed
// in LDS per workgroup: one node_prep workgroup per CU), when S <= CLAMP_LDS_SPECS
static_assert(CLAMP_LDS_SPECS == 4096, "node_prep's LDS member tables are 64 x 64");
constexpr size_t NP_OFF_CS = 8 * (size_t)CLAMP_LDS_SPECS;            // ms i64, then cs u32
constexpr size_t NP_OFF_MK = NP_OFF_CS + 4 * (size_t)CLAMP_LDS_SPECS;  // 64 x 64 u64 masks
constexpr size_t NP_OFF_CK = NP_OFF_MK + 8 * 64 * 64;                 // 64 x 65 u8
constexpr size_t NP_OFF_CJ = NP_OFF_CK + 64 * 65;                     // 64 x 65 u8
constexpr size_t NP_OFF_C = (NP_OFF_CJ + 64 * 65 + 15) / 16 * 16;     // private C
constexpr size_t NODE_PREP_LDS = NP_OFF_C + 8 * (size_t)NP_C_CELLS;
constexpr int NP_BINS = 2 * (int)CLAMP_BIN_T_MAX;
constexpr uint32_t NP_ST_MAX = 16;  // LDS search tables sample up to 16 x 4096 specs
constexpr size_t NODE_PREP_LDS_SRCH = NP_OFF_MK;  // the search tables alone (S > 4096)
__host__ __device__ inline uint32_t np_stride(int64_t S) {  // smallest power of two >= S / 4096
  uint32_t st = 1;
  while (st < NP_ST_MAX && (int64_t)st * CLAMP_LDS_SPECS < S) st *= 2;
  return st;
}
// MODE 2: S <= 4096, every table in LDS; 1: S <= NP_ST_MAX * 4096, sampled search tables in
// LDS, the rest in memory; 0: everything in memory (one instantiation per mode: each
// carries only its own path's registers).  A pass is SUB x 1024 rows (clamp_pass_rows(n)
// of the call), worked on in SUB sub-steps of one row per thread; each sub-step's rows
// are loaded while the previous one is worked on.
// NC: the clamp in the fit (launch_node_prep's fast_cl; MODE 2 only): no search or count
// tables, no clamp cells or records; each streamed row's clamp value goes to fast_cl and the
// rows clamped for every spec sum into counters[CNT_CLAMP_ALL].
template <int MODE, int SUB, bool NC>
__global__ __launch_bounds__(KCC_NODE_PREP_BLOCK) void node_prep_kernel(int64_t n, const uint64_t* __restrict__ alloc_cpu,
                                 const int64_t* __restrict__ alloc_mem,
                                 const int64_t* __restrict__ alloc_pods,
                                 const int64_t* __restrict__ pod_count,
                                 const uint64_t* __restrict__ used_cpu,
                                 const int64_t* __restrict__ used_mem,
                                 FitGroupA* __restrict__ fast_a, FitGroup* __restrict__ fast_b,
                                 SlowNode* __restrict__ slow, int64_t* __restrict__ slow_list,
                                 int64_t S, ClampWork cw,
                                 unsigned long long* __restrict__ counters,
                                 int32_t chunk, int32_t dense, int64_t pass0, PlaceArgs pa,
                                 int32_t* __restrict__ fast_cl) {
  static_assert(!NC || MODE == 2, "the clamp in the fit: S <= CLAMP_LDS_SPECS only");
  if ((int32_t)blockIdx.x < pa.n_blocks) {  // spec_place's workgroups, in front (MODE 2)
    spec_place_body(pa, blockIdx.x);
    return;
  }
  const int32_t bid = (int32_t)blockIdx.x - pa.n_blocks, nbid = (int32_t)gridDim.x - pa.n_blocks;
  KCC_TL(bid % 1024, 2);
  constexpr int64_t PR = (int64_t)KCC_NODE_PREP_BLOCK * SUB;  // rows per pass
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t stride = (int64_t)nbid * PR;
  // one row's six values: the next sub-step's, loaded while the current one is worked on;
  // this workgroup's first ones go out before the table setup below (their latency hides
  // behind it)
  uint64_t ld_ac, ld_uc;
  int64_t ld_am, ld_um, ld_P, ld_pc;
  auto load_row = [&](int64_t i) {
    ld_ac = ld_uc = 0;
    ld_am = ld_um = ld_P = ld_pc = 0;
    if (i < n) {
      ld_ac = alloc_cpu[i];
      ld_uc = used_cpu[i];
      ld_am = alloc_mem[i];
      ld_um = used_mem[i];
      ld_P = alloc_pods[i];
      ld_pc = pod_count[i];
    }
  };
  load_row((int64_t)bid * PR + threadIdx.x);
  __shared__ uint32_t np_wc[KCC_NODE_PREP_BLOCK / 64];  // streamed rows per wave
  __shared__ uint64_t np_base;                          // this pass's stream position
  __shared__ uint32_t np_tot;
  __shared__ uint32_t np_bcnt[NP_BINS];                 // binned records per bin (this pass)
  __shared__ uint32_t np_bstart[NP_BINS];               // their exclusive prefix
  // the class counts from spec_rank's per-block counts (spec_place may run beside this
  // launch): every wave sums them (one load per lane at S <= 4096)
  uint64_t cls_n = 0;  // class A | class B << 32
  {
    const uint64_t* bc = reinterpret_cast<const uint64_t*>(cw.bcnt);
    for (int64_t b = lane; b < (S + 63) / 64; b += 64) cls_n += bc[b];
    cls_n = readlane_u64(wave_incl_scan_u64(cls_n), 63);
  }
  const bool want_b = (cls_n >> 32) != 0;                       // class-B specs exist
  const int64_t nN = (int64_t)(uint32_t)cls_n + (int64_t)(cls_n >> 32);  // normal specs
  const bool slow_all = nN < S;                    // exact-path specs exist
  const int64_t T = (nN + 63) / 64, W = T + 2;
  // T <= CLAMP_BIN_T_MAX (always at S <= 4096: MODE 2 carries no table atomics)
  const bool binned = MODE == 2 || clamp_binned(S);
  const int NB = (int)(2 * T);                     // bins: x-groups, then y-blocks
  // this workgroup's copies of the tables: workgroups are dealt round-robin over the XCDs
  int64_t* Cc = cw.C + (int64_t)(bid % C_COPIES) * cw.c_stride;
  int64_t* H2c = cw.H2 + (int64_t)(bid % H2_COPIES) * cw.h_stride;
  int64_t* H3c = cw.H3 + (int64_t)(bid % H2_COPIES) * cw.h_stride;
  // in LDS when S <= CLAMP_LDS_SPECS: the sorted spec requests of the searches (c clamped
  // to 2^23 (> every U = fc / P, fc < 2^23) as u32, m as i64); the member tables of the
  // x-group / y-block counts: mk[g][Y] = bit set of the y-ranks in y-block Y of x-group g's
  // specs, ck[g][Y] = #{specs of x-group g with y < 64 Y}, cj[Y][G] = #{specs of y-block
  // Y whose x-group < G}; then C's private copy
  extern __shared__ __attribute__((aligned(16))) unsigned char np_lds[];
  int64_t* ms_l = reinterpret_cast<int64_t*>(np_lds);
  uint32_t* cs_l = reinterpret_cast<uint32_t*>(np_lds + NP_OFF_CS);
  unsigned long long* mk_l = reinterpret_cast<unsigned long long*>(np_lds + NP_OFF_MK);
  uint8_t* ck_l = np_lds + NP_OFF_CK;
  uint8_t* cj_l = np_lds + NP_OFF_CJ;
  unsigned long long* c_l = reinterpret_cast<unsigned long long*>(np_lds + NP_OFF_C);
  constexpr bool lds = MODE == 2;  // S <= CLAMP_LDS_SPECS: T <= 64 and W * W <= NP_C_CELLS
  constexpr bool cpriv = lds;
  // the search tables in LDS hold every st-th request (st = 1 when S <= 4096; a search
  // ends with the st - 1 requests of its bucket from memory), up to NP_ST_MAX
  constexpr bool srch = MODE >= 1;
  const uint32_t st = lds ? 1u : np_stride(S);
  for (int b = threadIdx.x; b < NP_BINS; b += KCC_NODE_PREP_BLOCK) np_bcnt[b] = 0;
  constexpr int PER = (int)(CLAMP_LDS_SPECS / KCC_NODE_PREP_BLOCK);
  uint32_t yv[PER];  // y-rank of x-rank tid + 1024 u
  if (srch && !NC) {
    // the sorted requests (spec_rank's last arrivers write them): every load first, guarded by S (a kernel argument) rather than nN, so they
    // travel with the class counts' load (one memory round trip); entries nN.. are masked
    uint64_t cv[PER], mv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t k = threadIdx.x + (int64_t)KCC_NODE_PREP_BLOCK * u;
      const int64_t e = (k + 1) * st - 1;  // the sampled entry
      cv[u] = e < S ? cw.cs[e] : ~0ull;
      mv[u] = e < S ? (uint64_t)cw.ms[e] : (uint64_t)INT64_MAX;
      yv[u] = lds && k < S ? cw.mr_c[k] : 0xffffffffu;
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t k = threadIdx.x + (int64_t)KCC_NODE_PREP_BLOCK * u;
      const bool in = (k + 1) * st - 1 < nN;  // padded: +inf
      cs_l[np_slot((uint32_t)k)] = in && cv[u] < FAST_FC_MAX ? (uint32_t)cv[u] : 0xffffffffu;
      ms_l[np_slot((uint32_t)k)] = in ? (int64_t)mv[u] : INT64_MAX;
      if (!in) yv[u] = 0xffffffffu;
      if (lds) mk_l[k] = 0ull;  // 64 x 64 masks: one per spec slot
    }
    if (cpriv)
      for (int64_t e = threadIdx.x; e < W * W; e += KCC_NODE_PREP_BLOCK) c_l[e] = 0ull;
  }
  __syncthreads();  // masks zero
  KCC_TL(bid % 1024, 6);
  if (lds && !NC) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t x = threadIdx.x + (int64_t)KCC_NODE_PREP_BLOCK * u;
      if (x < nN)
        __hip_atomic_fetch_or((lds_ull*)(mk_l + mk_at((uint32_t)x >> 6, yv[u] >> 6)), 1ull << (yv[u] & 63),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();  // masks complete
  KCC_TL(bid % 1024, 7);
  // smallest normal requests (rows below either dominate no spec): the tables' first
  // entries (+inf when there are none; cs[0] >= 1; MODE 1's LDS tables are sampled)
  const uint32_t cmin = NC ? 0u : lds ? cs_l[np_slot(0u)]
                            : (nN > 0 ? (cw.cs[0] < FAST_FC_MAX ? (uint32_t)cw.cs[0] : 0xffffffffu)
                                      : 0xffffffffu);
  const int64_t mmin = NC ? 0 : lds ? ms_l[np_slot(0u)] : (nN > 0 ? cw.ms[0] : INT64_MAX);
  if (lds && !NC) {  // the prefix counts: row g along Y and column Y = g along G, lane = index;
    // rows g and g + 16 in one 32-bit scan of four byte fields (each count and prefix is
    // a member count of one x-group or y-block, <= 64: no carries between the bytes)
    static_assert(KCC_NODE_PREP_BLOCK == 1024, "16 waves: rows wv, wv + 16, wv + 32, wv + 48");
    for (int g = wv; g < 64; g += 32) {
      const uint32_t pk = (uint32_t)__popcll(mk_l[mk_at(g, lane)]) |
                          (uint32_t)__popcll(mk_l[mk_at(lane, g)]) << 8 |
                          (uint32_t)__popcll(mk_l[mk_at(g + 16, lane)]) << 16 |
                          (uint32_t)__popcll(mk_l[mk_at(lane, g + 16)]) << 24;
      const uint32_t inc = wave_incl_scan_u32(pk), exc = inc - pk;
      ck_l[g * 65 + lane] = (uint8_t)exc;
      cj_l[g * 65 + lane] = (uint8_t)(exc >> 8);
      ck_l[(g + 16) * 65 + lane] = (uint8_t)(exc >> 16);
      cj_l[(g + 16) * 65 + lane] = (uint8_t)(exc >> 24);
      if (lane == 63) {
        ck_l[g * 65 + 64] = (uint8_t)inc;
        cj_l[g * 65 + 64] = (uint8_t)(inc >> 8);
        ck_l[(g + 16) * 65 + 64] = (uint8_t)(inc >> 16);
        cj_l[(g + 16) * 65 + 64] = (uint8_t)(inc >> 24);
      }
    }
  }
  // a C cell: the workgroup's LDS copy (an explicit LDS pointer: through the lambda the
  // generic pointer became flat atomics), or the device copy
  auto c_add = [&](int64_t cell, int64_t w) {
    if (cpriv) lds_add_u64(c_l + cell, (uint64_t)w);
    else np_atomic(&Cc[cell], w);
  };
  __syncthreads();
  KCC_TL(bid % 1024, 0);
  // Passes of SUB x 1024 rows (thread t: rows i0 + t + 1024 q), one sub-step q after the
  // other; one stream position (a returning atomic on one word) and one bin scan per pass.
  // Workgroup-uniform trip count (the stream positions and the bins meet in LDS).
  for (int64_t i0 = (int64_t)bid * PR; i0 < n; i0 += stride) {
    const int64_t pass = pass0 + i0 / PR;
    // kept to the pass's end: the stream entry of each sub-step's row (free memory < 2^50,
    // free cpu < 2^23 and P of a fast row, else 0), its ballots, the packed records
    uint64_t r_fm[SUB];
    uint32_t r_fc[SUB];
    int32_t r_P[SUB];
    int32_t r_cl[SUB];  // NC: the clamp value of a streamed row
    unsigned long long sbal[SUB];
    uint32_t pk1[SUB], pk2[SUB], pk3[SUB];
    uint64_t always_sum = 0;
    uint64_t base_ret = 0;
    uint32_t t_pass = 0;
#pragma unroll
    for (int q = 0; q < SUB; ++q) {
      const int64_t i = i0 + q * KCC_NODE_PREP_BLOCK + threadIdx.x;
      const bool valid = i < n;
      // phase 1: the free capacity, the slow rows; the 64-bit loads die here
      bool ok = false;
      int32_t cl_q = 0;
      r_fm[q] = 0;
      r_fc[q] = 0;
      r_P[q] = 0;
      if (valid) {
        const uint64_t fc = ld_ac > ld_uc ? ld_ac - ld_uc : 0;                                 // CC:119-123
        const int64_t fm = ld_am > ld_um ? (int64_t)((uint64_t)ld_am - (uint64_t)ld_um) : 0;  // CC:125-129
        const int64_t P = ld_P;
        const int64_t cl = (int64_t)((uint64_t)P - (uint64_t)ld_pc);                          // CC:135
        ok = fc < FAST_FC_MAX && fm >= 0 && fm < FAST_FM_MAX && P >= -FAST_P_ABS &&
             P <= FAST_P_ABS && cl >= -FAST_CL_ABS && cl <= FAST_CL_ABS;
        if (ok) {
          r_fm[q] = (uint64_t)fm;
          r_fc[q] = (uint32_t)fc;
          r_P[q] = (int32_t)P;
          cl_q = (int32_t)cl;
        }
        if (slow_all || !ok) {
          SlowNode sn;
          sn.fc = fc;
          sn.fm = fm;
          sn.P = P;
          sn.cl = cl;
          slow[i] = sn;
        }
      }
      {
        const unsigned long long bl = __ballot(valid && !ok);
        if (bl) {
          unsigned long long base = 0;
          if (lane == 0)
            base = atomicAdd(&counters[CNT_SLOW_ROWS + chunk], (unsigned long long)__popcll(bl));
          base = __shfl(base, 0);
          if (valid && !ok) slow_list[base + __popcll(bl & ((1ull << lane) - 1ull))] = i;
        }
      }
      // the next sub-step's row (the load registers are free now)
      load_row(q + 1 < SUB ? i + KCC_NODE_PREP_BLOCK : i0 + stride + threadIdx.x);
      // the fit's node stream: the rows with something to add
      sbal[q] = __ballot(dense ? valid : (r_fc[q] > 0 && r_fm[q] > 0 && r_P[q] > 0));  // 0 unless ok
      if (q == SUB - 1) {
        // every sub-step's ballots are known: the pass's stream position (one returning
        // atomic by thread 0) is in flight during the last phase 2
        uint32_t wave_streamed = 0;
#pragma unroll
        for (int q2 = 0; q2 < SUB; ++q2) wave_streamed += (uint32_t)__popcll(sbal[q2]);
        if (lane == 0) np_wc[wv] = wave_streamed;
        __syncthreads();  // np_wc
        if (threadIdx.x == 0) {
          for (int u = 0; u < KCC_NODE_PREP_BLOCK / 64; ++u) t_pass += np_wc[u];
          const uint32_t padded = (t_pass + FIT_GROUP - 1) / FIT_GROUP * FIT_GROUP;  // whole groups
          if (padded) base_ret = atomicAdd(&counters[CNT_STREAM + chunk], (unsigned long long)padded);
        }
        KCC_TL(bid % 1024, 3);
      }
      // phase 2: the clamp correction's cells and records, in steps without data-dependent
      // branches around the LDS reads: (a) weight and bounds, (b) the two binary searches,
      // (c) the member counts, (d) cells and bin ranks
      // (a) c <= U  <=>  floor(fc / c) >= P  and  m <= V  <=>  floor(fm / m) >= P, with
      // U = floor(fc / P), V = floor(fm / P) from the rounded-up reciprocal of P (exact:
      // fc, fm < 2^50, P < 2^51); U < cmin or V < mmin: no spec dominated
      const int64_t P = r_P[q], Penc = P > 0 ? P : 0;
      const int64_t wfull = Penc - (int64_t)cl_q;  // contribution = min(x, Penc) - w when clamped
      if (ok && nN > 0 && P <= 0) always_sum += (uint64_t)wfull;  // x >= P for every spec
      r_cl[q] = cl_q;
      if constexpr (NC) {
        pk1[q] = pk2[q] = pk3[q] = 0u;
      } else {
      const double rP = recip_up_f64(P > 0 ? (uint64_t)P : 1ull);
      const int64_t V0 = (int64_t)((double)r_fm[q] * rP);  // floor(fm / P): exact (§5)
      const uint32_t U0 = (uint32_t)((double)r_fc[q] * rP);
      const bool act = ok && nN > 0 && P > 0 && wfull != 0 && U0 >= cmin && V0 >= mmin;
      const int64_t w = act ? wfull : 0;  // |w| <= 2^21
      const uint32_t U = act ? U0 : 0u;   // every request is >= 1: counts 0
      const int64_t V = act ? V0 : 0;
      uint32_t L = 0, b = 0;
      if (srch) {  // (b) over the LDS tables (every st-th request), then the bucket in memory
        uint32_t iL = 1, ib = 1;  // np_slot's tree
#pragma unroll
        for (int lv = 0; lv < 12; ++lv) {
          iL = 2 * iL + (cs_l[iL] <= U ? 1u : 0u);
          ib = 2 * ib + (ms_l[ib] <= V ? 1u : 0u);
        }
        L = iL - 4096u;
        b = ib - 4096u;
        L += L == 4095u && cs_l[0] <= U ? 1u : 0u;  // the last entry (slot 0)
        b += b == 4095u && ms_l[0] <= V ? 1u : 0u;
        if (!lds) {  // st > 1: #{a <= v} = c st + #{j < st - 1 : a[c st + j] <= v} (a[(c + 1) st - 1] > v)
          L *= st;
          b *= st;
          uint32_t addL = 0, addb = 0;
#pragma unroll 4
          for (uint32_t j = 0; j + 1 < st; ++j) {  // uniform trip count
            addL += w && L + j < (uint64_t)nN && cw.cs[L + j] <= (uint64_t)U ? 1u : 0u;
            addb += w && b + j < (uint64_t)nN && cw.ms[b + j] <= V ? 1u : 0u;
          }
          L += addL;
          b += addb;
        }
      } else {  // S > NP_ST_MAX * 4096: binary searches in memory
        L = w ? upper_bound_count(cw.cs, nN, (uint64_t)U) : 0u;
        b = w ? upper_bound_count(cw.ms, nN, V) : 0u;
      }
      // (c) L >= 1 and b >= 1 for an active row; L = 64 GX + rx, b = 64 GY + ry.  H2's
      // k = #{specs of x-group GX with y < b} (rx > 0, so GX < T), H3's j = #{specs of
      // y-block GY whose x-group < GX} (ry > 0, GY < T)
      const uint32_t GX = L >> 6, rx = L & 63u, GY = b >> 6, ry = b & 63u;
      uint32_t k, j;
      if (lds) {  // the members below y-block b >> 6, + those in it below b
        const uint32_t gx = GX < 63u ? GX : 63u, yb = GY < 63u ? GY : 63u;
        const uint64_t mk = mk_l[mk_at(gx, yb)];
        k = (uint32_t)ck_l[gx * 65 + GY] + (uint32_t)__popcll(mk & ((1ull << ry) - 1ull));
        j = cj_l[yb * 65 + GX];
      } else {  // x >> 6 < GX  <=>  x < 64 GX (the groups' members below nN only)
        const int64_t mx = nN - 64 * (int64_t)GX, my = nN - 64 * (int64_t)GY;
        k = w && rx ? count_lt64(cw.mr_c + 64 * GX, b, (uint32_t)(mx < 64 ? mx : 64)) : 0u;
        j = w && ry && GX > 0 ? count_lt64(cw.cr_m + 64 * GY, GX << 6, (uint32_t)(my < 64 ? my : 64)) : 0u;
      }
      // (d)
      if (w && GX > 0 && GY > 0) c_add((int64_t)GX * W + GY, w);
      const bool has2 = w && rx > 0 && k > 0;            // first rx members of x-group GX
      const bool has3 = w && ry > 0 && GX > 0 && j > 0;  // members of y-block GY in x-groups < GX
      if (!binned) {
        if (has2) np_atomic(&H2c[((int64_t)GX * 65 + k) * 64 + rx], w);
        if (has3) np_atomic(&H3c[((int64_t)GY * 65 + j) * 64 + ry], w);
      }
      const bool rec2 = binned && has2, rec3 = binned && has3;
      const uint32_t bin2 = rec2 ? GX : 0u, bin3 = rec3 ? (uint32_t)T + GY : 0u;
      // the records in three words: cells (13 bits each, 0: no record — a record's cell
      // is >= 64), ranks within their bins (LDS counters, < 2^13 per pass: zeroed by the
      // scan below), bins (9 bits each), and the weight (|w| <= 2^21, 23 bits) in 6/6/11
      // bit slices: pk1 = cell2 | cell3 << 13 | w[0:6] << 26, pk2 = rk2 | rk3 << 13 |
      // w[6:12] << 26, pk3 = bin2 | bin3 << 9 | w[12:] << 18 (arithmetic)
      const uint32_t rk2 = rec2 ? atomicAdd(&np_bcnt[bin2], 1u) : 0u;
      const uint32_t rk3 = rec3 ? atomicAdd(&np_bcnt[bin3], 1u) : 0u;
      const uint32_t wu = (uint32_t)(int32_t)w;
      pk1[q] = (rec2 ? k * 64 + rx : 0u) | (rec3 ? j * 64 + ry : 0u) << 13 | (wu & 63u) << 26;
      pk2[q] = rk2 | rk3 << 13 | ((wu >> 6) & 63u) << 26;
      pk3[q] = bin2 | bin3 << 9 | (uint32_t)((int32_t)wu >> 12) << 18;
      }  // (!NC)
      // the scheduler keeps each sub-step to itself (hoisting the next one's work
      // across this point ran the SUB = 4 kernels out of registers)
      __builtin_amdgcn_sched_barrier(0);
    }
    {  // rows clamped for every spec: one wave-summed add into C[T+1][T+1]
      uint64_t v = always_sum;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
      if (NC) {
        if (lane == 0 && v) atomicAdd(&counters[CNT_CLAMP_ALL], (unsigned long long)v);
      } else if (lane == 0 && v) {
        c_add((T + 1) * W + T + 1, (int64_t)v);
      }
    }
    if (threadIdx.x == 0) {
      np_base = base_ret;
      np_tot = t_pass;
    }
    __syncthreads();  // np_base, and every record's rank
    KCC_TL(bid % 1024, 4);
    if (binned && !NC && wv == 1) {
      // the bins' starts: runs of per bins per lane, a shuffle scan of the run totals;
      // the pass's directory row (starts + total) goes out here, the counters return to 0
      const int per = (NB + 63) / 64;
      const int b0 = lane * per, b1 = min(b0 + per, NB);
      uint32_t ls = 0;
      for (int bb = b0; bb < b1; ++bb) ls += np_bcnt[bb];
      uint32_t li = ls;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(li, d, 64);
        if (lane >= d) li += t;
      }
      uint32_t* drow = cw.dir + pass * cw.d_stride;
      uint32_t run = li - ls;
      for (int bb = b0; bb < b1; ++bb) {
        const uint32_t c = np_bcnt[bb];
        np_bstart[bb] = run;
        drow[bb] = run;
        np_bcnt[bb] = 0;
        run += c;
      }
      if (lane == 63) drow[NB] = li;
    }
    __syncthreads();
    {
      uint32_t before = 0;
      for (int u = 0; u < wv; ++u) before += np_wc[u];
      const uint64_t sb0 = np_base + before;
      const uint32_t tot = np_tot;
      const uint32_t pad = (tot + FIT_GROUP - 1) / FIT_GROUP * FIT_GROUP - tot;
// (non-temporal stores here, so fewer dirty lines wait for the end-of-kernel write-back,
// measured: C4 step 0.2895 -> 0.3171 ms — the rows' scattered partial-group stores then
// reach HBM one by one — 8-way rank 0.0594 -> 0.0582; round 5, profiles/r05_ab_np_nt.txt)
#define NP_ST(ref, v) ((ref) = (v))
      auto put = [&](uint64_t pos, uint64_t fmv, uint32_t fcv, uint32_t Pv, int32_t clv) {
        const int kk = (int)(pos % FIT_GROUP);
        if (NC) NP_ST(fast_cl[pos], clv);
        FitGroupA& a = fast_a[pos / FIT_GROUP];
        NP_ST(a.fm[kk], fmv);
        NP_ST(a.fc[kk], fcv);
        NP_ST(a.P[kk], Pv);
        if (want_b) {
          FitGroup& g = fast_b[pos / FIT_GROUP];
          NP_ST(g.fc[kk], (double)fcv);                      // exact
          NP_ST(g.fm[kk], (double)fmv);                      // exact (< 2^50)
          NP_ST(g.Pb[kk], FIT_BIAS + (double)Pv);            // exact (P <= 2^20)
        }
      };
      uint32_t done = 0;  // streamed rows of this wave's earlier sub-steps
      uint64_t* prec = cw.rec + pass * (2 * PR);
#pragma unroll
      for (int q = 0; q < SUB; ++q) {
        if ((sbal[q] >> lane) & 1ull)  // P <= 0 streams only in the dense layout, as P = 0
          put(sb0 + done + (uint32_t)__popcll(sbal[q] & ((1ull << lane) - 1ull)), r_fm[q], r_fc[q],
              r_P[q] > 0 ? (uint32_t)r_P[q] : 0u, r_cl[q]);
        done += (uint32_t)__popcll(sbal[q]);
        const uint32_t c2 = pk1[q] & 0x1fffu, c3 = (pk1[q] >> 13) & 0x1fffu;
        if (c2 | c3) {
          const int32_t wr = (int32_t)pk3[q] >> 18 << 12 | (int32_t)((pk2[q] >> 26) << 6 | pk1[q] >> 26);
          const uint64_t wbits = (uint64_t)(uint32_t)wr << 32;  // record: cell | w << 32
          if (c2) NP_ST(prec[np_bstart[pk3[q] & 0x1ffu] + (pk2[q] & 0x1fffu)], wbits | c2);
          if (c3) NP_ST(prec[np_bstart[(pk3[q] >> 9) & 0x1ffu] + ((pk2[q] >> 13) & 0x1fffu)], wbits | c3);
        }
      }
      if (threadIdx.x < pad) put(np_base + tot + threadIdx.x, 0ull, 0u, 0u, 0);  // the last group's padding
    }
    __syncthreads();  // np_wc / np_base / np_bstart are rewritten by the next pass
    KCC_TL(bid % 1024, 5);
  }
  if (cpriv && !NC) {  // the private C into this workgroup's device copy: its non-zero cells
    for (int64_t e = threadIdx.x; e < W * W; e += KCC_NODE_PREP_BLOCK) {
      const unsigned long long v = c_l[e];
      if (v) np_atomic(&Cc[e], (int64_t)v);
    }
  }
  KCC_TL(bid % 1024, 1);
}

// Smallest f32 >= 1/v (1 <= v < 2^51, exact in f64).  1/v is first rounded to f64,
// then to f32 (a double rounding can only land on the upper neighbour when that one is
// already the smallest upper bound); the exact sign of r*v - 1 (fma, one rounding of a
// value that is either 0 or >= 2^-75 in magnitude) fixes an undershoot.
__device__ __forceinline__ float recip_up_f32(uint64_t v) {
  const double vd = (double)v;
  float r = (float)(1.0 / vd);
  if (fma((double)r, vd, -1.0) < 0.0) r = __uint_as_float(__float_as_uint(r) + 1u);  // next up
  return r;
}


// ---- spec setup: ranks (slices), then one thread per spec places it -----------------

// The rank of every normal spec (ties by index):
//   x(i) = #{normal j : (c_j, j) < (c_i, i)},   y(i) = #{normal j : (m_j, j) < (m_i, i)},
// summed over slices of RANK_L candidates with 64-bit keys v << 13 | (j mod 8192) (v = c or
// m < 2^51; non-normal specs ~0).  A slice's share is the count of its keys below a
// threshold: (v_i + 1) << 13 for an earlier slice (equal v sorts before; v_i = 2^51 - 1:
// every normal candidate), v_i << 13 | (i mod 8192) for i's own slice, v_i << 13 for a later
// one (RANK_L divides 8192: a slice never straddles two 8192-chunks, so j mod 8192 orders
// it by index).  Each slice stores its x / y counts write-through (sc1) and waits for them;
// the workgroup then adds to its query block's arrival counter (after the barrier that
// follows every wave's wait); the one that arrives last reads every slice (sc1 loads, after
// its add returned), writes the sorted arrays (cs, ms, mr_c, cr_m) and the ranks (x at
// rank[i], y at rank[S + i]), and resets the counter.  The slice-0 workgroups store
// the class-A / class-B counts of their 64-query blocks in bcnt[].  Every rank workgroup
// also zeroes its share of the counters (but the class counts, spec_place's) and of the
// coarse clamp table's cells (spec_rank_body).  `lds`: 16 KiB.
//
// S <= RANK_FULL_MAX: counting.  Workgroup (qb, sl) of ceil(S/64) x rank_slices(S); lane =
// query i = 64 qb + lane (the 4 waves hold the same 64 queries), the slice's RANK_L keys
// staged in LDS, a quarter per wave, read by broadcast and compared with the threshold.
// C4 (S = 4096): 256 workgroups of ~1 us riding in the reduce launch.
__device__ void spec_rank_count(const RankArgs& ra, int64_t blk, uint64_t* lds) {
  const int64_t S = ra.S;
  const uint64_t* __restrict__ c_in = ra.c_in;
  const int64_t* __restrict__ m_in = ra.m_in;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  typedef uint64_t u64x2_t __attribute__((ext_vector_type(2)));
  u64x2_t* key_l = reinterpret_cast<u64x2_t*>(lds);
  uint32_t* part = reinterpret_cast<uint32_t*>(lds);
  const int64_t ns = rank_slices(S);
  const int64_t qb = blk / ns, sl = blk % ns;
  const int64_t i = qb * 64 + lane;  // this lane's query
  const bool qv = i < S;
  const uint64_t c = qv ? c_in[i] : 0;
  const int64_t m = qv ? m_in[i] : 0;
  const int32_t ci = qv ? spec_class(c, m) : SPEC_EXACT;
  if (sl == 0 && wv == 0) {  // this query block's class counts
    const uint32_t na = (uint32_t)__popcll(__ballot(ci == SPEC_A));
    const uint32_t nb = (uint32_t)__popcll(__ballot(ci == SPEC_B));
    if (lane == 0) {
      ra.bcnt[2 * qb] = na;
      ra.bcnt[2 * qb + 1] = nb;
    }
  }
  const int64_t j0 = sl * RANK_L, j1 = j0 + RANK_L < S ? j0 + RANK_L : S;  // this slice
  for (int64_t j = j0 + tid; j < j1; j += 256) {  // stage the slice's keys
    const uint64_t cj = c_in[j];
    const int64_t mj = m_in[j];
    const bool nj = spec_class(cj, mj) != SPEC_EXACT;
    u64x2_t k;
    k.x = nj ? cj << 13 | (uint64_t)(j & 8191) : ~0ull;
    k.y = nj ? (uint64_t)mj << 13 | (uint64_t)(j & 8191) : ~0ull;
    key_l[j - j0] = k;
  }
  __syncthreads();
  const int64_t chq = i >> 13, chs = j0 >> 13;  // 8192-chunks of the query and the slice
  const uint64_t tc = chs < chq ? (c + 1) << 13 : (chs == chq ? c << 13 | (uint64_t)(i & 8191) : c << 13);
  const uint64_t tm = chs < chq ? ((uint64_t)m + 1) << 13
                                : (chs == chq ? (uint64_t)m << 13 | (uint64_t)(i & 8191) : (uint64_t)m << 13);
  const int n = (int)(j1 - j0);
  const int w0 = n * wv / 4, w1 = n * (wv + 1) / 4;  // this wave's quarter
  uint32_t rc = 0, rm = 0;
#pragma unroll 4
  for (int j = w0; j < w1; ++j) {
    const u64x2_t k = key_l[j];  // broadcast read
    rc += k.x < tc ? 1u : 0u;
    rm += k.y < tm ? 1u : 0u;
  }
  __syncthreads();  // the keys are read: the area takes the waves' counts
  part[(wv * 2 + 0) * 64 + lane] = rc;
  part[(wv * 2 + 1) * 64 + lane] = rm;
  __syncthreads();
  uint32_t* const slices = ra.part + 2 * S;  // [ns][2][S]
  if (wv < 2) {  // wave r: count r of this slice
    const uint32_t t = part[(0 * 2 + wv) * 64 + lane] + part[(1 * 2 + wv) * 64 + lane] +
                       part[(2 * 2 + wv) * 64 + lane] + part[(3 * 2 + wv) * 64 + lane];
    if (qv) __hip_atomic_store(slices + (sl * 2 + wv) * S + i, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();  // every storing wave has waited for its stores
  uint32_t& last_s = rank_small(lds)[0];
  if (tid == 0)
    last_s = ns == 1 ? 1u
                     : (uint32_t)(__hip_atomic_fetch_add(ra.arrive + qb, 1u, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)ns - 1u);
  __syncthreads();
  if (!last_s || wv != 0) return;  // (workgroup-uniform, then wave 0 alone)
  asm volatile("" ::: "memory");   // the slices' loads only after the arrival returned
  if (ns > 1 && lane == 0) ra.arrive[qb] = 0;  // every slice has arrived: reset for the next call
  if (!qv || ci == SPEC_EXACT) return;
  uint32_t x = 0, y = 0;
  for (int64_t k = 0; k < ns; ++k) {
    x += __hip_atomic_load(slices + (k * 2 + 0) * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    y += __hip_atomic_load(slices + (k * 2 + 1) * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ra.cs[x] = c;
  ra.ms[y] = m;
  ra.mr_c[x] = y;
  ra.cr_m[y] = x;
  ra.part[i] = x;
  ra.part[S + i] = y;
}

// S > RANK_FULL_MAX: sort and search, O(S log S).  Workgroup (qb, sl) of rank_slices(S)^2;
// query block qb = the specs [RANK_L qb, RANK_L (qb + 1)) (4 per thread); the workgroup sorts
// its slice's keys (bitonic network: registers, then LDS exchanges) and finds each query's
// count by binary search.  C5 (S = 16384): 256 workgroups (round 2 counted every candidate
// per query: 4096 workgroups, 44 us in a launch of its own).
__device__ void spec_rank_sort(const RankArgs& ra, int64_t blk, uint64_t* lds) {
  const int64_t S = ra.S;
  const uint64_t* __restrict__ c_in = ra.c_in;
  const int64_t* __restrict__ m_in = ra.m_in;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t ns = rank_slices(S);
  const int64_t qb = blk / ns, sl = blk % ns;
  // the slice's candidates j0 + 4 tid + q (q < 4), keys v << 13 | (j mod 8192) (v < 2^51 for
  // normal specs; RANK_L divides 8192, so within the slice the key orders (v, j)), ~0 for
  // the others; sorted ascending by a bitonic network: stages within the 4 registers of a
  // thread (j < 4), across the lanes of a wave (j < 256: the partner's key of the same q in
  // lane l ^ (j / 4)), across waves through LDS (j >= 256)
  const int64_t j0 = sl * RANK_L;
  uint64_t kx[4], ky[4];
  uint32_t nrm = 0;  // normal candidates among this thread's 4
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t j = j0 + 4 * tid + q;
    const uint64_t cj = j < S ? c_in[j] : 0;
    const int64_t mj = j < S ? m_in[j] : 0;
    const bool nj = j < S && spec_class(cj, mj) != SPEC_EXACT;
    kx[q] = nj ? cj << 13 | (uint64_t)(j & 8191) : ~0ull;
    ky[q] = nj ? (uint64_t)mj << 13 | (uint64_t)(j & 8191) : ~0ull;
    nrm += nj ? 1u : 0u;
  }
  uint64_t* const lx = lds;           // [RANK_L] x keys
  uint64_t* const ly = lds + RANK_L;  // [RANK_L] y keys
  auto cx = [](uint64_t& a, uint64_t& b, bool asc) {  // a <= b afterwards when asc
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = asc ? lo : hi;
    b = asc ? hi : lo;
  };
  typedef uint64_t u64x2_t __attribute__((ext_vector_type(2)));
  // partner lane l ^ m of a wave-local stage (m = j / 4 < 64): DPP quad permutes (m = 1, 2),
  // ds_swizzle bit masks within 32 lanes (m = 4, 8, 16), ds_bpermute (m = 32); the network
  // is fully unrolled, so m is a constant at every call
  auto xlane = [&](uint32_t v, int msk) -> uint32_t {
    switch (msk) {
      case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
      case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
      case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
      case 8: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (8 << 10));
      case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (16 << 10));
      default: return (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, (int)v);
    }
  };
  auto xlane64 = [&](uint64_t v, int msk) -> uint64_t {
    return (uint64_t)xlane((uint32_t)(v >> 32), msk) << 32 | xlane((uint32_t)v, msk);
  };
#pragma unroll
  for (int k = 2; k <= RANK_L; k <<= 1) {
#pragma unroll
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      if (jj >= 256) {  // partner thread in another wave: through LDS
        const int pt = tid ^ (jj >> 2);
        u64x2_t* wx = reinterpret_cast<u64x2_t*>(lx + 4 * tid);
        u64x2_t* wy = reinterpret_cast<u64x2_t*>(ly + 4 * tid);
        wx[0] = u64x2_t{kx[0], kx[1]};
        wx[1] = u64x2_t{kx[2], kx[3]};
        wy[0] = u64x2_t{ky[0], ky[1]};
        wy[1] = u64x2_t{ky[2], ky[3]};
        __syncthreads();
        const u64x2_t* rx = reinterpret_cast<const u64x2_t*>(lx + 4 * pt);
        const u64x2_t* ry = reinterpret_cast<const u64x2_t*>(ly + 4 * pt);
        const u64x2_t px0 = rx[0], px1 = rx[1], py0 = ry[0], py1 = ry[1];
        const uint64_t px[4] = {px0.x, px0.y, px1.x, px1.y}, py[4] = {py0.x, py0.y, py1.x, py1.y};
        const bool asc = ((4 * tid) & k) == 0, lower = (tid & (jj >> 2)) == 0;
        const bool keep_min = asc == lower;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          kx[q] = keep_min ? (kx[q] < px[q] ? kx[q] : px[q]) : (kx[q] < px[q] ? px[q] : kx[q]);
          ky[q] = keep_min ? (ky[q] < py[q] ? ky[q] : py[q]) : (ky[q] < py[q] ? py[q] : ky[q]);
        }
        __syncthreads();  // every partner has read before the next writes
      } else if (jj >= 4) {  // partner lane l ^ (j / 4) of the same wave, same q
        const int msk = jj >> 2;
        // element 4 tid + q: ascending block when bit k of it is 0; the lower of the pair
        // keeps the smaller key in an ascending block
        const bool asc = ((4 * tid) & k) == 0, lower = (tid & msk) == 0;
        const bool keep_min = asc == lower;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint64_t px = xlane64(kx[q], msk), py = xlane64(ky[q], msk);
          kx[q] = keep_min ? (kx[q] < px ? kx[q] : px) : (kx[q] < px ? px : kx[q]);
          ky[q] = keep_min ? (ky[q] < py ? ky[q] : py) : (ky[q] < py ? py : ky[q]);
        }
      } else if (jj == 2) {  // pairs (0, 2), (1, 3)
        const bool asc = ((4 * tid) & k) == 0;  // k >= 4
        cx(kx[0], kx[2], asc);
        cx(kx[1], kx[3], asc);
        cx(ky[0], ky[2], asc);
        cx(ky[1], ky[3], asc);
      } else {  // pairs (0, 1), (2, 3)
        const bool a0 = ((4 * tid) & k) == 0, a1 = ((4 * tid + 2) & k) == 0;
        cx(kx[0], kx[1], a0);
        cx(kx[2], kx[3], a1);
        cx(ky[0], ky[1], a0);
        cx(ky[2], ky[3], a1);
      }
    }
  }
  {  // the sorted keys, for the searches
    u64x2_t* wx = reinterpret_cast<u64x2_t*>(lx + 4 * tid);
    u64x2_t* wy = reinterpret_cast<u64x2_t*>(ly + 4 * tid);
    wx[0] = u64x2_t{kx[0], kx[1]};
    wx[1] = u64x2_t{kx[2], kx[3]};
    wy[0] = u64x2_t{ky[0], ky[1]};
    wy[1] = u64x2_t{ky[2], ky[3]};
  }
  // this thread's queries (loaded after the sort: fewer registers live across it): i_e = qb * RANK_L + 256 e + tid (a wave's lanes: 64 neighbours)
  uint64_t c[4];
  int64_t m[4];
  int32_t ci[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = qb * RANK_L + 256 * e + tid;
    const bool qv = i < S;
    c[e] = qv ? c_in[i] : 0;
    m[e] = qv ? m_in[i] : 0;
    ci[e] = qv ? spec_class(c[e], m[e]) : SPEC_EXACT;
    if (sl == 0) {  // the class counts of the query block of 64 this wave holds
      const uint32_t na = (uint32_t)__popcll(__ballot(ci[e] == SPEC_A));
      const uint32_t nb = (uint32_t)__popcll(__ballot(ci[e] == SPEC_B));
      const int64_t q64 = qb * (RANK_L / 64) + 4 * e + wv;
      if (lane == 0 && q64 * 64 < S) {
        ra.bcnt[2 * q64] = na;
        ra.bcnt[2 * q64 + 1] = nb;
      }
    }
  }
  // normal candidates in the slice (the count for a query at v = 2^51 - 1, whose
  // threshold (v + 1) << 13 does not fit)
  uint32_t* const nrm_s = rank_small(lds) + 4;
  {
    const uint32_t wsum = (uint32_t)readlane_u64(wave_incl_scan_u64(nrm), 63);
    if (lane == 0) nrm_s[wv] = wsum;
  }
  __syncthreads();
  const uint32_t n_norm = nrm_s[0] + nrm_s[1] + nrm_s[2] + nrm_s[3];
  // Per normal query (ties by index), this slice's share of
  //   x(i) = #{normal j : (c_j, j) < (c_i, i)},   y(i) = #{normal j : (m_j, j) < (m_i, i)}:
  // an earlier slice counts v_j <= v_i (keys below (v_i + 1) << 13), a later one v_j < v_i
  // (below v_i << 13), i's own slice the keys below i's own: lower bounds by binary search.
  auto lower_bound = [](const uint64_t* a, uint64_t t) -> uint32_t {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t step = RANK_L / 2; step > 0; step >>= 1)
      pos += a[pos + step - 1] < t ? step : 0u;
    return pos + (a[pos] < t ? 1u : 0u);  // pos <= RANK_L - 1 here
  };
  uint32_t* const slices = ra.part + 2 * S;  // [ns][2][S]
  constexpr uint64_t V_TOP = (1ull << 51) - 1;  // largest normal request
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = qb * RANK_L + 256 * e + tid;
    if (i >= S) continue;
    uint32_t rx = 0, ry = 0;
    if (ci[e] != SPEC_EXACT) {
      const uint64_t own = (uint64_t)(i & 8191);
      if (sl < qb) {
        rx = c[e] == V_TOP ? n_norm : lower_bound(lx, (c[e] + 1) << 13);
        ry = (uint64_t)m[e] == V_TOP ? n_norm : lower_bound(ly, ((uint64_t)m[e] + 1) << 13);
      } else if (sl > qb) {
        rx = lower_bound(lx, c[e] << 13);
        ry = lower_bound(ly, (uint64_t)m[e] << 13);
      } else {
        rx = lower_bound(lx, c[e] << 13 | own);
        ry = lower_bound(ly, (uint64_t)m[e] << 13 | own);
      }
    }
    __hip_atomic_store(slices + (sl * 2 + 0) * S + i, rx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(slices + (sl * 2 + 1) * S + i, ry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave has waited for its stores
  uint32_t& last_s = rank_small(lds)[0];
  if (tid == 0)
    last_s = ns == 1 ? 1u
                     : (uint32_t)(__hip_atomic_fetch_add(ra.arrive + qb, 1u, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)ns - 1u);
  __syncthreads();
  if (!last_s) return;            // (workgroup-uniform)
  asm volatile("" ::: "memory");  // the slices' loads only after the arrival returned
  if (ns > 1 && tid == 0) ra.arrive[qb] = 0;  // every slice has arrived: reset for the next call
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = qb * RANK_L + 256 * e + tid;
    if (i >= S || ci[e] == SPEC_EXACT) continue;
    uint32_t x = 0, y = 0;
    for (int64_t k = 0; k < ns; ++k) {
      x += __hip_atomic_load(slices + (k * 2 + 0) * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      y += __hip_atomic_load(slices + (k * 2 + 1) * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ra.cs[x] = c[e];
    ra.ms[y] = m[e];
    ra.mr_c[x] = y;
    ra.cr_m[y] = x;
    ra.part[i] = x;
    ra.part[S + i] = y;
  }
}

__device__ void spec_rank_body(const RankArgs& ra, int64_t blk, uint64_t* lds) {
  const int tid = threadIdx.x;
  if (ra.zero_only) {
    // the clamp in the fit needs no ranks: this one workgroup zeroes the counters and
    // writes what spec_place and node_prep read of the ranks' output — the class counts
    // of every 64-spec block (bcnt) — from the classes of the S <= CLAMP_LDS_SPECS specs
    // (wave w: blocks w, w + 4, ...; one ballot per block)
    const bool wt = ra.done_flag != nullptr;  // node prep in this launch: write through
    if (tid < CNT_N && tid != CNT_SPECS_A && tid != CNT_SPECS_B) {
      if (wt) __hip_atomic_store(ra.counters + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else ra.counters[tid] = 0;
    }
    const int lane = tid & 63;
    const int64_t nqb = (ra.S + 63) / 64;
    int32_t cls[CLAMP_LDS_SPECS / 256];
#pragma unroll
    for (int u = 0; u < (int)(CLAMP_LDS_SPECS / 256); ++u) {  // every load first
      const int64_t j = ((int64_t)(tid >> 6) + 4 * u) * 64 + lane;
      cls[u] = j < ra.S ? spec_class(ra.c_in[j], ra.m_in[j]) : SPEC_EXACT;
    }
#pragma unroll
    for (int u = 0; u < (int)(CLAMP_LDS_SPECS / 256); ++u) {
      const int64_t qb = (tid >> 6) + 4 * u;
      const uint32_t na = (uint32_t)__popcll(__ballot(cls[u] == SPEC_A));
      const uint32_t nb = (uint32_t)__popcll(__ballot(cls[u] == SPEC_B));
      if (qb < nqb && lane == 0) {
        if (wt) {
          __hip_atomic_store(ra.bcnt + 2 * qb, na, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(ra.bcnt + 2 * qb + 1, nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          ra.bcnt[2 * qb] = na;
          ra.bcnt[2 * qb + 1] = nb;
        }
      }
    }
    if (wt) {  // every wave's stores performed, then the flag
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(ra.done_flag + NP_DONE,
                           __hip_atomic_load(ra.done_flag + NP_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  {  // zero duties, spread over the workgroups
    const int64_t gt = blk * 256 + tid, nt = (int64_t)ra.n_blocks * 256;
    if (gt < CNT_N && gt != CNT_SPECS_A && gt != CNT_SPECS_B) ra.counters[gt] = 0;
    for (int64_t e = gt; e < C_COPIES * ra.c_cells; e += nt)
      ra.C[(e / ra.c_cells) * ra.c_stride + e % ra.c_cells] = 0;
  }
  if (ra.S <= RANK_FULL_MAX) spec_rank_count(ra, blk, lds);
  else spec_rank_sort(ra, blk, lds);
}

__global__ __launch_bounds__(256) void spec_rank_kernel(RankArgs ra) {
  __shared__ __attribute__((aligned(16))) uint64_t lds[RANK_LDS_WORDS];
  spec_rank_body(ra, blockIdx.x, lds);
}


// spec_place: one thread per spec (caller index i = blk * blockDim + thread; a wave = a
// query block of 64).  Partition position = class base + the class counts of the
// earlier query blocks (bcnt) + the wave's ballot prefix.  Writes the SpecRec (with its
// rounded-up reciprocals) and perm there, zeroes partial[i] and partial[S + i], and for
// normal specs dperm[x] = position; the threads [nN, 64 T) pad mr_c and cr_m; thread 0 sets
// the class counters.
__device__ void spec_place_body(const PlaceArgs& pa, int64_t blk) {
  const int64_t S = pa.S;
  const uint64_t* __restrict__ c_in = pa.c_in;
  const int64_t* __restrict__ m_in = pa.m_in;
  const SpecPrep& sp = pa.sp;
  const ClampWork& cw = pa.cw;
  int64_t* __restrict__ partial = pa.partial;
  unsigned long long* __restrict__ counters = pa.counters;
  const int64_t i = blk * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t nqb = (S + 63) / 64, qb = i >> 6;
  const bool in = i < S;
  const uint64_t c = in ? c_in[i] : 0;
  const int64_t m = in ? m_in[i] : 0;
  const int32_t cls = in ? spec_class(c, m) : SPEC_EXACT;
  const bool normal = cls != SPEC_EXACT;
  // the x-rank (spec_rank's last arrivers; none with no_ranks)
  const uint32_t x = in && normal && !pa.no_ranks ? cw.rank[i] : 0u;
  // class totals and this block's prefix: the wave's lanes take every 64th block (the
  // counts packed A | B << 32), then one DPP scan each
  uint64_t tot = 0, pre = 0;
  // (agent-scope loads: with node prep in the reduce launch, the rank workgroup wrote them
  // through in the same launch, possibly on another XCD)
  const unsigned long long* bc = reinterpret_cast<const unsigned long long*>(cw.bcnt);
  for (int64_t b = lane; b < nqb; b += 64) {
    const uint64_t v = __hip_atomic_load(bc + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tot += v;
    pre += b < qb ? v : 0ull;
  }
  tot = readlane_u64(wave_incl_scan_u64(tot), 63);
  pre = readlane_u64(wave_incl_scan_u64(pre), 63);
  const uint32_t nA = (uint32_t)tot, nB = (uint32_t)(tot >> 32);
  const uint32_t pA = (uint32_t)pre, pB = (uint32_t)(pre >> 32);
  const int64_t nN = (int64_t)nA + nB;
  const unsigned long long mA = __ballot(cls == SPEC_A && in), mB = __ballot(cls == SPEC_B && in);
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t rA = (uint32_t)__popcll(mA & below), rB = (uint32_t)__popcll(mB & below);
  if (!pa.no_ranks && i >= nN && i < (nN + 63) / 64 * 64) {  // padding of the last x-group / y-block
    cw.mr_c[i] = 0xffffffffu;
    cw.cr_m[i] = 0xffffffffu;
  }
  if (i == 0) {
    counters[CNT_SPECS_A] = nA;
    counters[CNT_SPECS_B] = nB;
  }
  if (!in) return;
  const int64_t pos = cls == SPEC_A ? (int64_t)pA + rA
                    : cls == SPEC_B ? (int64_t)nA + pB + rB
                                    : nN + (qb * 64 - pA - pB) + (lane - rA - rB);
  SpecRec rec;
  rec.c = c;
  rec.m = m;
  rec.rc = normal ? recip_up_f64(c) : 0.0;
  rec.rm = normal ? recip_up_f64((uint64_t)m) : 0.0;
  rec.rcf = cls == SPEC_A ? recip_up_f32(c) : 0.0f;
  rec.cls = cls;
  rec.pad = 0;
  sp.rec[pos] = rec;
  sp.perm[pos] = (int32_t)i;
  partial[i] = 0;
  // (the give-ups of this step's reduce are in the words when spec_place runs after it;
  // on the fused path its workgroups run inside the reduce launch, and a give-up that comes
  // later in that launch is marked by the fit's by == 0 workgroup, which adds the mark too:
  // a faulted call's count is >= SPEC_FAULT_MARK, not an exact multiple of it)
  partial[S + i] = device_faulted(pa.faults) ? (int64_t)SPEC_FAULT_MARK : 0;
  if (!normal || pa.no_ranks) return;
  cw.dperm[x] = (int32_t)pos;
}


// ---- clamp correction: D_s and partial[s] -= D_s (one launch) ----------------------
// clamp_apply_kernel: 2T workgroups of 1024 threads, after the fit.
//   workgroup g < T (x-group g, the specs x = 64 g + l): H2[g] summed over its copies into
//     LDS and the copies zeroed, its 2-D suffix sums S2[k][r] = Σ_{k' >= k, r' >= r} H2; the
//     coarse part Σ_{G > g, GY > gy} C from the column sums of C's rows below g (LDS
//     atomics) and one suffix scan (when (T+2)^2 <= C_FULL_CELLS; otherwise
//     clamp_crows_kernel wrote C's row suffix sums to Crow and each lane sums its column);
//     then for each spec (wave 0, lane l; y = mr_c[x], kpos = #{specs of the group with a
//     smaller y}):  D_x = Csuf(g, y >> 6) + S2[kpos + 1][l + 1]  (r = 64 does not exist: 0);
//   workgroup T + Y (y-block Y, the specs y = 64 Y + l): H3[Y] likewise -> S3; for each spec
//     (x = cr_m[y], jpos = #{specs of the block with a smaller x}):  D_y = S3[jpos + 1][l + 1].
// partial[dperm[x]] -= D_x and -= D_y (atomics: two workgroups touch one spec) for the
// normal specs of clamp-free waves.  C's copies are read by every x-group and stay dirty:
// the next call's spec_place zeroes them.  The scans are DPP (VALU), not lane shuffles.
constexpr int CP_THREADS = 1024;
constexpr int CP_WAVES = CP_THREADS / 64;
constexpr int64_t C_FULL_CELLS = 4624;  // (T+2)^2 for T <= 66 (S <= 4224)
constexpr int H_CELLS = 65 * 64;
__host__ __device__ inline bool clamp_c_full(int64_t T) { return (T + 2) * (T + 2) <= C_FULL_CELLS; }

// The bin's records of every pass summed into tab (64-bit LDS atomics), in windows of
// CP_PW passes: each thread loads CP_PW / CP_THREADS passes' (start, count) of the bin,
// a workgroup scan of the counts gives the window's records a flat numbering, and each
// wave's lanes take consecutive records (coalesced loads; a lane per pass re-fetched a
// whole line per 8-B record: 48 us at C4), CP_RB loads in flight per lane.
constexpr int CP_PW = 4096;
constexpr int64_t CP_SPLIT = 4;  // workgroups per bin at most (binned clamp tables)
constexpr int CP_RB = 8;  // records per thread in flight
__device__ __forceinline__ void clamp_consume_bin(const ClampWork& cw, int64_t bin, uint64_t* tab,
                                                  uint32_t* w_lo, uint32_t* w_off, uint64_t* scratch,
                                                  uint32_t h, uint32_t G) {
  constexpr int PPT = CP_PW / CP_THREADS;  // passes per thread and window
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t* wsum = reinterpret_cast<uint32_t*>(scratch);  // CP_WAVES wave totals
  for (int64_t p0 = 0; p0 < cw.n_pass; p0 += CP_PW) {
    const int np = (int)(cw.n_pass - p0 < CP_PW ? cw.n_pass - p0 : CP_PW);
    uint32_t lo[PPT], cnt[PPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int p = tid * PPT + u;
      lo[u] = 0;
      cnt[u] = 0;
      if (p < np) {
        const uint32_t* d = cw.dir + (p0 + p) * cw.d_stride + bin;
        lo[u] = d[0];
        cnt[u] = d[1];
      }
    }
    uint32_t ts = 0;
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      cnt[u] -= lo[u];
      ts += cnt[u];
    }
    uint32_t inc = ts;  // inclusive scan over the workgroup: waves, then the wave totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(inc, d, 64);
      if (lane >= d) inc += t;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w2 = 0; w2 < CP_WAVES; ++w2) {
      const uint32_t t = wsum[w2];
      before += w2 < wv ? t : 0u;
      total += t;
    }
    uint32_t run = before + inc - ts;
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int p = tid * PPT + u;
      w_lo[p] = lo[u];
      w_off[p] = run;
      run += cnt[u];
    }
    if (tid == 0) w_off[CP_PW] = total;  // sentinel (passes past np hold count 0)
    __syncthreads();
    // the window's records in flat order, a contiguous share per wave (whole 64-record
    // rows): lane l takes records J0 + 64 k + l, so a wave's loads cover consecutive
    // records (one pass's run of the bin: whole lines).  A lane's pass only moves
    // forward: one step (or a binary search over w_off when it jumps further) per record
    // instead of a search per record (12 dependent LDS reads each: 16 us at C4).
    int top = 1;  // highest power of two <= np (w_off[np ..] = total)
    while (2 * top <= np) top *= 2;
    auto search = [&](uint32_t j) {  // the last pass with w_off[p] <= j (count > 0)
      int p = 0;
      for (int st = top; st >= 1; st >>= 1)
        if (w_off[p + st] <= j) p += st;
      return p;
    };
    // share h of G of the window's records (the bin split over G workgroups)
    const uint32_t s0 = (uint32_t)((uint64_t)total * h / G), s1 = (uint32_t)((uint64_t)total * (h + 1) / G);
    const uint32_t per_w = (s1 - s0 + CP_WAVES * 64 - 1) / (CP_WAVES * 64) * 64;
    const uint32_t J0 = s0 + (uint32_t)wv * per_w;
    const uint32_t J1 = J0 + per_w < s1 ? J0 + per_w : s1;
    // a lane's pass p, where its records leave it (nxt = w_off[p + 1]) and its start in
    // the pass's slots minus its first flat index (gb), in registers
    int p = J0 + lane < J1 ? search(J0 + lane) : 0;
    uint32_t nxt = w_off[p + 1], gb = w_lo[p] - w_off[p];
    const uint64_t* rec0 = cw.rec + p0 * cw.pass_recs;
    auto load_batch = [&](uint64_t (&rv)[CP_RB], uint32_t jb) {
#pragma unroll
      for (int u = 0; u < CP_RB; ++u) {
        const uint32_t j = jb + (uint32_t)(64 * u + lane);
        rv[u] = 0;
        if (j < J1) {
          if (j >= nxt) {  // the next pass of the bin (or a search when it is further)
            p = w_off[p + 2] <= j ? search(j) : p + 1;
            nxt = w_off[p + 1];
            gb = w_lo[p] - w_off[p];
          }
          rv[u] = rec0[(int64_t)p * cw.pass_recs + (uint32_t)(j + gb)];
        }
      }
    };
    auto add_batch = [&](const uint64_t (&rv)[CP_RB], uint32_t jb) {
#pragma unroll
      for (int u = 0; u < CP_RB; ++u)
        if (jb + (uint32_t)(64 * u + lane) < J1)
          atomicAdd(reinterpret_cast<unsigned long long*>(&tab[(uint32_t)rv[u]]),
                    (unsigned long long)(int64_t)(int32_t)(rv[u] >> 32));
    };
    const uint32_t step = 64u * CP_RB;
    uint64_t ra[CP_RB], rb[CP_RB];
    load_batch(ra, J0);
    for (uint32_t jb = J0; jb < J1; jb += 2 * step) {
      load_batch(rb, jb + step);
      add_batch(ra, jb);
      load_batch(ra, jb + 2 * step);
      add_batch(rb, jb + step);
    }
    __syncthreads();  // tab complete / the window's arrays free
  }
}

// One bin's part of the clamp correction (clamp_apply_kernel): every thread of the
// workgroup enters and leaves together (the fused finalize's barrier follows).
__device__ __forceinline__ void clamp_apply_bin(const ClampWork& cw, int64_t S,
                                                int64_t* __restrict__ partial, int64_t nN,
                                                int64_t u, uint32_t G, uint32_t h) {
  __shared__ uint64_t tab[H_CELLS];
  __shared__ uint64_t ctot[CP_WAVES][64];
  __shared__ uint64_t colsum[128];
  __shared__ uint32_t pos_s[64];          // the specs' kpos / jpos (wave 15 -> every wave)
  __shared__ uint32_t cp_lo[CP_PW];       // binned: a window's passes' bin starts
  __shared__ uint32_t cp_off[CP_PW + 1];  // and the exclusive prefix of their counts
  const int64_t T = (nN + 63) / 64, W = T + 2;
  KCC_TL(1024 + blockIdx.x % 1024, 0);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool x_side = u < T;
  const int64_t g = x_side ? u : u - T;
  const bool full = clamp_c_full(T);
  // this workgroup's 64 specs (wave 0), loaded up front
  const int64_t q = 64 * g + lane;  // x (x side) or y (y side)
  uint32_t other = 0xffffffffu;  // wave 0 (the specs' lookups) and wave 15 (their positions)
  if (wv == 0 || wv == CP_WAVES - 1) other = (x_side ? cw.mr_c : cw.cr_m)[q];  // y of x, or x of y (padding: ~0)
  if (tid < 128) colsum[tid] = 0;
  // the table: binned records (below), or every copy's cells first, then LDS and zeroes
  const bool binned = clamp_binned(S);
  int64_t* H = (x_side ? cw.H2 : cw.H3) + g * H_CELLS;
  constexpr int PER = (H_CELLS + CP_THREADS - 1) / CP_THREADS;
  uint64_t v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + CP_THREADS * k;
    v[k] = 0;
    if (!binned) {
#pragma unroll
      for (int c = 0; c < H2_COPIES; ++c) v[k] += e < H_CELLS ? (uint64_t)H[c * cw.h_stride + e] : 0ull;
    }
  }
  // the coarse table's rows G > g (x side, C in the full form): loads first as well
  constexpr int CPER = (int)((C_FULL_CELLS + CP_THREADS - 1) / CP_THREADS);
  uint64_t cv[CPER];
  const int64_t c0 = (g + 1) * W, c1 = W * W;  // cells of rows g+1 .. T+1
  const bool do_c = x_side && full && h == 0;  // the coarse parts: part 0 of the bin
#pragma unroll
  for (int k = 0; k < CPER; ++k) {
    const int64_t e = c0 + tid + CP_THREADS * k;
    cv[k] = 0;
    if (do_c && e < c1) {
#pragma unroll
      for (int c = 0; c < C_COPIES; ++c) cv[k] += (uint64_t)cw.C[c * cw.c_stride + e];
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + CP_THREADS * k;
    if (e < H_CELLS) {
      tab[e] = v[k];
      if (!binned) {
#pragma unroll
        for (int c = 0; c < H2_COPIES; ++c) H[c * cw.h_stride + e] = 0;  // zero between calls
      }
    }
  }
  __syncthreads();  // tab and colsum's zeroes
  KCC_TL(1024 + blockIdx.x % 1024, 1);
  if (binned) clamp_consume_bin(cw, x_side ? g : T + g, tab, cp_lo, cp_off, &ctot[0][0], h, G);
  KCC_TL(1024 + blockIdx.x % 1024, 2);
  if (do_c) {
#pragma unroll
    for (int k = 0; k < CPER; ++k) {
      const int64_t e = c0 + tid + CP_THREADS * k;
      if (e < c1 && cv[k]) atomicAdd(reinterpret_cast<unsigned long long*>(&colsum[e % W]), cv[k]);
    }
  }
  // wave 0: the specs' internal positions, in flight during the suffix work below
  int32_t p = 0x7fffffff;
  if (wv == 0 && q < nN) p = cw.dperm[x_side ? q : (int64_t)other];
  // rows of tab: suffix along r (lanes reversed, DPP inclusive scan); wave 15 (fewest
  // rows) also ranks the specs: pos = #{members with a smaller y (x side) / x (y side)}
  for (int k = wv; k < 65; k += CP_WAVES) {
    const uint64_t sr = wave_incl_scan_u64(tab[k * 64 + 63 - lane]);
    tab[k * 64 + 63 - lane] = sr;
  }
  if (wv == CP_WAVES - 1) {
    uint32_t pos = 0;
    for (int l = 0; l < 64; ++l) pos += (uint32_t)__builtin_amdgcn_readlane((int)other, l) < other ? 1u : 0u;
    pos_s[lane] = pos;
  }
  __syncthreads();
  // spec l needs S2[pos_l + 1][l + 1] = Σ_{k > pos_l} rowsuf[k][l + 1] (column 64: none):
  // each wave sums its chunk of rows under that mask, wave 0 adds the chunks
  constexpr int KCH = (65 + CP_WAVES - 1) / CP_WAVES;
  const int k0 = wv * KCH, k1 = k0 + KCH < 65 ? k0 + KCH : 65;
  {
    const uint32_t posl = pos_s[lane];
    uint64_t part = 0;
    for (int k = k0; k < k1; ++k)
      part += (lane < 63 && (uint32_t)k > posl) ? tab[k * 64 + lane + 1] : 0ull;
    ctot[wv][lane] = part;
  }
  __syncthreads();
  if (wv != 0) return;  // (no barrier below)
  KCC_TL(1024 + blockIdx.x % 1024, 3);
  // wave 0: the 64 specs
  uint64_t csuf = 0;  // x side: Σ_{GY > gy} colsum[GY] per lane
  if (do_c) {  // suffix of colsum over GY in place (W <= 68: two chunks from the top)
    uint64_t carry = 0;
    for (int ch = 1; ch >= 0; --ch) {
      const int col = ch * 64 + 63 - lane;  // lanes reversed: an inclusive scan is the suffix
      uint64_t sv = col < W ? colsum[col] : 0ull;
      sv = wave_incl_scan_u64(sv) + carry;
      carry = readlane_u64(sv, 63);
      if (col < W) colsum[col] = sv;
    }
    const uint32_t gy1 = other == 0xffffffffu ? 0xffffffffu : (other >> 6) + 1;
    csuf = gy1 < W ? colsum[gy1] : 0ull;
  }
  if (q >= nN) return;
  uint64_t d = csuf;
#pragma unroll
  for (int w2 = 0; w2 < CP_WAVES; ++w2) d += ctot[w2][lane];
  if (x_side && !full && h == 0) {
    const int64_t gy = other >> 6;
    uint64_t part[8] = {};
    for (int64_t G = g + 1; G <= T + 1; G += 8) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        part[r] += G + r <= T + 1 ? (uint64_t)cw.Crow[(G + r) * W + gy + 1] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) d += part[r];
  }
  if (d && p < clamp_n_pure(nN, S)) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[p]), 0ull - d);
  KCC_TL(1024 + blockIdx.x % 1024, 4);
}

// The fused finalize (clamp_apply_kernel): every
// wave's atomics into partial are performed (vmcnt counts the stores and atomics too on
// gfx9) before the workgroup arrives; the last workgroup to arrive reads partial at agent
// scope and writes the totals in caller order.  Every thread of the workgroup calls, from
// one call site.
//
// The hand-off needs no cache maintenance: the payload (partial) is written only by 8-B
// agent-scope atomics and read only by 8-B agent-scope loads, every wave waits for its
// atomics (vmcnt(0)) before the workgroup barrier, and one lane then makes a RELAXED
// agent-scope add to the arrival counter — MI355X_MICROARCH.md's "{8-B agent atomics both
// sides}" form with the "workgroup whose add came last" signal (an acq_rel add lowers to a
// buffer_wbl2 + buffer_inv pair per workgroup: an L2 write-back each).
//
// The arrivals go to `ctr` (`expect` of them; the last arriver resets it), and the last
// arriver finalizes specs [s0, s1) of the S.
__device__ void fused_finalize(const FinArgs& fin, int64_t S, const int64_t* partial,
                               uint32_t* ctr, uint32_t expect, int64_t s0, int64_t s1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ uint32_t last_s;
  if (threadIdx.x == 0) {
    last_s = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             expect - 1u;
    if (last_s) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last_s) return;
  const bool faulted = device_faulted(fin.faults);
  // FIN_PER specs per thread per round, every load of the round issued before any store
  // (one memory round trip per round: S <= 4 x the workgroup is one round)
  constexpr int FIN_PER = 4;
  const int64_t nt = blockDim.x;
  for (int64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += (int64_t)FIN_PER * nt) {
    int64_t t[FIN_PER], e[FIN_PER];
    int32_t dst[FIN_PER];
#pragma unroll
    for (int k = 0; k < FIN_PER; ++k) {
      // past the end: reload spec s1-1 (branch-free, so no wait splits the batch)
      const int64_t i = min(i0 + (int64_t)k * nt, s1 - 1);
      t[k] = __hip_atomic_load(partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e[k] = __hip_atomic_load(partial + S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dst[k] = fin.perm[i];
    }
#pragma unroll
    for (int k = 0; k < FIN_PER; ++k) {
      if (i0 + (int64_t)k * nt >= s1) break;
      const bool fk = faulted || (uint64_t)e[k] >= SPEC_FAULT_MARK;
      fin.totals[dst[k]] = e[k] != 0 || fk ? 0 : t[k];
      fin.spec_err[dst[k]] = fk ? SPEC_ERR_FAULT : e[k] != 0 ? SPEC_ERR_DIV0 : 0;
    }
  }
}

__global__ __launch_bounds__(CP_THREADS) void clamp_apply_kernel(ClampWork cw,
                                                                 const unsigned long long* __restrict__ counters,
                                                                 int64_t S, int64_t* __restrict__ partial,
                                                                 FinArgs fin) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t T = (nN + 63) / 64;
  // blockIdx = h * 2 Tm + u: part h of the G parts of bin u (launch_clamp_apply)
  const int64_t Tm = (S + 63) / 64;
  const uint32_t G = gridDim.x / (uint32_t)(2 * Tm), h = blockIdx.x / (uint32_t)(2 * Tm);
  const int64_t u = blockIdx.x % (uint32_t)(2 * Tm);
  if (u < 2 * T) clamp_apply_bin(cw, S, partial, nN, u, G, h);  // (else: no bin)
  if (fin.totals) fused_finalize(fin, S, partial, fin.arrive, gridDim.x, 0, S);
}

// clamp_crows_kernel (only when C does not fit clamp_apply's full form): one wave per row
// G of C: the copies summed and Crow[G][GY] = Σ_{GY' >= GY} C[G][GY'].
__global__ __launch_bounds__(256) void clamp_crows_kernel(ClampWork cw,
                                                          const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t T = (nN + 63) / 64, W = T + 2;
  const int64_t G = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (nN == 0 || clamp_c_full(T) || G >= W) return;
  uint64_t carry = 0;
  for (int64_t ch = (W + 63) / 64 - 1; ch >= 0; --ch) {
    const int64_t gy = ch * 64 + 63 - lane;  // lanes reversed: an inclusive scan is the suffix
    uint64_t v = 0;
#pragma unroll
    for (int c = 0; c < C_COPIES; ++c) v += gy < W ? (uint64_t)cw.C[c * cw.c_stride + G * W + gy] : 0ull;
    v = wave_incl_scan_u64(v) + carry;
    carry = readlane_u64(v, 63);
    if (gy < W) cw.Crow[G * W + gy] = (int64_t)v;
  }
}

// Lane = spec (its request, reciprocals and running total live in VGPRs); the node
// stream is wave-uniform: the fields of a FitGroup arrive by scalar loads and feed the
// VALU as SGPR operands.  The main loops are branch-free: rows outside the fast bounds
// carry zero fields and are re-done exactly from slow_list.  No cross-lane reduction
// until the block's end (one 64-bit atomic per spec).  Everything is exact (DESIGN.md
// §5, "Fit fast path: exactness").
//
// The fast loops (normal specs: 1 <= c, m < 2^51) sum  min(findMin(qc, qm), P)  per
// node, which equals the reference's contribution `x >= P ? P - podCount : x`
// (CC:133-136) except where the clamp applies — there it is larger by w = podCount;
// the clamp correction (ClampWork, clamp_*_kernel) subtracts  Σ w  over those nodes
// from each spec's total.  The per-pair work is the two quotients and one min:
//
// Class A (m >= 2^18; fc < 2^23, fm < 2^50), round-toward--inf, integers read as denormals:
//   qc = bits(RD32(fc*2^-149 * rcf)) = floor(fc * rcf) = floor(fc / c)   (rcf = RU32(1/c))
//     — one v_pk_mul_f32 for two nodes (an SGPR pair of free CPUs);
//   qm = low32(bits(RD64(fm*2^-1074 * rm))) = floor(fm / m)             (rm = RU64(1/m))
//     — one v_mul_f64 (qm < 2^50 / 2^18 = 2^32, so the low dword is all of it);
//   min3(qc, qm, P) — one v_min3_u32; two nodes per v_add3_u32.
// The products are exact reals rounded once onto the 2^-149 / 2^-1074 grid, so the
// rounding down IS floor; a quotient that is an integer is never undershot (the
// reciprocal is rounded up), a non-integer one lies >= 1/c below the next integer,
// more than the relative error (< 2^-23 resp. 2^-52) covers while fc < 2^23, fm < 2^52.
// Per node and 64-spec wavefront: 3 VALU instructions.
//
// Class B (memory requests below 2^18, where fm/m may exceed 32 bits): f64 values,
// round-toward--inf, one fused multiply-add per quotient doing floor AND the
// conversion: qc' = RD(fc * rc + 2^52) = 2^52 + floor(fc / c), likewise qm';
// min(qc', qm', 2^52 + P) and its low dword.  4.5 VALU instructions per node and wave.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// MODE register FP_ROUND[3:0]: [1:0] f32, [3:2] f64/f16; 0 nearest-even, 2 toward -inf.
// The fast loops run in round-toward--inf; the exact path (whose 64-bit integer
// division the compiler expands with f32 reciprocal steps) runs in the default mode.
// The switch is inline asm on purpose: LLVM's SIModeRegister pass would otherwise
// re-insert a switch back to the function's default mode in front of every FP
// instruction it emits.  Invisible to it, the compiler-generated v_mul/v_fma in the
// loops run in the mode set here (tests/test_isa.py pins the window and checks the
// compiler adds no switch of its own).
__device__ __forceinline__ void set_round_down() {
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 10\n\ts_nop 1" ::: "memory");
}
__device__ __forceinline__ void set_round_nearest() {
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 0\n\ts_nop 1" ::: "memory");
}
// min(x, p) with p a loaded (wave-uniform) double: asm, because the compiler would first
// quiet p with a v_max_f64 (it cannot see that 2^52 + P is no signalling NaN)
__device__ __forceinline__ double min_f64_s(double x, double p) {
  double d;
  asm("v_min_f64 %0, %1, %2" : "=v"(d) : "v"(x), "s"(p));
  return d;
}

constexpr int FIT_SPW = 256;           // specs per 256-thread workgroup (one column per wave)
constexpr int FIT_CHUNK_GROUPS = 128;  // 1024 nodes: |sum of contributions| <= 2^30 in i32
constexpr uint32_t FIT_QCHUNK = 32;  // node groups per claim from a sub-queue
static_assert(FIT_QCHUNK >= 2 && FIT_QCHUNK <= FIT_CHUNK_GROUPS, "claims sum in i32");
constexpr uint32_t FIT_QDIV = 2;   // guided claims: (what remains of the segment) / (QDIV x its workgroups)
constexpr uint32_t FIT_QMIN = 2;   // node groups per claim at least (guided claims)
// the static first claim at most share / this: the 8-way C4 rank 0.0624 -> 0.0618 ms (r04z),
// C4 unchanged (its share / 8 > qsz)
constexpr uint32_t FIT_Q1_DIV = 8;
constexpr uint32_t FIT_Q_HALVE = 128;  // claims of FIT_QCHUNK / 2 when a workgroup's share is below this
constexpr uint32_t FIT_WG_PER_SUB = 24;  // workgroups per sub-queue at most, about (8 to 32 sub-queues)
constexpr uint32_t FIT_QSUBS = (uint32_t)FIT_QSUBS_MAX;

__device__ __forceinline__ double f64_at(const i32x16& v, int k) {
  return __longlong_as_double(((int64_t)(uint32_t)v[2 * k + 1] << 32) | (uint32_t)v[2 * k]);
}

// Work distribution: a workgroup = 4 waves = 256 specs (a spec column), each wave 64
// specs; node groups come from a queue.  The grid holds gx * gy workgroups (one round of
// resident workgroups).  A column's stream is cut into nsub segments (the workgroups with
// by % nsub == sub, i.e. of one XCD, share segment sub), and the workgroups of a segment
// claim FIT_QCHUNK node groups at a time from its sub-queue: one returning 32-bit atomic
// by wave 0, in flight while the current chunk is summed, its result handed to the four
// waves through LDS at the chunk's barrier (the four waves read the same node groups:
// scalar-cache hits).  The workgroups that run faster take more chunks and none waits for
// a ragged last round; each wave sums its claims in registers and adds them to partial
// with one 64-bit atomic per spec at the end: S * gy atomics per launch (C4: gy ~ 450,
// 3.7 MB) instead of one per spec and static node share.  Sub-queues sit in 64-B lines of
// their own ([0] claims, [1] workgroups done: returning atomics on one line serialise);
// the last workgroup of a sub-queue to finish resets both to zero for the next launch
// (every workgroup of it has made its last claim by then); the buffer is zeroed once when
// allocated.
// 8 waves per SIMD: the register budget that leaves (the compiler otherwise takes ~106
// SGPRs, 6 waves); the loops stay spill-free (tests/test_isa.py).  Half or a quarter of
// the resident workgroups per column measured slower (round 3, prepare + run: C4 172 ->
// 220 / 372 us, its 8-way shard 57 -> 63 / 83 us, profiles/r03o_ab_fit_grid.jsonl)
#define KCC_FIT_ATTR __attribute__((amdgpu_waves_per_eu(8)))
// NC: the clamp in the fit (fast_cl, launch_fit) — its own instantiation, so the
// clamp-correction layout's registers are not the larger loops' (one kernel holding both
// spilled 52 SGPRs: C4 fit 116 -> 120 us)
// (the body of fit_kernel; b = the workgroup's index in the fit's grid, q_slot = 2 words of
// LDS)
template <bool NC>
__device__ __forceinline__ void fit_body(
    int64_t n_nodes, uint32_t* __restrict__ queue, const FitGroupA* __restrict__ fast_a,
    const FitGroup* __restrict__ fast_b, const SlowNode* __restrict__ slow,
    const int64_t* __restrict__ slow_list, int64_t S, const SpecRec* __restrict__ specs,
    int64_t* __restrict__ partial, unsigned long long* __restrict__ counters, int32_t chunk,
    int32_t gx, int32_t gy, const int32_t* __restrict__ fast_cl,
    const unsigned long long* __restrict__ faults, const int32_t b, uint32_t* q_slot) {
  // XCD-aware order (speed only, never correctness): workgroups are dealt round-robin
  // over the 8 XCDs, so give every spec group of one node chunk the same b % 8
  const int32_t xcd = b & 7, r = b >> 3;
  const int32_t bx = r % gx, by = (r / gx) * 8 + xcd;
  if (by >= gy) return;  // padding of gy up to a multiple of 8 (whole workgroup)
  // issue priority falls with the workgroup's progress through its share (below): the
  // arbiter otherwise serves the oldest waves first, and a late starter sat on its claims
  __builtin_amdgcn_s_setprio(3);
  KCC_TL(2048 + b % 4096, 0);
  const int32_t wv = __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)bx * FIT_SPW + threadIdx.x;
  const bool active = s < S;
  const bool idle = !__any(active);  // a wave wholly past S (still takes the barriers)
  SpecRec sr;  // one 48-B record per lane
  if (active) {
    sr = specs[s];
  } else {  // a class-A placeholder (its sums are never stored)
    sr.c = 1;
    sr.m = CLASS_A_M_MIN;
    sr.rc = 1.0;
    sr.rm = 1.0 / (double)CLASS_A_M_MIN;
    sr.rcf = 1.0f;
    sr.cls = SPEC_A;
  }
  const uint64_t c = sr.c;
  const int64_t m = sr.m;
  const double rm = sr.rm, rc = sr.rc;
  const bool wave_exact = __any(sr.cls == SPEC_EXACT);
  const bool wave_b = __any(sr.cls == SPEC_B);
  const bool wave_fast = !wave_exact && !idle;  // sums the node stream
  KCC_TL(2048 + b % 4096, 5);  // (the spec records are in)

  // the node stream node_prep wrote (its length is on the device; 32-bit: < 2^31 groups)
  const uint32_t n_groups = (uint32_t)(counters[CNT_STREAM + chunk] / FIT_GROUP);
  uint32_t lim = n_groups;  // claims end here
  uint32_t base = 0;        // queue: the segment's start
  uint32_t nxt = 0;         // queue: the claim in flight (wave 0, lane 0)
  // sub-queues: gy if gy < 8, else 8, 16 or 32 (a power of two: whole XCDs each), about
  // FIT_WG_PER_SUB workgroups per sub-queue (measured: 56 per line 8 % slower at C4 than
  // 28; fewer than 2 per line lose the balancing)
  uint32_t nsub = (uint32_t)gy / FIT_WG_PER_SUB;
  nsub = nsub <= 8u ? 8u : (nsub >= FIT_QSUBS ? FIT_QSUBS : 1u << (31 - __builtin_clz(nsub)));
  if ((uint32_t)gy < nsub) nsub = (uint32_t)gy;
  const uint32_t sub = (uint32_t)by % nsub;
  uint32_t* const qp = queue + ((uint32_t)bx * FIT_QSUBS + sub) * 16u;
  // claim size: halved when a workgroup's share is small (8-way shards of C4: ~35 groups
  // per workgroup; two claims each keep the balancing)
  const uint32_t qsz = n_groups / (uint32_t)gy < FIT_Q_HALVE ? FIT_QCHUNK / 2u : FIT_QCHUNK;
  // the static first claim: qsz, or at most a 1/FIT_Q1_DIV of a workgroup's share — the
  // workgroups begin their loops up to ~11 us apart on small shards, and a late one's
  // static claim was the fit's tail
  uint32_t q1 = qsz;
  {
    const uint32_t sh = n_groups / (uint32_t)gy / FIT_Q1_DIV;
    q1 = sh < q1 ? (sh > FIT_QMIN ? sh : FIT_QMIN) : q1;
  }

  // lane 0 of wave 0 issues the claim in asm, so the compiler does not wait for it where
  // it is issued (its atomic-optimizer expansion reads the result at once); wave 0 waits
  // for it (vmcnt) at the end of the chunk — the loop bodies issue no other vector memory
  // operations (tests/test_isa.py: nothing touches its register before that wait)
  auto claim_issue = [&](uint32_t sz) {
    if (wv == 0 && lane == 0)
      asm volatile("global_atomic_add %0, %1, %2, off sc0"
                   : "=v"(nxt) : "v"(qp), "v"(sz) : "memory");
  };
  // guided claims: a claim's size is (what remained of the segment at the workgroup's
  // current claim) / (2 x its workgroups), between FIT_QMIN and qsz, so the claims
  // shrink as the segment drains and the workgroups finish together (fixed claims of
  // qsz left a tail of one to two claims: 10-20 us at C4).  Every wave computes the
  // same sizes (workgroup-uniform); claims never overlap (fetch-and-add of each size).
  // The first claim is static — the segment's first wseg x qsz groups, qsz per workgroup
  // by its rank in the segment — so no workgroup waits on the queue line at launch (2048
  // returning atomics on 256 lines at once); the queue hands out what follows.
  const uint32_t wps = ((uint32_t)gy + nsub - 1u) / nsub;  // workgroups per segment (at most)
  const uint32_t wseg = ((uint32_t)gy - sub + nsub - 1u) / nsub;  // this segment's workgroups
  const uint32_t dyn0 = wseg * q1;                         // the queue's first group
  uint32_t qcur = q1;   // size of the claim whose result is read next
  auto claim_publish = [&](uint32_t slot) {
    if (wv == 0) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(nxt) : : "memory");
      if (lane == 0) q_slot[slot] = dyn0 + nxt;
    }
    __syncthreads();
  };
  {
    const uint32_t seg = ((n_groups + nsub - 1u) / nsub + 7u) / 8u * 8u;
    base = sub * seg < n_groups ? sub * seg : n_groups;
    lim = base + seg < n_groups ? base + seg : n_groups;
    KCC_TL(2048 + b % 4096, 1);
  }
  const uint32_t first = ((uint32_t)by / nsub) * q1;  // the static first claim's offset
  uint32_t pr_done = 0;  // groups summed (workgroup-uniform), against an equal share
  const uint32_t pr_share = (lim - base) / wseg > 0 ? (lim - base) / wseg : 1u;
#ifdef KCC_TIMELINE
  uint32_t tl_done = 0;  // groups this workgroup summed
#endif
  uint64_t acc = 0;
  uint64_t errs = 0;
  uint32_t slow_iters = 0;

  // exact Go semantics, 64-bit (CC:119-136)
  auto eval_slow = [&](int64_t i) {
    ++slow_iters;
    const SlowNode sn = slow[i];
    int64_t qc = 0, qm = 0;
    bool z = false;
    if (sn.fc != 0) {
      if (c == 0) z = true;
      else qc = (int64_t)(sn.fc / c);
    }
    if (sn.fm != 0) {
      if (m == 0) z = true;
      else if (m == -1) qm = (int64_t)(0ull - (uint64_t)sn.fm);
      else qm = sn.fm / m;
    }
    int64_t q = qc <= qm ? qc : qm;
    if (q >= sn.P) q = sn.cl;
    errs += z ? 1u : 0u;  // branch-free: a select between &acc and &errs spills to scratch
    acc += z ? 0ull : (uint64_t)q;
  };

  // class A: node groups [g0, g0 + cnt)
  auto sum_a = [&](uint32_t g0, int cnt) {
    cnt = __builtin_amdgcn_readfirstlane(cnt);  // keep the trip count scalar
    const FitGroupA* gbase = fast_a + g0;
    const f32x2 rcf2 = {sr.rcf, sr.rcf};
    int32_t acc32 = 0;
    set_round_down();
    for (int gi = 0; gi < cnt; ++gi) {
      // index opaque to loop-strength reduction: one base per group, immediate offsets
      int io = gi;
      asm volatile("" : "+s"(io));
      const FitGroupA* g = gbase + io;
      const i32x16 fmv = *reinterpret_cast<const i32x16*>(g->fm);
      const i32x8 fcv = *reinterpret_cast<const i32x8*>(g->fc);
      const i32x8 Pv = *reinterpret_cast<const i32x8*>(g->P);
#pragma unroll
      for (int u = 0; u < FIT_GROUP / 2; ++u) {
        const f32x2 fcp = {__int_as_float(fcv[2 * u]), __int_as_float(fcv[2 * u + 1])};
        const f32x2 q = fcp * rcf2;  // two nodes' floor(fc / c), as integers
        uint32_t m3[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * u + h;
          const uint32_t qm = (uint32_t)__double_as_longlong(f64_at(fmv, k) * rm);
          const uint32_t qc = __float_as_uint(h ? q.y : q.x);
          m3[h] = min(min(qc, qm), (uint32_t)Pv[k]);  // min(findMin(qc, qm), P)
        }
        acc32 += (int32_t)(m3[0] + m3[1]);
      }
      asm volatile("; fit: full" : "+v"(acc32));  // (the ISA tests' marker)
    }
    set_round_nearest();
    acc += (uint64_t)(int64_t)acc32;
  };
  // the clamp in the fit (fast_cl: launch_node_prep's NC mode): x >= P ? clamp : x per
  // node (CC:133-136), the clamp value from fast_cl, P >= 1 on every streamed row (padding:
  // x = 0 >= P = 0, clamp 0).  Class A: 5.0 VALU per node, the clamp values by vector loads
  // (uniform addresses: one line per wave), so the select takes them as VGPRs.  By scalar
  // loads each needs a move first (a select reads one scalar operand at most, vcc
  // included): 6.0, 2 % slower per rank (round 3, profiles/r03z_ab_clamp_vload.txt); one
  // inline-asm v_mov_b64 per two nodes (5.5): C4 8-way fit 33.3 -> 36.2 us.  Class B: 6.5.
  const __amdgpu_buffer_rsrc_t cl_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)fast_cl, (short)0, (int)(fit_groups(n_nodes) * FIT_GROUP * 4), 0x00020000);
  auto sum_a_nc = [&](uint32_t g0, int cnt) {
    cnt = __builtin_amdgcn_readfirstlane(cnt);
    const FitGroupA* gbase = fast_a + g0;
    const f32x2 rcf2 = {sr.rcf, sr.rcf};
    int32_t acc32 = 0;
    typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));
    set_round_down();
    for (int gi = 0; gi < cnt; ++gi) {
      int io = gi;
      asm volatile("" : "+s"(io));
      const FitGroupA* g = gbase + io;
      const i32x16 fmv = *reinterpret_cast<const i32x16*>(g->fm);
      const i32x8 fcv = *reinterpret_cast<const i32x8*>(g->fc);
      const i32x8 Pv = *reinterpret_cast<const i32x8*>(g->P);
      const int so = (int)((g0 + (uint32_t)io) * FIT_GROUP * 4);
      const i32x4_t c0 = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(cl_rs, 0, so, 0));
      const i32x4_t c1 = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(cl_rs, 16, so, 0));
      const int32_t clv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int u = 0; u < FIT_GROUP / 2; ++u) {
        const f32x2 fcp = {__int_as_float(fcv[2 * u]), __int_as_float(fcv[2 * u + 1])};
        const f32x2 q = fcp * rcf2;
        int32_t m3[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * u + h;
          const uint32_t qm = (uint32_t)__double_as_longlong(f64_at(fmv, k) * rm);
          const uint32_t qc = __float_as_uint(h ? q.y : q.x);
          const uint32_t x = min(qc, qm);                            // findMin(qc, qm)
          m3[h] = x >= (uint32_t)Pv[k] ? clv[k] : (int32_t)x;        // CC:134-135
        }
        acc32 += m3[0] + m3[1];
      }
      asm volatile("; fit: full" : "+v"(acc32));  // (the ISA tests' marker)
    }
    set_round_nearest();
    acc += (uint64_t)(int64_t)acc32;
  };
  auto sum_b_nc = [&](uint32_t g0, int cnt) {
    cnt = __builtin_amdgcn_readfirstlane(cnt);
    const FitGroup* gbase = fast_b + g0;
    const int32_t* cbase = fast_cl + (size_t)g0 * FIT_GROUP;
    const double bias = FIT_BIAS;
    int32_t acc32 = 0;
    set_round_down();
    for (int gi = 0; gi < cnt; ++gi) {
      int io = gi;
      asm volatile("" : "+s"(io));
      const FitGroup* g = gbase + io;
      const i32x16 fcv = *reinterpret_cast<const i32x16*>(g->fc);
      const i32x16 fmv = *reinterpret_cast<const i32x16*>(g->fm);
      const i32x16 Pv = *reinterpret_cast<const i32x16*>(g->Pb);
      const i32x8 clv = *reinterpret_cast<const i32x8*>(cbase + (size_t)io * FIT_GROUP);
#pragma unroll
      for (int u = 0; u < FIT_GROUP / 2; ++u) {
        int32_t x[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * u + h;
          const double qc = __builtin_fma(f64_at(fcv, k), rc, bias);  // 2^52 + floor(fc/c)
          const double qm = __builtin_fma(f64_at(fmv, k), rm, bias);  // 2^52 + floor(fm/m)
          const double xb = __builtin_fmin(qc, qm);
          const int32_t xi = (int32_t)(uint32_t)__double_as_longlong(xb);
          x[h] = xb >= f64_at(Pv, k) ? clv[k] : xi;                   // CC:134-135
        }
        acc32 += x[0] + x[1];
      }
    }
    set_round_nearest();
    acc += (uint64_t)(int64_t)acc32;
  };
  // class B (and class-A lanes sharing its wave)
  auto sum_b = [&](uint32_t g0, int cnt) {
    cnt = __builtin_amdgcn_readfirstlane(cnt);  // keep the trip count scalar
    const FitGroup* gbase = fast_b + g0;
    const double bias = FIT_BIAS;
    int32_t acc32 = 0;
    set_round_down();
    for (int gi = 0; gi < cnt; ++gi) {
      int io = gi;
      asm volatile("" : "+s"(io));
      const FitGroup* g = gbase + io;
      const i32x16 fcv = *reinterpret_cast<const i32x16*>(g->fc);
      const i32x16 fmv = *reinterpret_cast<const i32x16*>(g->fm);
      const i32x16 Pv = *reinterpret_cast<const i32x16*>(g->Pb);
#pragma unroll
      for (int u = 0; u < FIT_GROUP / 2; ++u) {
        int32_t x[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * u + h;
          const double qc = __builtin_fma(f64_at(fcv, k), rc, bias);  // 2^52 + floor(fc/c)
          const double qm = __builtin_fma(f64_at(fmv, k), rm, bias);  // 2^52 + floor(fm/m)
          const double xb = min_f64_s(__builtin_fmin(qc, qm), f64_at(Pv, k));
          x[h] = (int32_t)(uint32_t)__double_as_longlong(xb);  // min(findMin(qc, qm), P)
        }
        acc32 += x[0] + x[1];
      }
    }
    set_round_nearest();
    acc += (uint64_t)(int64_t)acc32;
  };

  {
    // every wave of the workgroup runs the loop (the barrier per chunk); the slot the
    // chunk's claim is read from was written before the previous barrier, the slot
    // wave 0 writes during it was last read before that barrier
    for (uint32_t k = 0;; ++k) {
      const uint32_t cur = base + (k == 0 ? first : __builtin_amdgcn_readfirstlane(q_slot[k & 1u]));
      if (cur >= lim) break;  // workgroup-uniform
      const uint32_t rem = lim - cur;
      uint32_t qn = rem / (FIT_QDIV * wps);
      qn = qn < FIT_QMIN ? FIT_QMIN : (qn > qsz ? qsz : qn);

      claim_issue(qn);
      const int cnt = (int)((cur + qcur < lim ? cur + qcur : lim) - cur);
      qcur = qn;
      if (wave_fast) {
        if constexpr (NC) {
          if (!wave_b) sum_a_nc(cur, cnt);
          else sum_b_nc(cur, cnt);
        } else {
          if (!wave_b) sum_a(cur, cnt);
          else sum_b(cur, cnt);
        }
      }
      claim_publish((k + 1u) & 1u);
      {  // priority 3, 2, 1, 0 through the quarters of the share (round 5 A/B: boosted
         // through the static first claim only, or then 1 / 0 by halves: slower / equal;
         // 3 only until the loop starts, then 2, 2, 1, 0 or 2, 1, 0, 0: equal / slower)
        pr_done += (uint32_t)cnt;
        const uint32_t lv = (4u * pr_done) / pr_share;
        if (lv == 0) __builtin_amdgcn_s_setprio(3);
        else if (lv == 1) __builtin_amdgcn_s_setprio(2);
        else if (lv == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      KCC_TLV(2048 + b % 4096, 4, (uint64_t)k + 1);
#ifdef KCC_TIMELINE
      tl_done += (uint32_t)cnt;
      if (k == 0) KCC_TL(2048 + b % 4096, 6);
#endif
    }
    if (wv == 0 && lane == 0) {  // this workgroup made its last claim
      const uint32_t d = atomicAdd(qp + 1, 1u);
      if (d == wseg - 1u) {  // the segment's last one:
        qp[0] = 0;                                               // reset for the next launch
        qp[1] = 0;
      }
    }
  }
  KCC_TL(2048 + b % 4096, 2);
#ifdef KCC_TIMELINE
  KCC_TLV(2048 + b % 4096, 7, tl_done);
#endif
  if (idle) return;  // a wave wholly past S (it took the claims' barriers)
  if (wave_exact) {  // exact-path specs: every node row (SlowNode), this workgroup's share
    const uint32_t nn = (uint32_t)n_nodes;  // < 2^28 per device
    const uint32_t pn = (nn + (uint32_t)gy - 1u) / (uint32_t)gy;
    const uint32_t a0 = (uint32_t)by * pn < nn ? (uint32_t)by * pn : nn;
    const int64_t i1 = a0 + pn < nn ? a0 + pn : nn;
    for (int64_t i = a0; i < i1; ++i) eval_slow(i);
  } else {  // rows outside the fast bounds, shared out over the column's workgroups
    const int64_t n_slow = (int64_t)counters[CNT_SLOW_ROWS + chunk];
    for (int64_t j = by; j < n_slow; j += gy) eval_slow(slow_list[j]);
  }

  {  // (node, spec) pairs evaluated on the exact path (statistics)
    const unsigned long long act = __ballot(active);
    if (slow_iters && lane == 0)
      atomicAdd(&counters[CNT_SLOW_PAIRS], (unsigned long long)slow_iters * (unsigned long long)__popcll(act));
  }
  // the clamp in the fit: the rows clamped for every spec (P <= 0, never streamed), once
  // per spec (the column's workgroup by == 0) for the normal specs (exact waves walked
  // every row on the exact path)
  if (NC && by == 0 && wave_fast) acc -= (uint64_t)counters[CNT_CLAMP_ALL];
  // a faulted device's partial carries the fault to every consumer (SPEC_FAULT_MARK)
  if (by == 0 && device_faulted(faults)) errs += SPEC_FAULT_MARK;
  if (active) {
    atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[s]), acc);
    if (errs) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[S + s]), errs);
  }
  KCC_TL(2048 + b % 4096, 3);
}

template <bool NC>
__global__ __launch_bounds__(256) KCC_FIT_ATTR void fit_kernel(
    int64_t n_nodes, uint32_t* __restrict__ queue, const FitGroupA* __restrict__ fast_a,
    const FitGroup* __restrict__ fast_b, const SlowNode* __restrict__ slow,
    const int64_t* __restrict__ slow_list, int64_t S, const SpecRec* __restrict__ specs,
    int64_t* __restrict__ partial, unsigned long long* __restrict__ counters, int32_t chunk,
    int32_t gx, int32_t gy, const int32_t* __restrict__ fast_cl,
    const unsigned long long* __restrict__ faults) {
  __shared__ uint32_t q_slot[2];
  fit_body<NC>(n_nodes, queue, fast_a, fast_b, slow, slow_list, S, specs, partial, counters, chunk,
               gx, gy, fast_cl, faults, (int32_t)blockIdx.x, q_slot);
}

__global__ void fit_finalize_kernel(int64_t S, const int64_t* __restrict__ partial,
                                    const int32_t* __restrict__ perm, int64_t* __restrict__ totals,
                                    int32_t* __restrict__ spec_err,
                                    const unsigned long long* __restrict__ faults) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  const int32_t dst = perm[i];
  const bool err = partial[S + i] != 0;
  const bool faulted = device_faulted(faults) || (uint64_t)partial[S + i] >= SPEC_FAULT_MARK;
  totals[dst] = err || faulted ? 0 : partial[i];
  spec_err[dst] = faulted ? SPEC_ERR_FAULT : err ? SPEC_ERR_DIV0 : 0;
}

// One-shot exchange + finalize (P2PArgs, kcc_internal.h).  256 threads, specs strided over
// the grid (at most P2P_MAX_WG workgroups: all resident at once, since each waits for the
// flag the last one publishes).
[[maybe_unused]] constexpr uint32_t P2P_SPIN_MAX = 1u << 21;  // flag polls before a wait gives up (seconds)
constexpr int64_t P2P_MAX_WG = 256;
__global__ __launch_bounds__(256) void exchange_finalize_kernel(P2PArgs a) {
  const int64_t S = a.S, smax = a.smax, i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t gs = (int64_t)gridDim.x * 256;
  // this launch's epoch: one past the last one pushed (a device word that the launch's last
  // workgroup to push advances, after every workgroup read it here: each reads it before
  // it arrives), so a replayed graph pushes a new epoch every time
  const uint64_t epoch = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  // a fault word set before this launch (an earlier give-up): the results stay marked
  const bool faulted_in = device_faulted(a.faults);
  const int W = a.W, par = (int)(epoch & 1u);
  const int64_t slot = ((int64_t)par * W + a.rank) * 2 * smax;  // this sender's data slot
  const size_t fw = p2p_flag_words(W);
  // 1. push this rank's two words of each of its specs into every mailbox
  for (int64_t i = i0; i < S; i += gs) {
    const int64_t v0 = a.partial[i], v1 = a.partial[S + i];
    for (int p = 0; p < W; ++p) {
      int64_t* d = reinterpret_cast<int64_t*>(a.mbox[p]) + fw + slot;
      d[i] = v0;
      d[smax + i] = v1;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the pushes are performed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1u) {  // every workgroup has pushed: publish the epoch
      __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.epoch, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int p = 0; p < W; ++p)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(a.mbox[p]) + ((int64_t)par * W + a.rank) * 8,
                           epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // 2. every sender's flag of this epoch in this rank's own mailbox (thread p polls p's)
  __shared__ uint32_t gave_up;
  if (threadIdx.x == 0) gave_up = 0;
  __syncthreads();
  if (threadIdx.x < (unsigned)W) {
#ifdef KCC_DIAG_P2P_GIVEUP  // fault-path test builds only: every wait gives up at once
    atomicAdd(&a.faults[FAULT_P2P], 1ull);
    gave_up = 1;
#else
    const uint64_t* f =
        reinterpret_cast<const uint64_t*>(a.mbox[a.rank]) + ((int64_t)par * W + threadIdx.x) * 8;
    uint32_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (++spins >= P2P_SPIN_MAX) {  // a peer never pushed: count it, go on (never on a healthy run)
        atomicAdd(&a.faults[FAULT_P2P], 1ull);
        gave_up = 1;  // (a plain LDS store: any waiter that gave up sets it)
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
#endif
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale mailbox lines
  const bool faulted = faulted_in || gave_up != 0;
  // 3. the sums over the W senders, finalized
  const int64_t* d = reinterpret_cast<const int64_t*>(a.mbox[a.rank]) + fw + (int64_t)par * W * 2 * smax;
  for (int64_t i = i0; i < S; i += gs) {
    uint64_t s0 = 0, s1 = 0;
    for (int p = 0; p < W; ++p) {
      s0 += (uint64_t)__builtin_nontemporal_load(d + (int64_t)p * 2 * smax + i);
      s1 += (uint64_t)__builtin_nontemporal_load(d + (int64_t)p * 2 * smax + smax + i);
    }
    const int32_t dst = a.perm[i];
    const bool fi = faulted || s1 >= SPEC_FAULT_MARK;  // (a sender's fault, in its counts)
    a.totals[dst] = s1 != 0 || fi ? 0 : (int64_t)s0;
    a.spec_err[dst] = fi ? SPEC_ERR_FAULT : s1 != 0 ? SPEC_ERR_DIV0 : 0;
  }
}

__global__ void partial_add_kernel(int64_t n, int64_t* __restrict__ dst,
                                   const int64_t* __restrict__ src) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (int64_t)((uint64_t)dst[i] + (uint64_t)src[i]);
}

inline unsigned grid_for(int64_t n, int block, int64_t cap) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace

namespace {
// Resident workgroups of `kern` (block threads, lds dynamic bytes) on the current device:
// the occupancy API's answer per CU x the CU count, cached per device ordinal (contexts on
// several devices each get their own; concurrent first calls store the same value).
constexpr int MAX_DEVS = 64;
int64_t resident_blocks(std::atomic<int64_t> (&cache)[MAX_DEVS], const void* kern, int block,
                        size_t lds, int64_t fallback) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return fallback;
  if (dev < MAX_DEVS) {
    const int64_t v = cache[dev].load(std::memory_order_relaxed);
    if (v) return v;
  }
  int cus = 0, blocks = 0;
  int64_t v = fallback;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kern, block, lds) == hipSuccess &&
      cus > 0 && blocks > 0)
    v = (int64_t)cus * blocks;
  if (dev < MAX_DEVS) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

int64_t reduce_resident_waves(bool limits) {
  static std::atomic<int64_t> cache[2][MAX_DEVS];
  int64_t r = RED_WAVES_PER_BLOCK *
              resident_blocks(cache[limits ? 1 : 0],
                              limits ? reinterpret_cast<const void*>(reduce_kernel<4, false>)
                                     : reinterpret_cast<const void*>(reduce_kernel<2, false>),
                              256, 0, 2048);
  return r;
}
}  // namespace

int32_t reduce_range(int64_t n_containers, bool limits, int64_t reserve_waves) {
  int64_t slots = reduce_resident_waves(limits) - reserve_waves;
  if (slots < 64) slots = 64;
  const int64_t r = slots * RED_TILE;
  int64_t t = (n_containers + r - 1) / r;
  if (t < 1) t = 1;
  if (t > ((int64_t)1 << 20)) t = (int64_t)1 << 20;  // range < 2^28 (int32 relative offsets)
  return (int32_t)(t * RED_TILE);
}

int64_t reduce_tail_records() {
  const int64_t a = reduce_resident_waves(false), b = reduce_resident_waves(true);
  return (a > b ? a : b) + 64;
}

hipError_t launch_reduce(int64_t n_nodes, int64_t c0, int64_t n_containers, const int64_t* node_ptr,
                         const uint64_t* cpu_req, const int64_t* mem_req,
                         const uint64_t* cpu_lim, const int64_t* mem_lim,
                         uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu, int64_t* lim_mem,
                         uint64_t* tail, unsigned long long* faults, hipStream_t s,
                         const RankArgs* rank, const NpArgs* npa, hipEvent_t ev_start,
                         hipEvent_t ev_stop) {
  RankArgs ra{};
  if (rank) ra = *rank;
  NpArgs np{};
  if (npa) np = *npa;
  const int32_t npb = np.n_place + np.n_rows;
  const bool limits = cpu_lim && mem_lim && lim_cpu && lim_mem;
  const bool red = n_nodes > 0 && n_containers > 0;
  if (n_nodes >= RED_MAX_NODES) return hipErrorInvalidValue;
  if (n_nodes > 0 && n_containers == 0) {  // no containers: every sum is 0
    hipError_t e;
    if ((e = hipMemsetAsync(used_cpu, 0, 8 * (size_t)n_nodes, s)) != hipSuccess ||
        (e = hipMemsetAsync(used_mem, 0, 8 * (size_t)n_nodes, s)) != hipSuccess)
      return e;
    if (limits && ((e = hipMemsetAsync(lim_cpu, 0, 8 * (size_t)n_nodes, s)) != hipSuccess ||
                   (e = hipMemsetAsync(lim_mem, 0, 8 * (size_t)n_nodes, s)) != hipSuccess))
      return e;
  }
  if (!red && ra.n_blocks == 0 && npb == 0) return hipSuccess;
  if (limits && (ra.n_blocks > 0 || npb > 0)) return hipErrorInvalidValue;  // (NA = 2 only)
  if (npb > 0 && (ra.n_blocks != 1 || !ra.zero_only || !ra.done_flag)) return hipErrorInvalidValue;
  // the rank workgroups: behind the reduce's on long reduces, so they take the slots of
  // its first waves to finish; in front on short ones, where the reduce's range is sized
  // for the slots they leave (one round of workgroups: a reduce workgroup that waited for
  // a rank workgroup's slot started ~10 us late on the 8-way C4 rank, round 5)
  const bool ranks_last = n_containers >= RED_RANKS_LAST_MIN;
  const int64_t reserve = ranks_last ? 0 : (int64_t)RED_WAVES_PER_BLOCK * ra.n_blocks;
  const int32_t range = red ? reduce_range(n_containers, limits, reserve) : RED_TILE;
  const int64_t waves = red ? (n_containers + range - 1) / range : 0;
  if (waves > reduce_tail_records()) return hipErrorInvalidValue;
  const int64_t red_blocks = (waves + RED_WAVES_PER_BLOCK - 1) / RED_WAVES_PER_BLOCK;
  const unsigned blocks = (unsigned)(red_blocks + ra.n_blocks + npb);
  np.ptr = node_ptr;
  np.c0 = c0;
  np.range = range;
  np.red_waves = (int32_t)waves;
  RedArgs a{};
  a.n_nodes = n_nodes;
  a.c0 = c0;
  a.c_end = c0 + n_containers;
  a.range = range;
  a.ptr = node_ptr;
  a.in[0] = cpu_req;
  a.in[1] = reinterpret_cast<const uint64_t*>(mem_req);
  a.in[2] = limits ? cpu_lim : nullptr;
  a.in[3] = limits ? reinterpret_cast<const uint64_t*>(mem_lim) : nullptr;
  a.out[0] = used_cpu;
  a.out[1] = reinterpret_cast<uint64_t*>(used_mem);
  a.out[2] = limits ? lim_cpu : nullptr;
  a.out[3] = limits ? reinterpret_cast<uint64_t*>(lim_mem) : nullptr;
  a.tail = tail;
  a.faults = faults;
  a.ranks_last = ranks_last ? 1 : 0;
  auto kern = limits ? reduce_kernel<4, false> : npb > 0 ? reduce_kernel<2, true> : reduce_kernel<2, false>;
  if (ev_start || ev_stop)  // (profiling: the dispatch packet's own timestamps)
    hipExtLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, ev_start, ev_stop, 0, a, ra, np);
  else
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, a, ra, np);
  return hipGetLastError();
}

hipError_t launch_node_prep(int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, FitGroupA* fast_a, FitGroup* fast_b,
                            SlowNode* slow, int64_t* slow_list, int64_t n_specs,
                            ClampWork cw, unsigned long long* counters, int chunk, int64_t row0,
                            int64_t call_nodes, hipStream_t s, bool dense,
                            const PlaceArgs* place, int32_t* fast_cl) {
  if (n_nodes <= 0 && !place) return hipSuccess;
  if (fast_cl && (n_specs > CLAMP_LDS_SPECS || dense)) return hipErrorInvalidValue;
  const int64_t pr = clamp_pass_rows(call_nodes);
  if (row0 % pr != 0 || (pr != 1024 && pr != 4096)) return hipErrorInvalidValue;
  // one resident round of workgroups (LDS-bound at S <= CLAMP_LDS_SPECS: one per CU)
  const int mode = n_specs <= CLAMP_LDS_SPECS ? 2 : n_specs <= (int64_t)NP_ST_MAX * CLAMP_LDS_SPECS ? 1 : 0;
  PlaceArgs pa{};
  if (place) {  // (node_prep reads only what spec_rank wrote)
    pa = *place;
    pa.n_blocks = (int32_t)((n_specs + KCC_NODE_PREP_BLOCK - 1) / KCC_NODE_PREP_BLOCK);
  }
  const bool nc = fast_cl != nullptr;  // (mode 2)
  const size_t lds_bytes = nc ? 0 : mode == 2 ? NODE_PREP_LDS : mode == 1 ? NODE_PREP_LDS_SRCH : 0;
  auto kern = nc ? (pr == 1024 ? node_prep_kernel<2, 1, true> : node_prep_kernel<2, 4, true>)
            : pr == 1024 ? (mode == 2 ? node_prep_kernel<2, 1, false> : mode == 1 ? node_prep_kernel<1, 1, false> : node_prep_kernel<0, 1, false>)
                         : (mode == 2 ? node_prep_kernel<2, 4, false> : mode == 1 ? node_prep_kernel<1, 4, false> : node_prep_kernel<0, 4, false>);
  static std::atomic<int64_t> resident[2][4][MAX_DEVS];
  const int64_t res = resident_blocks(resident[pr == 1024 ? 0 : 1][nc ? 3 : mode],
                                      reinterpret_cast<const void*>(kern), KCC_NODE_PREP_BLOCK,
                                      lds_bytes, 256);
  const int64_t cap = res < NODE_PREP_GRID ? res : NODE_PREP_GRID;
  const unsigned np_blocks = n_nodes > 0 ? grid_for(n_nodes, (int)pr, cap) : 0u;
  hipLaunchKernelGGL(kern, dim3(np_blocks + (unsigned)pa.n_blocks), dim3(KCC_NODE_PREP_BLOCK),
                     lds_bytes, s, n_nodes, alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu,
                     used_mem, fast_a, fast_b, slow, slow_list, n_specs, cw,
                     counters, (int32_t)chunk, (int32_t)(dense ? 1 : 0), row0 / pr, pa, fast_cl);
  return hipGetLastError();
}

RankArgs rank_args(int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
                   const ClampWork& cw, unsigned long long* counters, uint32_t* arrive,
                   bool zero_only) {
  RankArgs ra{};
  ra.S = n_specs;
  ra.c_in = spec_cpu;
  ra.m_in = spec_mem;
  ra.part = cw.rank;
  ra.arrive = arrive;
  ra.bcnt = cw.bcnt;
  ra.cs = cw.cs;
  ra.ms = cw.ms;
  ra.mr_c = cw.mr_c;
  ra.cr_m = cw.cr_m;
  ra.C = cw.C;
  ra.c_stride = cw.c_stride;
  const int64_t wmax = (n_specs + 63) / 64 + 2;  // >= this call's T + 2 (nN <= S)
  ra.c_cells = wmax * wmax < cw.c_stride ? wmax * wmax : cw.c_stride;
  ra.counters = counters;
  ra.n_blocks = n_specs <= 0 ? 0
               : zero_only ? 1
               : n_specs <= RANK_FULL_MAX ? (int32_t)((n_specs + 63) / 64 * rank_slices(n_specs))
                                          : (int32_t)(rank_slices(n_specs) * rank_slices(n_specs));
  ra.zero_only = zero_only ? 1 : 0;
  return ra;
}

hipError_t launch_spec_rank(const RankArgs& ra, hipStream_t s) {
  if (ra.n_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(spec_rank_kernel, dim3((unsigned)ra.n_blocks), dim3(256), 0, s, ra);
  return hipGetLastError();
}

hipError_t launch_clamp_apply(int64_t n_specs, int64_t n_nodes, ClampWork cw,
                              const unsigned long long* counters, int64_t* partial, hipStream_t s,
                              const FinArgs* fin) {
  if (n_specs <= 0) return hipSuccess;
  cw.n_pass = clamp_passes(n_nodes);
  cw.pass_recs = 2 * clamp_pass_rows(n_nodes);
  const int64_t T = (n_specs + 63) / 64;  // >= this call's T (normal specs only)
  if (!clamp_c_full(T))  // C's row suffix sums (the kernel exits when this call's C is full)
    hipLaunchKernelGGL(clamp_crows_kernel, dim3((unsigned)((T + 2 + 3) / 4)), dim3(256), 0, s, cw,
                       counters);
  // binned: each bin's records split over G workgroups (D is linear in the table: each
  // part subtracts its own share), as many as one round of resident workgroups holds
  // (C4: 1 per CU by registers, G = 2; more parts in a second round, G = 4 / 8: +7 / +24 us;
  // 64 VGPRs for 2 per CU and G = 4: equal)
  const FinArgs f = fin ? *fin : FinArgs{};
  hipLaunchKernelGGL(clamp_apply_kernel, dim3((unsigned)clamp_apply_blocks(n_specs)), dim3(CP_THREADS),
                     0, s, cw, counters, n_specs, partial, f);
  return hipGetLastError();
}

int64_t clamp_apply_blocks(int64_t n_specs) {
  if (n_specs <= 0) return 0;
  const int64_t T = (n_specs + 63) / 64;
  static std::atomic<int64_t> cache[MAX_DEVS];  // clamp_apply workgroups resident at once
  const int64_t resident = resident_blocks(cache, reinterpret_cast<const void*>(clamp_apply_kernel),
                                           CP_THREADS, 0, 256);
  int64_t G = 1;
  if (clamp_binned(n_specs))
    while (G < CP_SPLIT && 2 * T * G * 2 <= resident) G *= 2;
  return 2 * T * G;
}

int64_t fit_resident_blocks() {  // 256-thread fit workgroups resident on the device at once
  static std::atomic<int64_t> cache[MAX_DEVS];
  return resident_blocks(cache, reinterpret_cast<const void*>(fit_kernel<false>), 256, 0, 2048);
}

// the fit's workgroups per spec column: one round of resident workgroups (the queue
// balances the waves; the stream's length is only known on the device); a chunk of a
// pipelined call gets its node share of the round; no more waves per column than claims
// at the full length
static int64_t fit_grid_y(int64_t n_nodes, int64_t n_specs, int64_t grid_nodes) {
  const int64_t gx = (n_specs + FIT_SPW - 1) / FIT_SPW;
  const int64_t n_groups = fit_groups(n_nodes);
  int64_t gy = fit_resident_blocks() / gx;
  if (grid_nodes > n_nodes) gy = gy * n_nodes / grid_nodes;
  if (gy >= 16) gy = gy / 8 * 8;  // whole XCD rounds
  const int64_t claims = (n_groups + FIT_QCHUNK - 1) / FIT_QCHUNK;
  if (gy > claims) gy = claims;
  if (gy < 1) gy = 1;
  return gy;
}

hipError_t launch_fit(int64_t n_nodes, const FitGroupA* fast_a, const FitGroup* fast_b,
                      const SlowNode* slow,
                      const int64_t* slow_list, int64_t n_specs, SpecPrep sp, int64_t* partial,
                      unsigned long long* counters, uint32_t* queue, int chunk,
                      int64_t grid_nodes, hipStream_t s, const unsigned long long* faults,
                      const int32_t* fast_cl, hipEvent_t ev_start, hipEvent_t ev_stop) {
  if (n_nodes <= 0 || n_specs <= 0) return hipSuccess;
  const int64_t gx = (n_specs + FIT_SPW - 1) / FIT_SPW;
  const int64_t gy = fit_grid_y(n_nodes, n_specs, grid_nodes);
  // 1-D grid of gx * roundup(gy, 8) workgroups, remapped XCD-aware in the kernel
  const int64_t blocks = gx * ((gy + 7) / 8 * 8);
  if (blocks > 0x7fffffffLL || gy > 0x7fffffffLL) return hipErrorInvalidValue;
  auto kern = fast_cl ? fit_kernel<true> : fit_kernel<false>;
  if (ev_start || ev_stop)  // (profiling: the dispatch packet's own timestamps)
    hipExtLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, s, ev_start, ev_stop, 0, n_nodes,
                          queue, fast_a, fast_b, slow, slow_list, n_specs, sp.rec, partial, counters,
                          (int32_t)chunk, (int32_t)gx, (int32_t)gy, fast_cl, faults);
  else
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, s, n_nodes, queue, fast_a,
                       fast_b, slow, slow_list, n_specs, sp.rec, partial, counters, (int32_t)chunk,
                       (int32_t)gx, (int32_t)gy, fast_cl, faults);
  return hipGetLastError();
}

hipError_t launch_fit_finalize(int64_t n_specs, const int64_t* partial, const int32_t* perm,
                               int64_t* totals, int32_t* spec_err,
                               const unsigned long long* faults, hipStream_t s) {
  if (n_specs <= 0) return hipSuccess;
  hipLaunchKernelGGL(fit_finalize_kernel, dim3(grid_for(n_specs, 256, 1 << 30)), dim3(256), 0, s,
                     n_specs, partial, perm, totals, spec_err, faults);
  return hipGetLastError();
}

hipError_t launch_exchange_finalize(const P2PArgs& a, hipStream_t s) {
  if (a.S <= 0) return hipSuccess;
  if (a.S > a.smax || a.W < 1 || a.W > P2P_MAX_RANKS || a.rank < 0 || a.rank >= a.W ||
      !a.epoch || !a.faults || !a.arrive)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(exchange_finalize_kernel, dim3(grid_for(a.S, 256, P2P_MAX_WG)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_partial_add(int64_t n, int64_t* dst, const int64_t* src, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(partial_add_kernel, dim3(grid_for(n, 256, 1 << 30)), dim3(256), 0, s, n, dst,
                     src);
  return hipGetLastError();
}

}  // namespace kcc

#ifdef KCC_TIMELINE
// diagnostic builds only: copy the timeline stamps (4096 x 4 u64) to `host`, then zero them
extern "C" int kcc_debug_timeline(void* host) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(kcc::kcc_tl), sizeof(uint64_t) * 8192 * 8) != hipSuccess)
    return -2;
  static uint64_t zero[8192][8];
  return hipMemcpyToSymbol(HIP_SYMBOL(kcc::kcc_tl), zero, sizeof(zero)) == hipSuccess ? 0 : -3;
}
#endif
