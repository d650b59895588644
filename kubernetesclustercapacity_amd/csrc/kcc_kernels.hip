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

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kcc_internal.h"

namespace kcc {

namespace {

__device__ __forceinline__ unsigned long long atomic_add_u64(uint64_t* p, uint64_t v) {
  return atomicAdd(reinterpret_cast<unsigned long long*>(p),
                   static_cast<unsigned long long>(v));
}

// ----------------------------------------------------------------------------
// (a) segmented reduce
// ----------------------------------------------------------------------------

// Zero the outputs; for every wave range [c0 + x*range, ...) record the node owning
// its first container.  Node indices are local to the launch (ptr and the outputs are
// offset by the caller); the container offsets in ptr are absolute and the launch
// covers containers [c0, c_end).
__global__ void reduce_mark_kernel(int64_t n_nodes, int64_t c0, int64_t c_end, int32_t range,
                                   const int64_t* __restrict__ ptr,
                                   int64_t* __restrict__ wave_node, uint64_t* __restrict__ o0,
                                   uint64_t* __restrict__ o1, uint64_t* __restrict__ o2,
                                   uint64_t* __restrict__ o3) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_nodes; j += stride) {
    o0[j] = 0;
    o1[j] = 0;
    if (o2) o2[j] = 0;
    if (o3) o3[j] = 0;
    int64_t b = ptr[j] - c0, e = ptr[j + 1] - c0;  // relative to the launch's first container
    b = b < 0 ? 0 : b;
    e = e > c_end - c0 ? c_end - c0 : e;
    if (e > b) {
      for (int64_t x = (b + range - 1) / range * range; x < e; x += range)
        wave_node[x / range] = j;
    }
  }
}

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

// RED_IPL (=4) consecutive 64-bit values of one array for this lane: two 16-B
// range-checked buffer loads (outside the descriptor's range they read 0), so the
// prefetch is branch-free and never waits where it is issued.
// The lane offset (voff) is loop-invariant and the tile offset goes in soffset, so no
// address VGPR is recomputed per tile (a recomputed address register that the
// allocator shares with an in-flight load's destination forces a vmcnt(0) wait).
__device__ __forceinline__ void load_quad(__amdgpu_buffer_rsrc_t r, int32_t voff, int32_t soff,
                                          uint64_t (&x)[4]) {
  const u64x2 lo = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  const u64x2 hi =
      __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, soff, 0));
  x[0] = lo.x;
  x[1] = lo.y;
  x[2] = hi.x;
  x[3] = hi.y;
}

// One wavefront walks a contiguous range of `range` containers in tiles of
// RED_TILE = 256 (4 per lane, coalesced SoA buffer loads, next tile prefetched).
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
//      in front of the next tile's data wait.  Only the (at most two) nodes crossing
//      the range boundaries use 64-bit atomics.
// Nodes before the wave's first owned node and the empty nodes ahead of node0 are
// zeroed by reduce_mark_kernel; every other node of the wave's run, empty ones
// included, is written by its flush.
constexpr uint32_t RED_OOB_OFFSET = 0x7ffffff0u;  // > any output's range (n_nodes < 2^28)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int NA>
__global__ __launch_bounds__(256)
#ifdef KCC_RED_WAVES_PER_EU
__attribute__((amdgpu_waves_per_eu(KCC_RED_WAVES_PER_EU)))
#endif
void reduce_kernel(
    int64_t n_nodes, int64_t c0, int64_t n_cont, int32_t range, const int64_t* __restrict__ ptr,
    const uint64_t* __restrict__ in0, const uint64_t* __restrict__ in1,
    const uint64_t* __restrict__ in2, const uint64_t* __restrict__ in3,
    const int64_t* __restrict__ wave_node, uint64_t* __restrict__ out0,
    uint64_t* __restrict__ out1, uint64_t* __restrict__ out2, uint64_t* __restrict__ out3) {
  __shared__ __attribute__((aligned(16))) uint64_t pre_s[RED_WAVES_PER_BLOCK][NA][RED_TILE];
  const int lane = threadIdx.x & 63;
  // wave index made provably uniform (T20: no waterfall loops around the buffer ops)
  const int32_t w = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * RED_WAVES_PER_BLOCK +
                                                             (threadIdx.x >> 6)));
  // containers [c0, n_cont): absolute indices, like the offsets in ptr (node indices
  // are local to the launch)
  const int64_t wb = c0 + (int64_t)w * range;
  if (wb >= n_cont) return;  // wave-uniform; no block-level barrier in this kernel
  const int32_t len = (int32_t)(n_cont - wb < range ? n_cont - wb : range);
  uint64_t (*pre)[RED_TILE] = pre_s[threadIdx.x >> 6];
  const uint64_t* in[4] = {in0, in1, in2, in3};
  uint64_t* out[4] = {out0, out1, out2, out3};
  __amdgpu_buffer_rsrc_t rs[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k)  // whole 16-B pairs only: an odd last item is fixed up below
    rs[k] = __builtin_amdgcn_make_buffer_rsrc((void*)(in[k] + wb), (short)0,
                                              (int)((len & ~1) * 8), 0x00020000);

  const int64_t node0 = wave_node[w];
  const bool first_open = ptr[node0] < wb;           // node0 began in an earlier range
  const int64_t own_lo = node0 + (first_open ? 1 : 0);  // first node stored plainly
  int64_t cur = node0;  // node holding the current tile's first item
  uint64_t carry[NA];   // node cur's running sum over the earlier tiles of this range
  uint64_t res[NA];     // sums of block blk's nodes (lane l <-> node 64*blk + l)
#pragma unroll
  for (int k = 0; k < NA; ++k) carry[k] = res[k] = 0;

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
      for (int k = 0; k < NA; ++k) out[k][pend_j] = resF[k];
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
                                            (int)voff, 0, 0);
    pend = false;
  };

  uint64_t xa[NA][4], xb[NA][4];
#if KCC_RED_PREFETCH == 2
  uint64_t xc[NA][4];
#endif
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    load_quad(rs[k], lane * 32, 0, xa[k]);
#if KCC_RED_PREFETCH == 2
    load_quad(rs[k], lane * 32, RED_TILE * 8, xb[k]);
#endif
  }

  auto tile = [&](uint64_t (&x)[NA][4], uint64_t (&nx)[NA][4], const int32_t tb) {
#ifndef KCC_DIAG_RED_NOSTORE
    issue_pending();
#endif
#pragma unroll
    for (int k = 0; k < NA; ++k)
      load_quad(rs[k], lane * 32, (tb + KCC_RED_PREFETCH * RED_TILE) * 8, nx[k]);
#ifdef KCC_DIAG_RED_LOADONLY
#pragma unroll
    for (int k = 0; k < NA; ++k) carry[k] += x[k][0] + x[k][1] + x[k][2] + x[k][3];
    return;
#endif
    const int32_t p0 = tb + 4 * lane;  // relative position of this lane's first item
    if ((len & 1) && p0 <= len - 1 && len - 1 < p0 + 4) {  // odd tail: last item alone
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        const uint64_t v = in[k][wb + len - 1];
#pragma unroll
        for (int i = 0; i < 4; ++i)  // static indices only (no scratch)
          if (p0 + i == len - 1) x[k][i] = v;
      }
    }

    // --- 1. tile-local inclusive prefix sums -> LDS -----------------------------
    uint64_t tot[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const uint64_t q0 = x[k][0], q1 = q0 + x[k][1], q2 = q1 + x[k][2], q3 = q2 + x[k][3];
      const uint64_t P = wave_incl_scan_u64(q3);
      const uint64_t ex = P - q3;
      u64x2* dst = reinterpret_cast<u64x2*>(&pre[k][4 * lane]);
      dst[0] = u64x2{ex + q0, ex + q1};
      dst[1] = u64x2{ex + q2, P};
      tot[k] = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(P >> 32), 63) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((uint32_t)P, 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // --- 2./3. nodes ending in this tile, block by block ----------------------------
    const int32_t eN_rel = rel_clamp(eNr, wb);  // next block's ends (previous tile's load)
    const int32_t lim = tb + RED_TILE < len ? tb + RED_TILE : len;
    int32_t last_end = -1;  // end of the last node that ended in this tile (-1: none)
    for (;;) {
      const int64_t j = 64 * blk + lane;
      int32_t s = __builtin_amdgcn_update_dpp(0, eA, DPP_WAVE_SHR1, 0xf, 0xf, false);
      if (lane == 0) s = sA0;
      const bool act = (j >= cur) && (j < n_nodes) && (eA <= lim);
      if (act) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          uint64_t sum = 0;
          if (eA > s) {  // s <= tb only for node cur, which began in an earlier tile
            const uint64_t startp = s > tb ? pre[k][s - 1 - tb] : (0ull - carry[k]);
            sum = pre[k][eA - 1 - tb] - startp;
          }
          if (j == node0 && first_open) atomic_add_u64(&out[k][j], sum);
          res[k] = sum;
        }
      }
      const unsigned long long bal = __ballot(act);
      if (!bal) break;
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
    if (last_end >= 0) {  // node cur is open at the tile end: its sum so far
#pragma unroll
      for (int k = 0; k < NA; ++k)
        carry[k] = tot[k] - pre[k][last_end - 1 - tb];
    } else {
#pragma unroll
      for (int k = 0; k < NA; ++k) carry[k] += tot[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
#if KCC_RED_PREFETCH == 2
  for (int32_t tb = 0; tb < len; tb += 3 * RED_TILE) {
    tile(xa, xc, tb);
    if (tb + RED_TILE < len) tile(xb, xa, tb + RED_TILE);
    if (tb + 2 * RED_TILE < len) tile(xc, xb, tb + 2 * RED_TILE);
  }
#else
  for (int32_t tb = 0; tb < len; tb += 2 * RED_TILE) {
    tile(xa, xb, tb);
    if (tb + RED_TILE < len) tile(xb, xa, tb + RED_TILE);
  }
#endif
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
      for (int k = 0; k < NA; ++k) out[k][j] = res[k];
#endif
    }
  }
  // the node open at the end of the range continues into the next wave's range
  if (wb + len < n_cont && lane == 0 && cur < n_nodes) {
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if (carry[k] != 0) atomic_add_u64(&out[k][cur], carry[k]);
  }
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

// #{k < n : a[k] <= v} for a sorted ascending (binary search, n <= 2^31)
// #{k < 4096 : a[k] <= v} for a sorted ascending (8-ary: after the step of width s the
// answer lies in [lo, lo + s])
template <class T>
__device__ __forceinline__ uint32_t search8_4096(const T* a, T v) {
  static_assert(CLAMP_LDS_SPECS == 4096, "search8_4096 covers 8^4 entries");
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t s = 512; s >= 1; s /= 8) {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t j = 1; j < 8; ++j) cnt += a[lo + j * s - 1] <= v ? 1u : 0u;
    lo += cnt * s;
  }
  return lo;
}

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

// Per-node free capacity (CC:119-135 operands).  Rows that fit the fast-path
// bounds get exact FitGroupA fields (and FitGroup fields when class-B specs exist);
// the others get all-zero fields (contribute exactly 0 on the fast paths) and are
// appended to slow_list for the exact 64-bit path.  Covers the padding of the last
// group too (zero fields, not listed).
#define KCC_NODE_PREP_BLOCK 1024  // = PLIST_SLOT
#ifndef KCC_NODE_PREP_GRID
#define KCC_NODE_PREP_GRID 2048  // workgroups at most (each fills its LDS search tables once)
#endif
__global__ __launch_bounds__(KCC_NODE_PREP_BLOCK) void node_prep_kernel(int64_t n, const uint64_t* __restrict__ alloc_cpu,
                                 const int64_t* __restrict__ alloc_mem,
                                 const int64_t* __restrict__ alloc_pods,
                                 const int64_t* __restrict__ pod_count,
                                 const uint64_t* __restrict__ used_cpu,
                                 const int64_t* __restrict__ used_mem,
                                 FitGroupA* __restrict__ fast_a, FitGroup* __restrict__ fast_b,
                                 SlowNode* __restrict__ slow, int64_t* __restrict__ slow_list,
                                 ClampWork cw, unsigned long long* __restrict__ counters,
                                 int32_t chunk) {
  const int lane = threadIdx.x & 63;
  const int64_t n_pad = fit_groups(n) * FIT_GROUP;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool want_b = counters[CNT_SPECS_B] != 0;  // written by spec_prep (same stream)
  const int64_t nN = clamp_n_normal(counters);     // normal specs (clamp correction)
  const int64_t T = (nN + 63) / 64, hw = nN + 1;
  // this workgroup's copy of H: workgroups are dealt round-robin over the 8 XCDs
  int64_t* Hc = cw.H + (int64_t)(blockIdx.x % H_COPIES) * cw.h_stride;
  // the sorted spec requests of the binary searches, in LDS when they fit: c clamped
  // to 2^23 (> every U = fc / P, fc < 2^23) as u32, m as i64
  extern __shared__ __attribute__((aligned(16))) unsigned char np_lds[];
  int64_t* ms_l = reinterpret_cast<int64_t*>(np_lds);
  uint32_t* cs_l = reinterpret_cast<uint32_t*>(np_lds + 8 * CLAMP_LDS_SPECS);
  const bool lds = nN <= CLAMP_LDS_SPECS;
  // smallest normal requests (rows below either dominate no spec); cs[0] >= 1
  const uint32_t cmin = nN > 0 ? (cw.cs[0] < FAST_FC_MAX ? (uint32_t)cw.cs[0] : (uint32_t)FAST_FC_MAX)
                               : 0xffffffffu;
  const int64_t mmin = nN > 0 ? cw.ms[0] : INT64_MAX;
#ifndef KCC_DIAG_NO_FILL  // diagnostic timing build only: results are wrong
  if (lds) {
#else
  if (false) {
#endif
    for (int64_t k = threadIdx.x; k < CLAMP_LDS_SPECS; k += blockDim.x) {  // padded: +inf
      const uint64_t c = k < nN ? cw.cs[k] : ~0ull;
      cs_l[k] = c < FAST_FC_MAX ? (uint32_t)c : 0xffffffffu;
      ms_l[k] = k < nN ? cw.ms[k] : INT64_MAX;
    }
  }
  __syncthreads();
  __shared__ unsigned long long wcount[16];
  static_assert(KCC_NODE_PREP_BLOCK == PLIST_SLOT, "one plist slot per workgroup iteration");
  const int wv = threadIdx.x >> 6;
  // block-uniform trip count (the plist append below synchronises the workgroup)
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n_pad; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    const bool valid = i < n;
    bool ok = false;
    uint64_t fc_ok = 0;
    int64_t fm_ok = 0, P_ok = 0;
    int32_t cl_i = 0;
    if (valid) {
      const uint64_t ac = alloc_cpu[i], uc = used_cpu[i];
      const int64_t am = alloc_mem[i], um = used_mem[i];
      const int64_t P = alloc_pods[i], pc = pod_count[i];
      const uint64_t fc = ac > uc ? ac - uc : 0;                                  // CC:119-123
      const int64_t fm = am > um ? (int64_t)((uint64_t)am - (uint64_t)um) : 0;   // CC:125-129
      const int64_t cl = (int64_t)((uint64_t)P - (uint64_t)pc);                  // CC:135
      ok = fc < FAST_FC_MAX && fm >= 0 && fm < FAST_FM_MAX && P >= -FAST_P_ABS &&
           P <= FAST_P_ABS && cl >= -FAST_CL_ABS && cl <= FAST_CL_ABS;
      if (ok) {
        fc_ok = fc;
        fm_ok = fm;
        P_ok = P;
        cl_i = (int32_t)cl;
      }
      SlowNode sn;
      sn.fc = fc;
      sn.fm = fm;
      sn.P = P;
      sn.cl = cl;
      slow[i] = sn;
    }
    if (i < n_pad) {
      const int k = (int)(i % FIT_GROUP);
      FitGroupA& a = fast_a[i / FIT_GROUP];
      a.fm[k] = (uint64_t)fm_ok;
      a.fc[k] = (uint32_t)fc_ok;
      a.P[k] = (uint32_t)(P_ok > 0 ? P_ok : 0);  // P <= 0: x >= P always (clamp), as for P = 0
      if (want_b) {
        FitGroup& g = fast_b[i / FIT_GROUP];
        g.fc[k] = (double)fc_ok;                                         // exact
        g.fm[k] = (double)fm_ok;                                         // exact (< 2^50)
        g.Pb[k] = FIT_BIAS + (double)(P_ok > 0 ? P_ok : 0);              // exact (P <= 2^20)
      }
    }
    // clamp correction: where (and with which weight) this row's pod-slot clamp applies
    bool always = false, in_plist = false;
    int64_t w = 0;
    uint32_t key = 0, bnd = 0;
    if (ok && nN > 0) {
      const int64_t P = P_ok, Penc = P > 0 ? P : 0;
      w = Penc - (int64_t)cl_i;  // contribution = min(x, Penc) - w when clamped
      if (P <= 0) {
        always = true;  // x >= P for every spec
      } else {
        // c <= U  <=>  floor(fc / c) >= P  and  m <= V  <=>  floor(fm / m) >= P, with
        // U = floor(fc / P), V = floor(fm / P) from the rounded-up reciprocal of P
        // (exact: fc, fm < 2^50, P < 2^51)
        const double rP = recip_up_f64((uint64_t)P);
        const uint32_t U = (uint32_t)((double)fc_ok * rP);
        const int64_t V = (int64_t)((double)fm_ok * rP);
        uint32_t L = 0, b = 0;
        if (U >= cmin && V >= mmin) {  // else no spec is dominated
#ifdef KCC_DIAG_NO_SEARCH  // diagnostic timing build only: results are wrong
          L = U % (uint32_t)(nN + 1);
          b = (uint32_t)(V % (nN + 1));
#else
          if (lds) {  // 8-ary searches over the +inf-padded 4096-entry tables: 4 steps of
                      // 7 independent LDS reads each (a binary search chains 12)
            L = search8_4096(cs_l, U);
            b = search8_4096(ms_l, V);
          } else {
            L = upper_bound_count(cw.cs, nN, (uint64_t)U);
            b = upper_bound_count(cw.ms, nN, V);
          }
#endif
        }
        if (L > 0 && b > 0 && w != 0) {
          const uint32_t G = L >> 6, r = L & 63u;
#ifndef KCC_DIAG_NO_H_ATOMIC  // diagnostic timing build only: results are wrong
          if (G > 0) atomic_add_u64(reinterpret_cast<uint64_t*>(&Hc[G * hw + b]), (uint64_t)w);
#endif
          in_plist = r != 0;
          key = G << 6 | r;
          bnd = b;
        }
      }
    }
    {  // rows clamped for every spec: one wave-summed atomic into H[T][nN]
      uint64_t v = always ? (uint64_t)w : 0ull;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
      if (lane == 0 && v) atomic_add_u64(reinterpret_cast<uint64_t*>(&Hc[T * hw + nN]), v);
    }
#ifdef KCC_DIAG_NO_PLIST  // diagnostic timing build only: results are wrong
    in_plist = false;
#endif
    {  // plist: this workgroup's rows own slot i0 / PLIST_SLOT (no shared counter)
      const unsigned long long pm = __ballot(in_plist);
      if (lane == 0) wcount[wv] = __popcll(pm);
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += wcount[k];
        cw.pcount[i0 / PLIST_SLOT] = (uint32_t)tot;
      }
      if (in_plist) {
        int64_t j = i0;  // the slot's first entry (i0 is a multiple of PLIST_SLOT)
        for (int k = 0; k < wv; ++k) j += (int64_t)wcount[k];
        j += __popcll(pm & ((1ull << lane) - 1ull));
        cw.pkey[j] = key;
        cw.pb[j] = bnd;
        cw.pw[j] = (int32_t)w;
      }
      __syncthreads();  // wcount is reused by the next iteration
    }
    const unsigned long long b = __ballot(valid && !ok);
    if (b) {
      unsigned long long base = 0;
      if (lane == 0)
        base = atomicAdd(&counters[CNT_SLOW_ROWS + chunk], (unsigned long long)__popcll(b));
      base = __shfl(base, 0);
      if (valid && !ok) slow_list[base + __popcll(b & ((1ull << lane) - 1ull))] = i;
    }
  }
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

// Single-workgroup stable 3-way partition of the specs (class A, then B, then the
// exact-path specs), in two passes over contiguous per-thread chunks with one
// block-wide exclusive scan of the per-class counts in between.  Also zeroes
// partial[0..2S) and sets the counters (no memset launches).
__global__ __launch_bounds__(1024) void spec_prep_kernel(int64_t S, const uint64_t* __restrict__ c_in,
                                                         const int64_t* __restrict__ m_in,
                                                         SpecPrep sp, ClampWork cw,
                                                         int64_t* __restrict__ partial,
                                                         unsigned long long* __restrict__ counters) {
  __shared__ int64_t wsum[16][2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t per = (S + 1023) / 1024;
  const int64_t b0 = tid * per < S ? tid * per : S;
  const int64_t b1 = b0 + per < S ? b0 + per : S;
  // up to 8 specs per thread (S <= 8192) stay in registers: all loads issue at once
  constexpr int REG = 8;
  const bool in_regs = per <= REG;
  uint64_t rc_[REG];
  int64_t rm_[REG];
  if (in_regs) {
#pragma unroll
    for (int u = 0; u < REG; ++u) {
      const bool v = b0 + u < b1;
      rc_[u] = v ? c_in[b0 + u] : 0;
      rm_[u] = v ? m_in[b0 + u] : 0;
    }
  }
  auto spec_c = [&](int64_t i) -> uint64_t {
    if (in_regs) {
      uint64_t r = 0;
#pragma unroll
      for (int u = 0; u < REG; ++u) r = (i - b0 == u) ? rc_[u] : r;  // static indices only
      return r;
    }
    return c_in[i];
  };
  auto spec_m = [&](int64_t i) -> int64_t {
    if (in_regs) {
      int64_t r = 0;
#pragma unroll
      for (int u = 0; u < REG; ++u) r = (i - b0 == u) ? rm_[u] : r;
      return r;
    }
    return m_in[i];
  };
  int64_t cnt[2] = {0, 0};  // class A, class B
  for (int64_t i = b0; i < b1; ++i) {
    const int32_t k = spec_class(spec_c(i), spec_m(i));
    cnt[0] += k == SPEC_A ? 1 : 0;
    cnt[1] += k == SPEC_B ? 1 : 0;
  }
  // block exclusive scans of both counts (wave shuffles + 16 wave totals in LDS)
  int64_t incl[2] = {cnt[0], cnt[1]};
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t u = __shfl_up(incl[q], d);
      if (lane >= d) incl[q] += u;
    }
  }
  if (lane == 63) {
    wsum[wv][0] = incl[0];
    wsum[wv][1] = incl[1];
  }
  __syncthreads();
  int64_t wbase[2] = {0, 0}, tot[2] = {0, 0};
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (k < wv) wbase[q] += wsum[k][q];
      tot[q] += wsum[k][q];
    }
  }
  const int64_t ea = wbase[0] + incl[0] - cnt[0], eb = wbase[1] + incl[1] - cnt[1];
  int64_t pa = ea;                         // my first class-A slot
  int64_t pb = tot[0] + eb;                // my first class-B slot
  int64_t px = tot[0] + tot[1] + (b0 - ea - eb);  // my first exact-path slot
  for (int64_t i = b0; i < b1; ++i) {
    const uint64_t c = spec_c(i);
    const int64_t m = spec_m(i);
    const int32_t k = spec_class(c, m);
    const int64_t pos = k == SPEC_A ? pa++ : (k == SPEC_B ? pb++ : px++);
    SpecRec r;
    r.c = c;
    r.m = m;
    r.rc = k != SPEC_EXACT ? recip_up_f64(c) : 0.0;
    r.rm = k != SPEC_EXACT ? recip_up_f64((uint64_t)m) : 0.0;
    r.rcf = k == SPEC_A ? recip_up_f32(c) : 0.0f;
    r.cls = k;
    r.pad = 0;
    sp.rec[pos] = r;
    sp.perm[pos] = (int32_t)i;
  }
  for (int64_t i = tid; i < 2 * S; i += 1024) partial[i] = 0;
  for (int64_t i = tid; i < 3 * S; i += 1024) cw.rank[i] = 0;
  if (tid < CNT_N)
    counters[tid] = tid == CNT_SPECS_A ? (unsigned long long)tot[0]
                  : tid == CNT_SPECS_B ? (unsigned long long)tot[1] : 0ull;
}

// ---- clamp correction (see ClampWork in kcc_internal.h) ----------

// Ranks of the normal specs (internal positions [0, nN)) among themselves, by brute
// force over a 2-D grid of 256 x CLAMP_RANK_TILE tiles (exact, order-free atomics):
//   c-rank(p) = #{q : (c_q, q) < (c_p, p)},  m-rank(p) = #{q : (m_q, q) < (m_p, p)},
//   m-less(p) = #{q : m_q < m_p}
constexpr int CLAMP_RANK_TILE = 64;
__global__ __launch_bounds__(256) void clamp_rank_kernel(const SpecRec* __restrict__ rec,
                                                         ClampWork cw, int64_t S,
                                                         const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t p0 = (int64_t)blockIdx.x * 256, q0 = (int64_t)blockIdx.y * CLAMP_RANK_TILE;
  if (p0 >= nN || q0 >= nN) return;  // whole block
  __shared__ uint64_t cq[CLAMP_RANK_TILE];
  __shared__ int64_t mq[CLAMP_RANK_TILE];
  const int t = threadIdx.x;
  if (t < CLAMP_RANK_TILE) {
    const int64_t q = q0 + t;
    cq[t] = q < nN ? rec[q].c : ~0ull;
    mq[t] = q < nN ? rec[q].m : INT64_MAX;
  }
  __syncthreads();
  const int64_t p = p0 + t;
  if (p >= nN) return;
  const uint64_t c = rec[p].c;
  const int64_t m = rec[p].m;
  const int qn = (int)(nN - q0 < CLAMP_RANK_TILE ? nN - q0 : CLAMP_RANK_TILE);
  uint32_t rc = 0, rm = 0, ml = 0;
  for (int j = 0; j < qn; ++j) {
    const bool before = q0 + j < p;
    rc += (cq[j] < c || (cq[j] == c && before)) ? 1u : 0u;
    rm += (mq[j] < m || (mq[j] == m && before)) ? 1u : 0u;
    ml += mq[j] < m ? 1u : 0u;
  }
  if (rc) atomicAdd(&cw.rank[p], rc);
  if (rm) atomicAdd(&cw.rank[S + p], rm);
  if (ml) atomicAdd(&cw.rank[2 * S + p], ml);
}

// Sorted arrays from the ranks; zero the used part of H.
__global__ void clamp_scatter_kernel(const SpecRec* __restrict__ rec, ClampWork cw, int64_t S,
                                     const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t T = (nN + 63) / 64;
  const int64_t cells = (T + 1) * (nN + 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells || i < nN; i += stride) {
    if (i < cells) {
#pragma unroll
      for (int k = 1; k < H_COPIES; ++k) cw.H[k * cw.h_stride + i] = 0;
    }
    if (i < nN) {
      const uint32_t d = cw.rank[i];
      cw.cs[d] = rec[i].c;
      cw.dperm[d] = (int32_t)i;
      cw.m_less[d] = cw.rank[2 * S + i];
      cw.ms[cw.rank[S + i]] = rec[i].m;
    }
    if (i < cells) cw.H[i] = 0;
  }
}

// 2-D suffix sums of H, step 0: the XCD copies summed into copy 0 (all cells in parallel)
__global__ void clamp_hsum_kernel(ClampWork cw, const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t cells = ((nN + 63) / 64 + 1) * (nN + 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += stride) {
    uint64_t v = 0;
#pragma unroll
    for (int c = 0; c < H_COPIES; ++c) v += (uint64_t)cw.H[c * cw.h_stride + i];
    cw.H[i] = (int64_t)v;
  }
}

// step 1: down each column (G from T to 0), one thread per column, eight rows' loads
// in flight at a time
__global__ __launch_bounds__(64) void clamp_hcol_kernel(ClampWork cw,
                                                        const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (nN == 0 || b > nN) return;
  const int64_t T = (nN + 63) / 64, w = nN + 1;
  uint64_t run = 0;
  for (int64_t G0 = T; G0 >= 0; G0 -= 8) {
    uint64_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = G0 - k >= 0 ? (uint64_t)cw.H[(G0 - k) * w + b] : 0ull;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      run += v[k];
      if (G0 - k >= 0) cw.H[(G0 - k) * w + b] = (int64_t)run;
    }
  }
}

// step 2: along each row (b from nN to 0), one 1024-thread workgroup per row, in tiles
// of 1024 from the end (wave suffix scans + a carry)
__global__ __launch_bounds__(1024) void clamp_hrow_kernel(ClampWork cw,
                                                          const unsigned long long* __restrict__ counters) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t G = blockIdx.x;
  const int64_t T = (nN + 63) / 64;
  if (nN == 0 || G > T) return;  // whole block
  __shared__ uint64_t wtot[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t w = nN + 1;
  int64_t* row = cw.H + G * w;
  uint64_t carry = 0;
  for (int64_t end = w; end > 0; end -= 1024) {
    const int64_t i = end - 1 - tid;  // thread tid walks the row backwards
    uint64_t v = i >= 0 ? (uint64_t)row[i] : 0ull;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // inclusive scan in thread order = suffix in b
      const uint64_t u = __shfl_up(v, d);
      if (lane >= d) v += u;
    }
    if (lane == 63) wtot[wv] = v;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < wv) before += wtot[k];
      all += wtot[k];
    }
    if (i >= 0) row[i] = (int64_t)(v + before + carry);
    carry += all;
    __syncthreads();
  }
}

// D_partial: every plist entry (G, r, b, w) adds w to the specs with c-rank 64G + lane,
// lane < r, and m_less < b.  CLAMP_PARTIAL_WGS workgroups share the entries; each
// accumulates ALL nN specs in LDS (ds_add_u64; one entry per wave-iteration, lanes =
// the entry's group) and writes its row of dpart[CLAMP_PARTIAL_WGS][nN]; clamp_full
// sums the rows.  nN <= CLAMP_LDS_SPECS (else clamp_partial_big_kernel).
constexpr int CLAMP_PARTIAL_WGS = (int)CLAMP_PARTIAL_ROWS;
constexpr int CLAMP_PARTIAL_MAX_SLOTS = 1024;  // per workgroup (n_nodes <= 256 x 1024 x 1024)
static_assert(CLAMP_PARTIAL_WGS % 64 == 0, "clamp_full sums the rows in 8 splits, 8 at a time");
__global__ __launch_bounds__(1024) void clamp_partial_kernel(ClampWork cw,
                                                             const unsigned long long* __restrict__ counters,
                                                             int64_t n_nodes, int64_t* __restrict__ dpart) {
  const int64_t nN = clamp_n_normal(counters);
  if (nN == 0 || nN > CLAMP_LDS_SPECS) return;
  __shared__ uint32_t ml_l[CLAMP_LDS_SPECS];
  __shared__ unsigned long long acc_l[CLAMP_LDS_SPECS];
  for (int64_t q = threadIdx.x; q < nN; q += blockDim.x) {
    ml_l[q] = cw.m_less[q];
    acc_l[q] = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int32_t wv = __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));
  const int32_t nw = (int32_t)(blockDim.x >> 6);
  // this workgroup's plist slots [s0, s1), their entries taken as one sequence in
  // 64-entry batches by the workgroup's waves (slot counts prefix-summed in LDS)
  __shared__ uint32_t spre[CLAMP_PARTIAL_MAX_SLOTS + 1];
  const int64_t n_slots = (n_nodes + PLIST_SLOT - 1) / PLIST_SLOT;
  const int64_t s0 = n_slots * blockIdx.x / CLAMP_PARTIAL_WGS, s1 = n_slots * (blockIdx.x + 1) / CLAMP_PARTIAL_WGS;
  const int ns = (int)(s1 - s0);  // <= CLAMP_PARTIAL_MAX_SLOTS (host-checked)
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int k = 0; k < ns; ++k) {
      spre[k] = run;
      run += cw.pcount[s0 + k];
    }
    spre[ns] = run;
  }
  __syncthreads();
  const int64_t n_ent = spre[ns];
  for (int64_t e0 = (int64_t)wv * 64; e0 < n_ent; e0 += (int64_t)nw * 64) {
    const int64_t e = e0 + lane;
    int k = 0;  // slot of entry e (lanes of one batch span at most a few slots)
    while (k + 1 < ns && (int64_t)spre[k + 1] <= e) ++k;
    const bool in = e < n_ent;
    const int64_t j = (s0 + k) * PLIST_SLOT + (e - (int64_t)spre[k]);
    const uint32_t key_v = in ? cw.pkey[j] : 0u, bnd_v = in ? cw.pb[j] : 0u;
    const int32_t w_v = in ? cw.pw[j] : 0;
    const int cnt = (int)(n_ent - e0 < 64 ? n_ent - e0 : 64);
    // 64 entries by one coalesced load each, walked lane by lane from registers
    for (int kk = 0; kk < cnt; ++kk) {
      const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)key_v, kk);
      const uint32_t bnd = (uint32_t)__builtin_amdgcn_readlane((int)bnd_v, kk);
      const int32_t w = __builtin_amdgcn_readlane(w_v, kk);
      const int64_t q = (int64_t)(key >> 6) * 64 + lane;
      if ((uint32_t)lane < (key & 63u) && ml_l[q] < bnd)
        atomicAdd(&acc_l[q], (unsigned long long)(int64_t)w);
    }
  }
  __syncthreads();
  for (int64_t q = threadIdx.x; q < nN; q += blockDim.x)
    dpart[(int64_t)blockIdx.x * nN + q] = (int64_t)acc_l[q];
}

// the same for nN > CLAMP_LDS_SPECS: one wavefront per (group, slice of the plist),
// lanes = the group's 64 c-ranks; scans the 4-B keys, reads b / w only for matches,
// and subtracts straight from partial
constexpr int CLAMP_SLICES = 512;
__global__ __launch_bounds__(64) void clamp_partial_big_kernel(ClampWork cw,
                                                               const unsigned long long* __restrict__ counters,
                                                               int64_t S, int64_t n_nodes,
                                                               int64_t* __restrict__ partial) {
  const int64_t nN = clamp_n_normal(counters);
  if (nN <= CLAMP_LDS_SPECS) return;
  const int64_t T = (nN + 63) / 64;
  const int64_t g = blockIdx.x;
  if (g >= T) return;
  const int lane = threadIdx.x;
  const int64_t q = g * 64 + lane;
  const bool valid = q < nN;
  const uint32_t ml = valid ? cw.m_less[q] : 0xffffffffu;
  const int64_t n_slots = (n_nodes + PLIST_SLOT - 1) / PLIST_SLOT;
  const int64_t s0 = n_slots * blockIdx.y / CLAMP_SLICES, s1 = n_slots * (blockIdx.y + 1) / CLAMP_SLICES;
  uint64_t acc = 0;
  for (int64_t sl = s0; sl < s1; ++sl) {
    const int64_t j1 = sl * PLIST_SLOT + (int64_t)cw.pcount[sl];
    for (int64_t jb = sl * PLIST_SLOT; jb < j1; jb += 64) {
      const int64_t j = jb + lane;
      const uint32_t key = j < j1 ? cw.pkey[j] : 0xffffffffu;
      uint64_t mask = __ballot((int64_t)(key >> 6) == g);
      while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)key, k) & 63u;
        const int64_t jj = jb + k;
        const uint32_t bnd = cw.pb[jj];
        const int32_t w = cw.pw[jj];
        acc += ((uint32_t)lane < r && ml < bnd) ? (uint64_t)(int64_t)w : 0ull;
      }
    }
  }
  if (valid && acc) {
    const int32_t p = cw.dperm[q];
    if (p < clamp_n_pure(nN, S)) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[p]), 0ull - acc);
  }
}

// partial[p] -= D(p) = HS[g + 1][m_less + 1] + Σ_k dpart[k][q] for the normal specs of
// clamp-free waves (q = the spec's c-rank, g = q / 64).  Grid (nN / 64, CLAMP_FULL_SPLIT):
// split y sums dpart rows [y * R, (y + 1) * R), split 0 also the H term; one atomic each.
constexpr int CLAMP_FULL_SPLIT = 8;
__global__ __launch_bounds__(64) void clamp_full_kernel(ClampWork cw,
                                                        const unsigned long long* __restrict__ counters,
                                                        int64_t S, const int64_t* __restrict__ dpart,
                                                        int64_t* __restrict__ partial) {
  const int64_t nN = clamp_n_normal(counters);
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // c-rank
  if (q >= nN) return;
  const int32_t p = cw.dperm[q];
  if (p >= clamp_n_pure(nN, S)) return;
  uint64_t d = 0;
  if (blockIdx.y == 0) {
    const int64_t T = (nN + 63) / 64, w = nN + 1;
    const int64_t g1 = (q >> 6) + 1, b1 = (int64_t)cw.m_less[q] + 1;
    if (g1 <= T && b1 <= nN) d = (uint64_t)cw.H[g1 * w + b1];
  }
  if (nN <= CLAMP_LDS_SPECS) {  // the partial kernel's per-workgroup rows, 8 loads in flight
    constexpr int R = CLAMP_PARTIAL_WGS / CLAMP_FULL_SPLIT;
    uint64_t part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = (int)blockIdx.y * R; k < ((int)blockIdx.y + 1) * R; k += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) part[u] += (uint64_t)dpart[(int64_t)(k + u) * nN + q];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) d += part[u];
  }
  if (d) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[p]), 0ull - d);
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

#ifndef KCC_FIT_SPECS_PER_WG
#define KCC_FIT_SPECS_PER_WG 256  // 64/128 (waves split the node chunk, LDS-reduced atomics) measured slower
#endif
constexpr int FIT_SPW = KCC_FIT_SPECS_PER_WG;  // specs per 256-thread workgroup (64 or 256)
constexpr int FIT_SPLIT = 256 / FIT_SPW;       // waves per spec group (node chunk split)
static_assert(FIT_SPW == 64 || FIT_SPW == 128 || FIT_SPW == 256, "FIT_SPW");
constexpr int FIT_CHUNK_GROUPS = 128;  // 1024 nodes: |sum of contributions| <= 2^30 in i32
#ifndef KCC_FIT_TARGET_BLOCKS
#define KCC_FIT_TARGET_BLOCKS 32768
#endif

__device__ __forceinline__ double f64_at(const i32x16& v, int k) {
  return __longlong_as_double(((int64_t)(uint32_t)v[2 * k + 1] << 32) | (uint32_t)v[2 * k]);
}

__global__ __launch_bounds__(256) void fit_kernel(
    int64_t n_nodes, int64_t groups_per_block, const FitGroupA* __restrict__ fast_a,
    const FitGroup* __restrict__ fast_b, const SlowNode* __restrict__ slow,
    const int64_t* __restrict__ slow_list, int64_t S, const SpecRec* __restrict__ specs,
    int64_t* __restrict__ partial, unsigned long long* __restrict__ counters, int32_t chunk,
    int32_t gx, int32_t gy) {
  // XCD-aware order (speed only, never correctness): workgroups are dealt round-robin
  // over the 8 XCDs, so give every spec group of one node chunk the same b % 8 — the
  // chunk's FitGroup records then stay in that XCD's L2 for all of them.
  const int32_t b = blockIdx.x, xcd = b & 7, r = b >> 3;
  const int32_t bx = r % gx, by = (r / gx) * 8 + xcd;
  if (by >= gy) return;  // padding of gy up to a multiple of 8 (whole workgroup)
  // FIT_SPW specs per workgroup; its FIT_SPLIT waves share them and split the node chunk
  const int32_t wv = __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6) / (FIT_SPW / 64));
  const int64_t s = (int64_t)bx * FIT_SPW + (threadIdx.x % FIT_SPW);
  const bool active = s < S;
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

  const int64_t n_groups = fit_groups(n_nodes);
  int64_t g0 = (int64_t)by * groups_per_block;
  int64_t g1 = g0 + groups_per_block < n_groups ? g0 + groups_per_block : n_groups;
  if (FIT_SPLIT > 1) {  // this wave's part of the workgroup's node chunk
    const int64_t part = (g1 - g0 + FIT_SPLIT - 1) / FIT_SPLIT;
    g0 = g0 + wv * part < g1 ? g0 + wv * part : g1;
    g1 = g0 + part < g1 ? g0 + part : g1;
  }
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

  const int cnt = (int)(g1 - g0);
  if (!wave_exact && !wave_b) {
    // class A
    const FitGroupA* gbase = fast_a + g0;
    const f32x2 rcf2 = {sr.rcf, sr.rcf};
    set_round_down();
    for (int cb = 0; cb < cnt; cb += FIT_CHUNK_GROUPS) {
      const int ce = cb + FIT_CHUNK_GROUPS < cnt ? cb + FIT_CHUNK_GROUPS : cnt;
      int32_t acc32 = 0;
      for (int gi = cb; gi < ce; ++gi) {
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
      }
      acc += (uint64_t)(int64_t)acc32;
    }
    set_round_nearest();
  } else if (!wave_exact) {
    // class B (and class-A lanes sharing its wave)
    const FitGroup* gbase = fast_b + g0;
    const double bias = FIT_BIAS;
    set_round_down();
    for (int cb = 0; cb < cnt; cb += FIT_CHUNK_GROUPS) {
      const int ce = cb + FIT_CHUNK_GROUPS < cnt ? cb + FIT_CHUNK_GROUPS : cnt;
      int32_t acc32 = 0;
      for (int gi = cb; gi < ce; ++gi) {
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
      acc += (uint64_t)(int64_t)acc32;
    }
    set_round_nearest();
  } else {
    const int64_t i1 = g1 * FIT_GROUP < n_nodes ? g1 * FIT_GROUP : n_nodes;
    for (int64_t i = g0 * FIT_GROUP; i < i1; ++i) eval_slow(i);
  }
  if (!wave_exact) {  // rows outside the fast bounds, shared out over the node-chunk waves
    const int64_t n_slow = (int64_t)counters[CNT_SLOW_ROWS + chunk];
    for (int64_t j = (int64_t)by * FIT_SPLIT + wv; j < n_slow; j += (int64_t)gy * FIT_SPLIT)
      eval_slow(slow_list[j]);
  }

  {  // (node, spec) pairs evaluated on the exact path (statistics)
    const unsigned long long act = __ballot(active);
    if (slow_iters && (threadIdx.x & 63) == 0)
      atomicAdd(&counters[CNT_SLOW_PAIRS], (unsigned long long)slow_iters * (unsigned long long)__popcll(act));
  }
  if (FIT_SPLIT > 1) {  // the waves of one spec group meet in LDS: one atomic per spec
    __shared__ uint64_t red_s[2][FIT_SPLIT][FIT_SPW];
    red_s[0][wv][threadIdx.x % FIT_SPW] = acc;
    red_s[1][wv][threadIdx.x % FIT_SPW] = errs;
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int k = 1; k < FIT_SPLIT; ++k) {
      acc += red_s[0][k][threadIdx.x];
      errs += red_s[1][k][threadIdx.x];
    }
  }
#ifdef KCC_FIT_DIAG_NO_ATOMICS  // diagnostic timing build only: results are wrong
  if (active && acc == 0x5A5A5A5A5A5A5A5Aull) partial[s] = (int64_t)acc;
#else
  if (active) {
    atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[s]), acc);
    if (errs) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[S + s]), errs);
  }
#endif
}

__global__ void fit_finalize_kernel(int64_t S, const int64_t* __restrict__ partial,
                                    const int32_t* __restrict__ perm, int64_t* __restrict__ totals,
                                    int32_t* __restrict__ spec_err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  const int32_t dst = perm[i];
  const bool err = partial[S + i] != 0;
  totals[dst] = err ? 0 : partial[i];
  spec_err[dst] = err ? 1 : 0;
}

inline unsigned grid_for(int64_t n, int block, int64_t cap) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace

namespace {
int64_t reduce_resident_waves(bool limits) {
  static int64_t cache[2] = {0, 0};
  int64_t& w = cache[limits ? 1 : 0];
  if (w == 0) {
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, limits ? reduce_kernel<4> : reduce_kernel<2>, 256, 0) == hipSuccess &&
        cus > 0 && blocks > 0)
      w = (int64_t)cus * blocks * RED_WAVES_PER_BLOCK;
    else
      w = 8192;
  }
  return w;
}
}  // namespace

int32_t reduce_range(int64_t n_containers, bool limits) {
  const int64_t r = reduce_resident_waves(limits) * KCC_RED_ROUNDS * RED_TILE;
  int64_t t = (n_containers + r - 1) / r;
  if (t < 1) t = 1;
  if (t > ((int64_t)1 << 20)) t = (int64_t)1 << 20;  // range < 2^28 (int32 relative offsets)
  return (int32_t)(t * RED_TILE);
}

hipError_t launch_reduce_mark(int64_t n_nodes, int64_t c0, int64_t n_containers,
                              const int64_t* node_ptr, int64_t* wave_node, uint64_t* used_cpu,
                              int64_t* used_mem, uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s) {
  if (n_nodes <= 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_mark_kernel, dim3(grid_for(n_nodes, 256, 8192)), dim3(256), 0, s,
                     n_nodes, c0, c0 + n_containers, reduce_range(n_containers, lim_cpu != nullptr),
                     node_ptr, wave_node,
                     used_cpu,
                     reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                     reinterpret_cast<uint64_t*>(lim_mem));
  return hipGetLastError();
}

hipError_t launch_reduce(int64_t n_nodes, int64_t c0, int64_t n_containers, const int64_t* node_ptr,
                         const uint64_t* cpu_req, const int64_t* mem_req,
                         const uint64_t* cpu_lim, const int64_t* mem_lim,
                         const int64_t* wave_node, uint64_t* used_cpu, int64_t* used_mem,
                         uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s) {
  if (n_nodes <= 0 || n_containers <= 0) return hipSuccess;
  if (n_nodes >= RED_MAX_NODES) return hipErrorInvalidValue;
  const bool limits = cpu_lim && mem_lim && lim_cpu && lim_mem;
  const int32_t range = reduce_range(n_containers, limits);
  const int64_t waves = reduce_n_waves(n_containers, limits);
  const unsigned blocks = (unsigned)((waves + RED_WAVES_PER_BLOCK - 1) / RED_WAVES_PER_BLOCK);
  const bool lim = cpu_lim && mem_lim && lim_cpu && lim_mem;
  if (lim) {
    hipLaunchKernelGGL(reduce_kernel<4>, dim3(blocks), dim3(256), 0, s, n_nodes, c0,
                       c0 + n_containers, range, node_ptr, cpu_req, reinterpret_cast<const uint64_t*>(mem_req), cpu_lim,
                       reinterpret_cast<const uint64_t*>(mem_lim), wave_node, used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                       reinterpret_cast<uint64_t*>(lim_mem));
  } else {
    hipLaunchKernelGGL(reduce_kernel<2>, dim3(blocks), dim3(256), 0, s, n_nodes, c0,
                       c0 + n_containers, range, node_ptr, cpu_req, reinterpret_cast<const uint64_t*>(mem_req),
                       (const uint64_t*)nullptr, (const uint64_t*)nullptr, wave_node, used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), (uint64_t*)nullptr,
                       (uint64_t*)nullptr);
  }
  return hipGetLastError();
}

hipError_t launch_node_prep(int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, FitGroupA* fast_a, FitGroup* fast_b,
                            SlowNode* slow, int64_t* slow_list, ClampWork cw,
                            unsigned long long* counters, int chunk, hipStream_t s) {
  if (n_nodes <= 0) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel,
                     dim3(grid_for(fit_groups(n_nodes) * FIT_GROUP, KCC_NODE_PREP_BLOCK,
                                   KCC_NODE_PREP_GRID)),
                     dim3(KCC_NODE_PREP_BLOCK), (size_t)(12 * CLAMP_LDS_SPECS), s,
                     n_nodes, alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
                     fast_a, fast_b, slow, slow_list, cw, counters, (int32_t)chunk);
  return hipGetLastError();
}

hipError_t launch_spec_prep(int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
                            SpecPrep sp, ClampWork cw, int64_t* partial,
                            unsigned long long* counters, hipStream_t s) {
  if (n_specs <= 0) return hipSuccess;
  hipLaunchKernelGGL(spec_prep_kernel, dim3(1), dim3(1024), 0, s, n_specs, spec_cpu, spec_mem,
                     sp, cw, partial, counters);
  return hipGetLastError();
}

hipError_t launch_clamp_specs(int64_t n_specs, SpecPrep sp, ClampWork cw,
                              const unsigned long long* counters, hipStream_t s) {
  if (n_specs <= 0) return hipSuccess;
  hipLaunchKernelGGL(clamp_rank_kernel,
                     dim3((unsigned)((n_specs + 255) / 256),
                          (unsigned)((n_specs + CLAMP_RANK_TILE - 1) / CLAMP_RANK_TILE)),
                     dim3(256), 0, s, sp.rec, cw, n_specs, counters);
  hipLaunchKernelGGL(clamp_scatter_kernel, dim3(grid_for(clamp_h_cells(n_specs), 256, 2048)),
                     dim3(256), 0, s, sp.rec, cw, n_specs, counters);
  return hipGetLastError();
}

hipError_t launch_clamp_apply(int64_t n_specs, int64_t n_nodes, ClampWork cw,
                              const unsigned long long* counters, int64_t* partial, hipStream_t s) {
  if (n_specs <= 0 || n_nodes <= 0) return hipSuccess;
  if ((n_nodes + PLIST_SLOT - 1) / PLIST_SLOT > (int64_t)CLAMP_PARTIAL_WGS * CLAMP_PARTIAL_MAX_SLOTS)
    return hipErrorInvalidValue;  // > 2^28 nodes on one device
  const int64_t t_max = (n_specs + 63) / 64;
  hipLaunchKernelGGL(clamp_hsum_kernel, dim3(grid_for(clamp_h_cells(n_specs), 256, 2048)),
                     dim3(256), 0, s, cw, counters);
  hipLaunchKernelGGL(clamp_hcol_kernel, dim3(grid_for(n_specs + 1, 64, 1 << 30)), dim3(64), 0, s,
                     cw, counters);
  hipLaunchKernelGGL(clamp_hrow_kernel, dim3((unsigned)(t_max + 1)), dim3(1024), 0, s, cw,
                     counters);
  if (n_specs <= CLAMP_LDS_SPECS) {
    hipLaunchKernelGGL(clamp_partial_kernel, dim3(CLAMP_PARTIAL_WGS), dim3(1024), 0, s, cw,
                       counters, n_nodes, cw.dpart);
  } else {
    hipLaunchKernelGGL(clamp_partial_big_kernel, dim3((unsigned)t_max, CLAMP_SLICES), dim3(64), 0,
                       s, cw, counters, n_specs, n_nodes, partial);
  }
  hipLaunchKernelGGL(clamp_full_kernel, dim3(grid_for(n_specs, 64, 1 << 30), CLAMP_FULL_SPLIT),
                     dim3(64), 0, s, cw, counters, n_specs, cw.dpart, partial);
  return hipGetLastError();
}

hipError_t launch_fit(int64_t n_nodes, const FitGroupA* fast_a, const FitGroup* fast_b,
                      const SlowNode* slow,
                      const int64_t* slow_list, int64_t n_specs, SpecPrep sp, int64_t* partial,
                      unsigned long long* counters, int chunk, int64_t grid_nodes,
                      hipStream_t s) {
  if (n_nodes <= 0 || n_specs <= 0) return hipSuccess;
  const int64_t gx = (n_specs + FIT_SPW - 1) / FIT_SPW;
  const int64_t n_groups = fit_groups(n_nodes);
  // aim for KCC_FIT_TARGET_BLOCKS workgroups over `grid_nodes` nodes (the whole call's
  // node count: a chunk of a pipelined call gets its share, not a full grid); 2048 =
  // one round at 8 per CU, 16 rounds keep the ragged end of the last round short
  // (measured best of 4k..128k at C4); >= 8 groups (64 nodes) each
  int64_t gy_target = KCC_FIT_TARGET_BLOCKS / gx;
  if (gy_target < 1) gy_target = 1;
  const int64_t grid_groups = fit_groups(grid_nodes > n_nodes ? grid_nodes : n_nodes);
  int64_t gpb = (grid_groups + gy_target - 1) / gy_target;
  if (gpb < 8) gpb = 8;
  int64_t gy = (n_groups + gpb - 1) / gpb;
  // 1-D grid of gx * roundup(gy, 8) workgroups, remapped XCD-aware in the kernel; the
  // buffer descriptor of a block's groups needs gpb * 160 B < 2^31
  while (gx * ((gy + 7) / 8 * 8) > 0x7fffffffLL) {
    gpb *= 2;
    gy = (n_groups + gpb - 1) / gpb;
  }
  if (gpb * (int64_t)sizeof(FitGroup) >= 0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t blocks = gx * ((gy + 7) / 8 * 8);
  hipLaunchKernelGGL(fit_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n_nodes, gpb, fast_a,
                     fast_b, slow, slow_list, n_specs, sp.rec, partial, counters, (int32_t)chunk,
                     (int32_t)gx, (int32_t)gy);
  return hipGetLastError();
}

hipError_t launch_fit_finalize(int64_t n_specs, const int64_t* partial, const int32_t* perm,
                               int64_t* totals, int32_t* spec_err, hipStream_t s) {
  if (n_specs <= 0) return hipSuccess;
  hipLaunchKernelGGL(fit_finalize_kernel, dim3(grid_for(n_specs, 256, 1 << 30)), dim3(256), 0, s,
                     n_specs, partial, perm, totals, spec_err);
  return hipGetLastError();
}

}  // namespace kcc
