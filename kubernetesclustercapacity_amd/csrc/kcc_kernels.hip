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

constexpr int32_t HEAD_END = 0x7fffffff;  // "end of data" head marker

__device__ __forceinline__ unsigned long long atomic_add_u64(uint64_t* p, uint64_t v) {
  return atomicAdd(reinterpret_cast<unsigned long long*>(p),
                   static_cast<unsigned long long>(v));
}

// ----------------------------------------------------------------------------
// (a) segmented reduce
// ----------------------------------------------------------------------------

// Zero the outputs; for every wave range x*range record the node owning it.
__global__ void reduce_mark_kernel(int64_t n_nodes, int64_t n_cont, int32_t range,
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
    int64_t b = ptr[j], e = ptr[j + 1];
    b = b < 0 ? 0 : b;
    e = e > n_cont ? n_cont : e;
    if (e > b) {
      for (int64_t x = (b + range - 1) / range * range; x < e; x += range)
        wave_node[x / range] = j;
    }
  }
}

// DPP controls (gfx9 family): row_shr:n, row_bcast:15/31, wave_shl:1.
constexpr int DPP_ROW_SHR = 0x110;
constexpr int DPP_ROW_BCAST15 = 0x142;
constexpr int DPP_ROW_BCAST31 = 0x143;
constexpr int DPP_WAVE_SHL1 = 0x130;

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

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

// CSR offset of node j relative to the wave range start, clamped into int32.
__device__ __forceinline__ int32_t rel_clamp(int64_t raw, int64_t wb) {
  const int64_t v = raw - wb;  // any range is <= RED_TILE * RED_TILES_PER_WAVE
  constexpr int64_t HI = (int64_t)RED_TILE * RED_TILES_PER_WAVE + 2;
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
__device__ __forceinline__ void load_quad(__amdgpu_buffer_rsrc_t r, int32_t voff, uint64_t (&x)[4]) {
  const u64x2 lo = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
  const u64x2 hi = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, 0, 0));
  x[0] = lo.x;
  x[1] = lo.y;
  x[2] = hi.x;
  x[3] = hi.y;
}

// One wavefront walks a contiguous range of `range` containers in tiles of
// RED_TILE = 256 (4 per lane, coalesced SoA buffer loads, next tile prefetched).
// Per tile:
//   1. nodes starting inside the tile: the next 64 CSR offsets come from a sliding
//      register window (3 x 64 offsets, the third prefetched), gathered with
//      ds_bpermute, and are written as head marks into a per-wave LDS strip;
//   2. per lane a 4-item running sum, then one DPP inclusive prefix sum (64-bit,
//      all VALU) of the lane totals; a run's sum = prefix at its end - prefix
//      before its head, the head prefix coming from the lane that holds the head
//      (one ds_bpermute) or from the carry of the previous tile;
//   3. the lane holding a run's last container stores the node's sum — a plain
//      store when the run started inside this wave's range, an atomic add only
//      for the (at most two) runs crossing the range boundaries.
// Empty nodes are never visited (zeroed by reduce_mark_kernel).
template <int NA>
__global__ __launch_bounds__(256) void reduce_kernel(
    int64_t n_nodes, int64_t n_cont, int32_t range, const int64_t* __restrict__ ptr,
    const uint64_t* __restrict__ in0, const uint64_t* __restrict__ in1,
    const uint64_t* __restrict__ in2, const uint64_t* __restrict__ in3,
    const int64_t* __restrict__ wave_node, uint64_t* __restrict__ out0,
    uint64_t* __restrict__ out1, uint64_t* __restrict__ out2, uint64_t* __restrict__ out3) {
  constexpr int HS = RED_TILE + 4;  // LDS strip per wave (positions 0..RED_TILE)
  __shared__ __attribute__((aligned(16))) int32_t heads_s[RED_WAVES_PER_BLOCK * HS];
  const int lane = threadIdx.x & 63;
  // wave index made provably uniform (T20: no waterfall loops around the buffer ops)
  const int32_t w = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * RED_WAVES_PER_BLOCK +
                                                             (threadIdx.x >> 6)));
  const int64_t wb = (int64_t)w * range;
  if (wb >= n_cont) return;  // wave-uniform; no block-level barrier in this kernel
  const int32_t len = (int32_t)(n_cont - wb < range ? n_cont - wb : range);
  int32_t* heads = heads_s + (threadIdx.x >> 6) * HS;
  const uint64_t* in[4] = {in0, in1, in2, in3};
  uint64_t* out[4] = {out0, out1, out2, out3};
  __amdgpu_buffer_rsrc_t rs[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k)  // whole 16-B pairs only: an odd last item is fixed up below
    rs[k] = __builtin_amdgcn_make_buffer_rsrc((void*)(in[k] + wb), (short)0,
                                              (int)((len & ~1) * 8), 0x00020000);
  const unsigned long long lt_mask = (1ull << lane) - 1ull;

  const int64_t node0 = wave_node[w];
  const bool first_open = ptr[node0] < wb;  // node0's run began in an earlier range
  int64_t cur = node0;                      // node owning the current tile's first item
  uint64_t carry[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) carry[k] = 0;

  // sliding window of CSR offsets: win0/win1 (relative, clamped) hold nodes
  // [wbase, wbase+64), [wbase+64, +128); win2r (raw, still in flight) the next 64
  int64_t wbase = cur + 1;
  int32_t win0 = rel_ptr(ptr, wbase + lane, n_nodes, wb);
  int32_t win1 = rel_ptr(ptr, wbase + 64 + lane, n_nodes, wb);
  int64_t win2r = ptr_at(ptr, wbase + 128 + lane, n_nodes);
  const int32_t end_rel = (int32_t)(n_cont - wb < range + 2 ? n_cont - wb : range + 2);

  // Statically named tile buffers in rotation: the loads for tile t+KCC_RED_PREFETCH
  // are issued unconditionally (range-checked) at the top of tile t, so they stay in
  // flight across whole tiles and no register copy forces an early wait.
  uint64_t xa[NA][4], xb[NA][4];
#if KCC_RED_PREFETCH == 2
  uint64_t xc[NA][4];
#endif
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    load_quad(rs[k], lane * 32, xa[k]);
#if KCC_RED_PREFETCH == 2
    load_quad(rs[k], RED_TILE * 8 + lane * 32, xb[k]);
#endif
  }

  auto tile = [&](uint64_t (&x)[NA][4], uint64_t (&nx)[NA][4], const int32_t tb) {
#pragma unroll
    for (int k = 0; k < NA; ++k)
      load_quad(rs[k], (tb + KCC_RED_PREFETCH * RED_TILE) * 8 + lane * 32, nx[k]);
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

    // --- 1. head marks --------------------------------------------------------
    *reinterpret_cast<int4*>(&heads[4 * lane]) = make_int4(-1, -1, -1, -1);
    if (lane == 0) heads[RED_TILE] = -1;
    const int32_t X = tb + RED_TILE;
    while (cur + 1 - wbase >= 64) {  // slide the window (rarely more than once)
      win0 = win1;
      win1 = rel_clamp(win2r, wb);
      wbase += 64;
      win2r = ptr_at(ptr, wbase + 128 + lane, n_nodes);
    }
    const int off = (int)(cur + 1 - wbase);  // 0..63
    const int idx = off + lane;               // 0..126
    const int32_t g0 = __shfl(win0, idx & 63), g1 = __shfl(win1, idx & 63);
    const int32_t sj = idx < 64 ? g0 : g1;
    int32_t sj1 = __builtin_amdgcn_update_dpp(0, sj, DPP_WAVE_SHL1, 0xf, 0xf, false);
    const int32_t nxt = __shfl(win1, off);  // node cur+65
    if (lane == 63) sj1 = nxt;
    const int64_t j0 = cur + 1 + lane;
    const bool in_range = (j0 < n_nodes) && (sj <= X);
    if (in_range && sj1 > sj && sj > tb && sj < end_rel) heads[sj - tb] = (int32_t)(j0 - cur);
    unsigned long long bal = __ballot(in_range);
    int64_t cnt = __popcll(bal);
    // more than 64 node starts in this tile (runs of tiny or empty nodes): direct loads
    for (int64_t r = 64; (bal >> 63) & 1ull; r += 64) {
      const int64_t j = cur + 1 + r + lane;
      const int32_t s2 = rel_ptr(ptr, j, n_nodes, wb);
      const int32_t s21 = rel_ptr(ptr, j + 1, n_nodes, wb);
      const bool ir = (j < n_nodes) && (s2 <= X);
      if (ir && s21 > s2 && s2 > tb && s2 < end_rel) heads[s2 - tb] = (int32_t)(j - cur);
      bal = __ballot(ir);
      cnt += __popcll(bal);
    }
    if (lane == 0 && end_rel > tb && end_rel <= X) heads[end_rel - tb] = HEAD_END;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    const int4 h4 = *reinterpret_cast<const int4*>(&heads[4 * lane]);
    const int32_t h[5] = {h4.x, h4.y, h4.z, h4.w, heads[4 * lane + 4]};
    bool f[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) f[i] = h[i] >= 0;
    const bool any = f[0] || f[1] || f[2] || f[3];
    const unsigned long long hm = __ballot(any);
    const unsigned long long before = hm & lt_mask;
    const int L = before ? 63 - __clzll(before) : 0;  // last lane before me with a head
    const int32_t lid = f[3] ? h[3] : f[2] ? h[2] : f[1] ? h[1] : h[0];
    // every cross-lane read below runs on all 64 lanes, then selects
    const int32_t got_id = __shfl(lid, L);
    const int32_t prev_id = before ? got_id : 0;
    const bool last_end = (__ballot(f[4]) >> 63) & 1ull;

    // --- 2./3. prefix sums, run sums, emit ---------------------------------------
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      uint64_t q[4];  // running sums within the lane
      q[0] = x[k][0];
#pragma unroll
      for (int i = 1; i < 4; ++i) q[i] = q[i - 1] + x[k][i];
      const uint64_t P = wave_incl_scan_u64(q[3]);
      const uint64_t Pex = P - q[3];
      const uint64_t lhp = Pex + (f[3] ? q[2] : f[2] ? q[1] : f[1] ? q[0] : 0ull);
      const uint64_t got = shfl_u64(lhp, L);
      uint64_t sp = before ? got : (0ull - carry[k]);  // prefix before the open run's head
      int32_t cid = prev_id;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (f[i]) {
          sp = Pex + (i ? q[i - 1] : 0ull);
          cid = h[i];
        }
        if (f[i + 1] && p0 + i < len) {  // run ends at item i
          const int64_t nd = cur + cid;
          const uint64_t tot = Pex + q[i] - sp;
          if (nd < n_nodes) {
            if (nd == node0 && first_open) atomic_add_u64(&out[k][nd], tot);
            else out[k][nd] = tot;
          }
        }
      }
      const uint64_t tail = shfl_u64(P - sp, 63);
      carry[k] = last_end ? 0 : tail;
    }
    cur += cnt;
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
  // the run open at the end of the range continues into the next wave's range
  if (wb + len < n_cont && lane == 0 && cur < n_nodes) {
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if (carry[k] != 0) atomic_add_u64(&out[k][cur], carry[k]);
  }
}

// ----------------------------------------------------------------------------
// (b) fit
// ----------------------------------------------------------------------------

// Fast-path bounds (see DESIGN.md "fit kernel: exactness argument").
constexpr uint64_t FAST_FC_MAX = 1ull << 31;    // free CPU < 2^31
constexpr int64_t FAST_FM_MAX = 1ll << 53;      // 0 <= free mem < 2^53
constexpr int64_t FAST_P_MAX = 1ll << 16;       // allocatable pods <= 2^16
constexpr int64_t FAST_P_MIN = -(1ll << 20);
constexpr int64_t FAST_CL_ABS = 1ll << 20;      // |allocPods - podCount| <= 2^20
constexpr uint64_t FAST_C_MAX = 1ull << 23;     // 1 <= spec cpu < 2^23
constexpr int64_t FAST_M_MAX = 1ll << 37;       // 1 <= spec mem < 2^37
constexpr double FIT_RECIP_BIAS = 1.0 + 0x1p-20;  // see fit_fast

__device__ __forceinline__ bool spec_is_normal(uint64_t c, int64_t m) {
  return c >= 1 && c < FAST_C_MAX && m >= 1 && m < FAST_M_MAX;
}

// Per-node free capacity (CC:119-135 operands).  Rows that fit the fast-path
// bounds get an exact FitNode; the others get a FitNode that contributes exactly 0
// on the fast path and are appended to slow_list for the exact 64-bit path.
// counters[2] holds the largest fast-path spec cpu request (from spec_prep), which
// bounds P so that k*c fits in i32 for every spec.
__global__ void node_prep_kernel(int64_t n, const uint64_t* __restrict__ alloc_cpu,
                                 const int64_t* __restrict__ alloc_mem,
                                 const int64_t* __restrict__ alloc_pods,
                                 const int64_t* __restrict__ pod_count,
                                 const uint64_t* __restrict__ used_cpu,
                                 const int64_t* __restrict__ used_mem,
                                 FitNode* __restrict__ fast, SlowNode* __restrict__ slow,
                                 int64_t* __restrict__ slow_list,
                                 unsigned long long* __restrict__ counters) {
  const uint64_t cmax = counters[2];
  int64_t p_cap = cmax ? (int64_t)(0x7fffffffull / cmax) : 0x7fffffffll;
  if (p_cap > FAST_P_MAX) p_cap = FAST_P_MAX;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - lane < n; i += stride) {
    const bool valid = i < n;
    bool ok = false;
    if (valid) {
      const uint64_t ac = alloc_cpu[i], uc = used_cpu[i];
      const int64_t am = alloc_mem[i], um = used_mem[i];
      const int64_t P = alloc_pods[i], pc = pod_count[i];
      const uint64_t fc = ac > uc ? ac - uc : 0;                                  // CC:119-123
      const int64_t fm = am > um ? (int64_t)((uint64_t)am - (uint64_t)um) : 0;   // CC:125-129
      const int64_t cl = (int64_t)((uint64_t)P - (uint64_t)pc);                  // CC:135
      ok = fc < FAST_FC_MAX && fm >= 0 && fm < FAST_FM_MAX && P >= FAST_P_MIN &&
           P <= p_cap && cl >= -FAST_CL_ABS && cl <= FAST_CL_ABS;
      FitNode f;  // rows off the fast path: all-zero record, contributes exactly 0
      f.fm_d = ok ? (double)fm : 0.0;
      f.fc_f = ok ? (float)fc : 0.f;                  // one rounding (fc < 2^31)
      f.fm_f = ok ? (float)(double)fm : 0.f;          // exact in f64, one rounding to f32
      f.fc_i = ok ? (int32_t)fc : 0;
      f.P_f = ok && P > 0 ? (float)P : 0.f;
      f.P_i = ok ? (int32_t)P : 0;
      f.cl_i = ok ? (int32_t)cl : 0;
      fast[i] = f;
      SlowNode sn;
      sn.fc = fc;
      sn.fm = fm;
      sn.P = P;
      sn.cl = cl;
      slow[i] = sn;
    }
    const unsigned long long b = __ballot(valid && !ok);
    if (b) {
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(&counters[1], (unsigned long long)__popcll(b));
      base = __shfl(base, 0);
      if (valid && !ok) slow_list[base + __popcll(b & ((1ull << lane) - 1ull))] = i;
    }
  }
}

// Single-workgroup stable partition of the specs (fast-path specs first), in two
// passes over contiguous per-thread chunks with one block-wide exclusive scan in
// between.  Also zeroes partial[0..2S) and counters[0..1] (no memset launches) and
// writes counters[2] = the largest fast-path cpu request.
__global__ __launch_bounds__(1024) void spec_prep_kernel(int64_t S, const uint64_t* __restrict__ c_in,
                                                         const int64_t* __restrict__ m_in,
                                                         SpecPrep sp, int64_t* __restrict__ partial,
                                                         unsigned long long* __restrict__ counters) {
  __shared__ int64_t wsum[16];
  __shared__ unsigned long long wmax[16];
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
  int64_t cnt = 0;
  unsigned long long cmax = 0;
  for (int64_t i = b0; i < b1; ++i) {
    const uint64_t c = spec_c(i);
    if (spec_is_normal(c, spec_m(i))) {
      ++cnt;
      cmax = c > cmax ? c : cmax;
    }
  }
  // block exclusive scan of cnt (wave shuffles + 16 wave totals in LDS)
  int64_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t u = __shfl_up(incl, d);
    if (lane >= d) incl += u;
  }
  unsigned long long mx = cmax;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(mx, d);
    mx = o > mx ? o : mx;
  }
  if (lane == 63) wsum[wv] = incl;
  if (lane == 0) wmax[wv] = mx;
  __syncthreads();
  int64_t wbase = 0, tot_n = 0;
  unsigned long long gmax = 0;
  for (int k = 0; k < 16; ++k) {
    if (k < wv) wbase += wsum[k];
    tot_n += wsum[k];
    gmax = wmax[k] > gmax ? wmax[k] : gmax;
  }
  int64_t pn = wbase + incl - cnt;  // my first fast-path slot
  int64_t pa = tot_n + (b0 - (wbase + incl - cnt));  // my first exact-path slot
  for (int64_t i = b0; i < b1; ++i) {
    const uint64_t c = spec_c(i);
    const int64_t m = spec_m(i);
    const bool nm = spec_is_normal(c, m);
    const int64_t pos = nm ? pn++ : pa++;
    SpecRec r;
    r.c = c;
    r.m = m;
    r.md = (double)m;
    // reciprocals biased up by 2^-20 so the fit's quotient estimate never
    // undershoots (f64 division, then one rounding to f32)
    r.rc = nm ? (float)(FIT_RECIP_BIAS / (double)c) : 0.f;
    r.rm = nm ? (float)(FIT_RECIP_BIAS / (double)m) : 0.f;
    sp.rec[pos] = r;
    sp.perm[pos] = (int32_t)i;
  }
  for (int64_t i = tid; i < 2 * S; i += 1024) partial[i] = 0;
  if (tid == 0) {
    counters[0] = 0;
    counters[1] = 0;
    counters[2] = gmax;
  }
}

// Lane = spec (its request, reciprocals and running total live in VGPRs); the node
// stream is wave-uniform, so each 32-B FitNode arrives by one scalar load and feeds
// the VALU as SGPR operands.  The main loop is branch-free: rows outside the fast
// bounds carry a zero-contribution FitNode and are re-done exactly from slow_list.
// No cross-lane reduction until the block's end (one 64-bit atomic per spec).
//
// Fast path per (node, spec), exact (DESIGN.md "fit kernel: exactness argument"):
//   the spec reciprocals are biased up by 2^-20 (spec_prep), so the f32 estimate
//   e = min(fc*rc, fm*rm, P) satisfies t <= e < t + 1 for t = min(qc, qm, P)
//   (its relative error is below 4*2^-24, and t <= P <= 2^16): k = floor(e) is t
//   or t + 1, never below.  One exact check fixes it:
//     rcpu = fc - k*c      i32 (v_mad_i32_i24; k*c < 2^31 by node_prep's P cap)
//     rmem = fm - k*m      f64 fma, exact (every value an integer < 2^53)
//     t    = k - [rcpu < 0 or rmem < 0]          (sign bits: no compares)
//   contribution = t >= P ? P - podCount : t                       (CC:133-136)
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int32_t fit_fast(const FitNode& nd, f32x2 rcm, double md,
                                            int32_t negc) {
  const f32x2 q = f32x2{nd.fc_f, nd.fm_f} * rcm;  // one v_pk_mul_f32
  const float e = fminf(fminf(q.x, q.y), nd.P_f);  // t <= e < t + 1
  const int32_t k = (int32_t)e;
  const int32_t rcpu = __mul24(k, negc) + nd.fc_i;
  const double rmem = fma(-(double)k, md, nd.fm_d);
  const int32_t hi = (int32_t)(__double_as_longlong(rmem) >> 32);
  const int32_t t = k + ((rcpu | hi) >> 31);
  return (t >= nd.P_i) ? nd.cl_i : t;
}

constexpr int FIT_UNROLL = 8;
#ifndef KCC_FIT_TARGET_BLOCKS
#define KCC_FIT_TARGET_BLOCKS 16384
#endif
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));

// one s_load_dwordx8 per record (a vector load is never split into field loads)
__device__ __forceinline__ FitNode load_node(const i32x8* __restrict__ q, int i) {
  return __builtin_bit_cast(FitNode, q[i]);
}

__global__ __launch_bounds__(256) void fit_kernel(
    int64_t n_nodes, int64_t nodes_per_block, const FitNode* __restrict__ fast,
    const SlowNode* __restrict__ slow, const int64_t* __restrict__ slow_list, int64_t S,
    const SpecRec* __restrict__ specs, int64_t* __restrict__ partial,
    unsigned long long* __restrict__ counters, int32_t gx,
    int32_t gy) {
  // XCD-aware order (speed only, never correctness): workgroups are dealt round-robin
  // over the 8 XCDs, so give every spec group of one node chunk the same b % 8 — the
  // chunk's FitNode records then stay in that XCD's L2 for all of them.
  const int32_t b = blockIdx.x, xcd = b & 7, r = b >> 3;
  const int32_t bx = r % gx, by = (r / gx) * 8 + xcd;
  if (by >= gy) return;  // padding of gy up to a multiple of 8 (whole workgroup)
  const int64_t s = (int64_t)bx * 256 + threadIdx.x;
  const bool active = s < S;
  SpecRec sr;  // one 32-B record per lane (two 16-B loads)
  if (active) {
    sr = specs[s];
  } else {
    sr.c = 1;
    sr.m = 1;
    sr.md = 1.0;
    sr.rc = 1.f;
    sr.rm = 1.f;
  }
  const uint64_t c = sr.c;
  const int64_t m = sr.m;
  const double md = sr.md;
  const float rc = sr.rc, rm = sr.rm;
  const bool normal = rc > 0.f;
  const bool wave_fast = __all(normal);
  const int32_t negc = -(int32_t)(uint32_t)c;
  const f32x2 rcm = {rc, rm};

  const int64_t n0 = (int64_t)by * nodes_per_block;
  const int64_t n1 = n0 + nodes_per_block < n_nodes ? n0 + nodes_per_block : n_nodes;
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

  if (wave_fast) {
    const i32x8* p = reinterpret_cast<const i32x8*>(fast + n0);
    const int cnt = (int)(n1 - n0);
    for (int cb = 0; cb < cnt; cb += 1024) {
      const int ce = cb + 1024 < cnt ? cb + 1024 : cnt;
      int32_t acc32 = 0;  // |contribution| <= 2^20: 1024 of them fit in i32
      int i = cb;
      for (; i + FIT_UNROLL <= ce; i += FIT_UNROLL) {
        // index opaque to loop-strength reduction: one base per group, positive
        // immediate offsets -> FIT_UNROLL s_load_dwordx8, no per-field address math
        int io = i;
        asm volatile("" : "+s"(io));
        const i32x8* q = p + io;
#pragma unroll
        for (int u = 0; u < FIT_UNROLL; ++u) acc32 += fit_fast(load_node(q, u), rcm, md, negc);
      }
      for (; i < ce; ++i) acc32 += fit_fast(load_node(p, i), rcm, md, negc);
      acc += (uint64_t)(int64_t)acc32;
    }
    // rows outside the fast bounds, shared out over the node-chunk blocks
    const int64_t n_slow = (int64_t)counters[1];
    for (int64_t j = by; j < n_slow; j += gy) eval_slow(slow_list[j]);
  } else {
    for (int64_t i = n0; i < n1; ++i) eval_slow(i);
  }

#ifdef KCC_FIT_DIAG_NO_ATOMICS  // diagnostic timing build only: results are wrong
  if (active && acc == 0x5A5A5A5A5A5A5A5Aull) partial[s] = (int64_t)acc;
#else
  if (active) {
    atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[s]), acc);
    if (errs) atomic_add_u64(reinterpret_cast<uint64_t*>(&partial[S + s]), errs);
  }
#endif
  const unsigned long long act = __ballot(active);
  if (slow_iters && (threadIdx.x & 63) == 0)
    atomicAdd(counters, (unsigned long long)slow_iters * (unsigned long long)__popcll(act));
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

hipError_t launch_reduce_mark(int64_t n_nodes, int64_t n_containers, const int64_t* node_ptr,
                              int64_t* wave_node, uint64_t* used_cpu, int64_t* used_mem,
                              uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s) {
  if (n_nodes <= 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_mark_kernel, dim3(grid_for(n_nodes, 256, 8192)), dim3(256), 0, s,
                     n_nodes, n_containers, reduce_range(n_containers), node_ptr, wave_node, used_cpu,
                     reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                     reinterpret_cast<uint64_t*>(lim_mem));
  return hipGetLastError();
}

hipError_t launch_reduce(int64_t n_nodes, int64_t n_containers, const int64_t* node_ptr,
                         const uint64_t* cpu_req, const int64_t* mem_req,
                         const uint64_t* cpu_lim, const int64_t* mem_lim,
                         const int64_t* wave_node, uint64_t* used_cpu, int64_t* used_mem,
                         uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s) {
  if (n_nodes <= 0 || n_containers <= 0) return hipSuccess;
  const int32_t range = reduce_range(n_containers);
  const int64_t waves = reduce_n_waves(n_containers);
  const unsigned blocks = (unsigned)((waves + RED_WAVES_PER_BLOCK - 1) / RED_WAVES_PER_BLOCK);
  const bool lim = cpu_lim && mem_lim && lim_cpu && lim_mem;
  if (lim) {
    hipLaunchKernelGGL(reduce_kernel<4>, dim3(blocks), dim3(256), 0, s, n_nodes, n_containers,
                       range, node_ptr, cpu_req, reinterpret_cast<const uint64_t*>(mem_req), cpu_lim,
                       reinterpret_cast<const uint64_t*>(mem_lim), wave_node, used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                       reinterpret_cast<uint64_t*>(lim_mem));
  } else {
    hipLaunchKernelGGL(reduce_kernel<2>, dim3(blocks), dim3(256), 0, s, n_nodes, n_containers,
                       range, node_ptr, cpu_req, reinterpret_cast<const uint64_t*>(mem_req),
                       (const uint64_t*)nullptr, (const uint64_t*)nullptr, wave_node, used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), (uint64_t*)nullptr,
                       (uint64_t*)nullptr);
  }
  return hipGetLastError();
}

hipError_t launch_node_prep(int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, FitNode* fast, SlowNode* slow,
                            int64_t* slow_list, unsigned long long* counters, hipStream_t s) {
  if (n_nodes <= 0) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel, dim3(grid_for(n_nodes, 256, 8192)), dim3(256), 0, s,
                     n_nodes, alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
                     fast, slow, slow_list, counters);
  return hipGetLastError();
}

hipError_t launch_spec_prep(int64_t n_specs, const uint64_t* spec_cpu, const int64_t* spec_mem,
                            SpecPrep sp, int64_t* partial, unsigned long long* counters,
                            hipStream_t s) {
  if (n_specs <= 0) return hipSuccess;
  hipLaunchKernelGGL(spec_prep_kernel, dim3(1), dim3(1024), 0, s, n_specs, spec_cpu, spec_mem,
                     sp, partial, counters);
  return hipGetLastError();
}

hipError_t launch_fit(int64_t n_nodes, const FitNode* fast, const SlowNode* slow,
                      const int64_t* slow_list, int64_t n_specs, SpecPrep sp, int64_t* partial,
                      unsigned long long* counters, hipStream_t s) {
  if (n_nodes <= 0 || n_specs <= 0) return hipSuccess;
  const int64_t gx = (n_specs + 255) / 256;
  // aim for KCC_FIT_TARGET_BLOCKS workgroups (2048 = one full round at 8 per CU); >= 64
  // nodes each
  int64_t gy_target = KCC_FIT_TARGET_BLOCKS / gx;
  if (gy_target < 1) gy_target = 1;
  int64_t npb = (n_nodes + gy_target - 1) / gy_target;
  if (npb < 64) npb = 64;
  int64_t gy = (n_nodes + npb - 1) / npb;
  // 1-D grid of gx * roundup(gy, 8) workgroups, remapped XCD-aware in the kernel
  while (gx * ((gy + 7) / 8 * 8) > 0x7fffffffLL) {
    npb *= 2;
    gy = (n_nodes + npb - 1) / npb;
  }
  const int64_t blocks = gx * ((gy + 7) / 8 * 8);
  hipLaunchKernelGGL(fit_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n_nodes, npb, fast,
                     slow, slow_list, n_specs, sp.rec, partial, counters, (int32_t)gx, (int32_t)gy);
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
