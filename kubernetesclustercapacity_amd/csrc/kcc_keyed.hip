// kcc_keyed.hip — per-node request sums from containers in LIST order (SURVEY.md §8f
// row 1, the lister side of (a)).
//
// The reference lists the pods of one node at a time (CC:232-253, one List per node) and
// sums their containers' requests (CC:290-293).  A cluster-wide `Pods("").List` returns
// the pods in namespace/name order instead, each container tagged with the row of its
// node (key).  kcc_reduce_requests_keyed sums such an unsorted stream without sorting it:
// uint64/int64 wrapping addition is commutative and associative, so per-key atomic adds
// give the reference's sums bit for bit in any order.  kcc_count_by_key counts the pods
// per key (len(pods), CC:106/135).
//
// Three implementations; keys < 0 or >= n_keys are skipped (pods whose
// node is not a listed row).  Rows are cut into buckets of KB_ROWS (n_keys <= KB_NB_MAX *
// KB_ROWS):
//  - one sweep (requests without limits, and the pod counts: the default): kb_sweep
//    counting-sorts each tile of containers by bucket in LDS and writes it as one
//    contiguous run of 8-B records, kb_gather sums each pair of buckets' segments of every
//    tile into LDS rows and writes them once, kb_escape adds what the records cannot hold;
//  - bucketed (calls with limits, four arrays): kb_hist counts each tile's containers per
//    bucket (LDS histogram), kb_scan turns the counts into scatter offsets, kb_scatter
//    moves every container's (row in bucket, values) into its bucket's contiguous range
//    (LDS cursors), and kb_accum sums each bucket in LDS (64-bit LDS atomics) and writes
//    its rows once.  No global atomics;
//  - direct atomics (more keys, or no workspace): each lane takes KY_IPL consecutive containers, merges
//    runs of equal keys in registers (a pod's containers are consecutive in a List) and
//    issues one 64-bit device atomic per array and run — device-scope atomics to random
//    rows execute past the L2s at ~14 G/s, so this is the slow path.
#include "kcc_internal.h"

namespace kcc {
namespace {

// Diagnostic timeline (KCC_TIMELINE builds only): per-workgroup s_memrealtime stamps (100 MHz)
// of the one-sweep path's phases — kb_gather workgroups in slots [0, 512), kb_sweep's in
// [512, 1024) — read by kcc_debug_timeline_keyed (scripts/probe/keyed_timeline.py)
#ifdef KCC_TIMELINE
__device__ uint64_t kcc_tlk[1024][8];
#define KCC_TLK(slot, k) \
  do { if (threadIdx.x == 0) kcc_tlk[(slot) & 1023][(k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define KCC_TLK(slot, k) do { } while (0)
#endif

constexpr int KY_THREADS = 256;
constexpr int KY_IPL = 4;                             // containers per lane
constexpr int KY_BLOCK = KY_THREADS * KY_IPL;         // containers per workgroup

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// inclusive prefix sum of a 32-bit value over the wave's 64 lanes (DPP, all VALU)
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ void add_u64(uint64_t* p, uint64_t v) {
  __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NA>  // 2: requests; 4: requests and limits
__global__ __launch_bounds__(KY_THREADS) void reduce_keyed_kernel(
    int64_t n, int64_t n_keys, const int32_t* __restrict__ key, const uint64_t* __restrict__ a0,
    const uint64_t* __restrict__ a1, const uint64_t* __restrict__ a2, const uint64_t* __restrict__ a3,
    uint64_t* __restrict__ o0, uint64_t* __restrict__ o1, uint64_t* __restrict__ o2,
    uint64_t* __restrict__ o3) {
  const uint64_t* in[4] = {a0, a1, a2, a3};
  uint64_t* out[4] = {o0, o1, o2, o3};
  const int64_t c = ((int64_t)blockIdx.x * KY_THREADS + threadIdx.x) * KY_IPL;
  if (c >= n) return;
  int32_t k[KY_IPL];
  uint64_t v[NA][KY_IPL];
  if (c + KY_IPL <= n) {  // whole quad: vector loads (the arrays are 16-byte aligned)
    const i32x4 kk = *reinterpret_cast<const i32x4*>(key + c);
    k[0] = kk.x;
    k[1] = kk.y;
    k[2] = kk.z;
    k[3] = kk.w;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const u64x2 lo = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c));
      const u64x2 hi = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c + 2));
      v[a][0] = lo.x;
      v[a][1] = lo.y;
      v[a][2] = hi.x;
      v[a][3] = hi.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < KY_IPL; ++j) {
      const bool in_range = c + j < n;
      k[j] = in_range ? key[c + j] : -1;
#pragma unroll
      for (int a = 0; a < NA; ++a) v[a][j] = in_range ? in[a][c + j] : 0;
    }
  }
  // runs of equal keys: container j folds into the run that ends at j + 1 when the key
  // repeats, else the run's sums are added to the key's totals
  uint64_t run[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) run[a] = v[a][0];
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) {
    const bool last = j + 1 == KY_IPL || k[j + 1] != k[j];
    if (last) {
      if (k[j] >= 0 && (int64_t)k[j] < n_keys) {
#pragma unroll
        for (int a = 0; a < NA; ++a) add_u64(out[a] + k[j], run[a]);
      }
      if (j + 1 < KY_IPL) {
#pragma unroll
        for (int a = 0; a < NA; ++a) run[a] = v[a][j + 1];
      }
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a) run[a] += v[a][j + 1];
    }
  }
}

__global__ __launch_bounds__(KY_THREADS) void count_keyed_kernel(int64_t n, int64_t n_keys,
                                                                 const int32_t* __restrict__ key,
                                                                 uint64_t* __restrict__ count) {
  const int64_t c = ((int64_t)blockIdx.x * KY_THREADS + threadIdx.x) * KY_IPL;
  if (c >= n) return;
  int32_t k[KY_IPL];
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) k[j] = c + j < n ? key[c + j] : -1;
  uint64_t run = 1;
#pragma unroll
  for (int j = 0; j < KY_IPL; ++j) {
    if (j + 1 == KY_IPL || k[j + 1] != k[j]) {
      if (k[j] >= 0 && (int64_t)k[j] < n_keys) add_u64(count + k[j], run);
      run = 1;
    } else {
      ++run;
    }
  }
}

// ---- bucketed path -------------------------------------------------------------------
constexpr int KB_HIST_THREADS = 512;
constexpr int KB_SCAN_THREADS = 256;
constexpr int KB_ACC_THREADS = 1024;
constexpr int KB_UNROLL = 8;

// counts[g * nb + b] = #{valid containers of tile g in bucket b}
__global__ __launch_bounds__(KB_HIST_THREADS) void kb_hist(int64_t n, int64_t n_keys,
                                                           const int32_t* __restrict__ key, int nb,
                                                           uint32_t* __restrict__ counts, int64_t tile) {
  extern __shared__ uint32_t kb_h[];
  for (int b = threadIdx.x; b < nb; b += KB_HIST_THREADS) kb_h[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = min(t0 + tile, n);
  for (int64_t c0 = t0 + threadIdx.x; c0 < t1; c0 += (int64_t)KB_HIST_THREADS * KB_UNROLL) {
    int32_t k[KB_UNROLL];
#pragma unroll
    for (int u = 0; u < KB_UNROLL; ++u) {
      const int64_t c = c0 + (int64_t)u * KB_HIST_THREADS;
      k[u] = c < t1 ? __builtin_nontemporal_load(key + c) : -1;
    }
#pragma unroll
    for (int u = 0; u < KB_UNROLL; ++u)
      if (k[u] >= 0 && (int64_t)k[u] < n_keys) atomicAdd(&kb_h[k[u] >> KB_SHIFT], 1u);
  }
  __syncthreads();
  uint32_t* row = counts + (int64_t)blockIdx.x * nb;
  for (int b = threadIdx.x; b < nb; b += KB_HIST_THREADS) row[b] = kb_h[b];
}

// inclusive scan of one value per thread over a workgroup of NT threads (LDS)
template <int NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int d = 1; d < NT; d <<= 1) {
    const uint32_t t = threadIdx.x >= (unsigned)d ? sh[threadIdx.x - d] : 0u;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  return sh[threadIdx.x];
}

// per bucket b (one workgroup): counts[g * nb + b] -> exclusive offset of tile g within
// the bucket; tot[b] = the bucket's size
__global__ __launch_bounds__(KB_SCAN_THREADS) void kb_scan(int64_t G, int nb,
                                                          uint32_t* __restrict__ counts,
                                                          uint32_t* __restrict__ tot,
                                                          uint32_t* __restrict__ esc_n) {
  __shared__ uint32_t sh[KB_SCAN_THREADS];
  const int b = blockIdx.x;
  if (esc_n && b == 0 && threadIdx.x == 0) *esc_n = 0;  // (the call's first chunk)
  const int64_t per = (G + KB_SCAN_THREADS - 1) / KB_SCAN_THREADS;
  const int64_t g0 = (int64_t)threadIdx.x * per, g1 = min(g0 + per, G);
  uint32_t s = 0;
  for (int64_t g = g0; g < g1; ++g) s += counts[g * nb + b];
  const uint32_t incl = block_incl_scan<KB_SCAN_THREADS>(s, sh);
  uint32_t run = incl - s;
  for (int64_t g = g0; g < g1; ++g) {
    const uint32_t v = counts[g * nb + b];
    counts[g * nb + b] = run;
    run += v;
  }
  if (threadIdx.x == KB_SCAN_THREADS - 1) tot[b] = incl;
}

// tile g: every valid container to its bucket's range, as an 8-B record:
//   bits  0-11  row within the bucket
//   bits 12-31  the low 20 bits of the cpu request
//   bits 32-63  the memory request / 64, when it is a multiple of 64 in [0, 2^38) (every
//               Mi/Gi/M/G quantity up to 256 GiB), else 0
// (+ with limits the two limit values as 64-bit words) — 8 B per container instead of 18.
// A cpu request of 2^20 millicores or more, or a memory request outside that form, also
// appends (row, cpu high bits, memory) to the escape list, added by kb_escape after the
// accumulation (wrapping sums: the parts add to the requests exactly).  The tile goes in
// sub-chunks of KB_SUB: each element's rank within its bucket (LDS counters), a scan of the
// sub-chunk's bucket counts, and a counting sort into an LDS stage, so that the global
// writes leave in bucket order — a bucket's elements of one sub-chunk land on consecutive
// addresses (its range in the bucket is this workgroup's, contiguous), and a wave's stores
// coalesce instead of touching 64 lines.
constexpr int KB_CPU_BITS = 32 - KB_SHIFT;  // 20
constexpr uint64_t KB_CPU_LO = ((uint64_t)1 << KB_CPU_BITS) - 1;
constexpr int KB_MEM_SHIFT = 6;             // memory in units of 64 B
constexpr int KB_MEM_MAX_BITS = 32 + KB_MEM_SHIFT;
constexpr int kb_nv(int na) { return na > 2 ? na - 2 : 1; }  // 64-bit words beside the record
constexpr int kb_sub(int na) { return na > 2 ? 2048 : 4096; }

// whether the record holds a memory request (a multiple of 64 in [0, 2^38))
__device__ __forceinline__ bool kb_mem_ok(uint64_t mem) {
  return (mem & ((1u << KB_MEM_SHIFT) - 1)) == 0 && (mem >> KB_MEM_MAX_BITS) == 0;
}
// the record of one container (NA >= 2)
__device__ __forceinline__ uint64_t kb_record(uint32_t row, uint64_t cpu, uint64_t mem) {
  return (uint64_t)row | (cpu & KB_CPU_LO) << KB_SHIFT |
         (kb_mem_ok(mem) ? (mem >> KB_MEM_SHIFT) << 32 : 0ull);
}

template <int NA>
__global__ __launch_bounds__(KB_HIST_THREADS) void kb_scatter(
    int64_t n, int64_t n_keys, const int32_t* __restrict__ key, const uint64_t* __restrict__ a0,
    const uint64_t* __restrict__ a1, const uint64_t* __restrict__ a2, const uint64_t* __restrict__ a3,
    int nb, const uint32_t* __restrict__ counts, const uint32_t* __restrict__ tot,
    uint64_t* __restrict__ sr, uint64_t* __restrict__ sv, uint32_t* __restrict__ esc_n,
    int32_t* __restrict__ esc_row, uint64_t* __restrict__ esc_cpu, uint64_t* __restrict__ esc_mem,
    int64_t tile) {
  constexpr int NV = kb_nv(NA);
  constexpr int NS = NA > 0 ? NA : 1;
  constexpr int KB_SUB = kb_sub(NA);
  constexpr int KB_SUB_PER = KB_SUB / KB_HIST_THREADS;
  constexpr int SV_LEN = NA > 2 ? KB_SUB : 1;
  // dynamic LDS: cur[nb], lcnt[nb], lstart[nb], scan scratch[KB_HIST_THREADS]
  extern __shared__ uint32_t kb_dyn[];
  uint32_t* cur = kb_dyn;
  uint32_t* lcnt = cur + nb;
  uint32_t* lstart = lcnt + nb;
  uint32_t* sh = lstart + nb;
  __shared__ uint64_t st_r[KB_SUB];
  __shared__ uint64_t st_v[NV][SV_LEN];
  __shared__ uint32_t st_pos[KB_SUB];
  const uint64_t* in[4] = {a0, a1, a2, a3};
  // this tile's cursors: bucket base (exclusive scan of tot) + the tile's offset in it
  const int per = (nb + KB_HIST_THREADS - 1) / KB_HIST_THREADS;
  const int b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
  uint32_t s = 0;
  for (int b = b0; b < b1; ++b) s += tot[b];
  const uint32_t incl = block_incl_scan<KB_HIST_THREADS>(s, sh);
  uint32_t run = incl - s;
  const uint32_t* crow = counts + (int64_t)blockIdx.x * nb;
  for (int b = b0; b < b1; ++b) {
    cur[b] = run + crow[b];
    lcnt[b] = 0;
    run += tot[b];
  }
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = min(t0 + tile, n);
  // sub-chunk loads run one sub-chunk ahead: issued before this one's scan, stage and
  // writes, consumed at the top of the next iteration
  int32_t kn[KB_SUB_PER];
  uint64_t vn[NS][KB_SUB_PER];
  // 16-B loads: thread t takes quads of consecutive containers (4 keys, 2 x 2 values per
  // array); the tile and sub-chunk starts are multiples of 4 and the arrays 16-B aligned
  auto load_sub = [&](int64_t c0) {
#pragma unroll
    for (int q = 0; q < KB_SUB_PER / 4; ++q) {
      const int64_t c = c0 + 4 * ((int64_t)q * KB_HIST_THREADS + threadIdx.x);
      if (c + 4 <= t1) {
        const i32x4 kk = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(key + c));
        kn[4 * q] = kk.x;
        kn[4 * q + 1] = kk.y;
        kn[4 * q + 2] = kk.z;
        kn[4 * q + 3] = kk.w;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const u64x2 lo = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c));
          const u64x2 hi = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(in[a] + c + 2));
          vn[a][4 * q] = lo.x;
          vn[a][4 * q + 1] = lo.y;
          vn[a][4 * q + 2] = hi.x;
          vn[a][4 * q + 3] = hi.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = c + j < t1;
          kn[4 * q + j] = ok ? key[c + j] : -1;
#pragma unroll
          for (int a = 0; a < NA; ++a) vn[a][4 * q + j] = ok ? in[a][c + j] : 0;
        }
      }
    }
  };
  load_sub(t0);
  for (int64_t c0 = t0; c0 < t1; c0 += KB_SUB) {
    int32_t k[KB_SUB_PER];
    uint32_t rk[KB_SUB_PER];
    uint64_t v[NS][KB_SUB_PER];
#pragma unroll
    for (int u = 0; u < KB_SUB_PER; ++u) {
      k[u] = kn[u];
#pragma unroll
      for (int a = 0; a < NA; ++a) v[a][u] = vn[a][u];
    }
#pragma unroll
    for (int u = 0; u < KB_SUB_PER; ++u) {
      const bool valid = k[u] >= 0 && (int64_t)k[u] < n_keys;
      if (!valid) k[u] = -1;
      rk[u] = valid ? atomicAdd(&lcnt[k[u] >> KB_SHIFT], 1u) : 0u;
      if (NA >= 2 && valid) {
        const bool mem_ok = kb_mem_ok(v[1 % NS][u]);
        if (!mem_ok || (v[0][u] >> KB_CPU_BITS) != 0) {  // rare: what the record cannot hold
          const uint32_t e = atomicAdd(esc_n, 1u);
          esc_row[e] = k[u];
          esc_cpu[e] = v[0][u] & ~KB_CPU_LO;
          esc_mem[e] = mem_ok ? 0ull : v[1 % NS][u];
        }
      }
    }
    load_sub(c0 + KB_SUB);  // past t1: every lane reads nothing
    __syncthreads();
    // lstart = exclusive scan of lcnt: the first wave alone (runs of wb buckets per lane,
    // a shuffle scan of the run totals), no workgroup-wide scan barriers
    if (threadIdx.x < 64) {
      const int wb = (nb + 63) / 64;
      const int w0 = threadIdx.x * wb, w1 = min(w0 + wb, nb);
      uint32_t ls = 0;
      for (int b = w0; b < w1; ++b) ls += lcnt[b];
      uint32_t li = ls;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(li, d, 64);
        if ((int)threadIdx.x >= d) li += t;
      }
      uint32_t lr = li - ls;
      for (int b = w0; b < w1; ++b) {
        lstart[b] = lr;
        lr += lcnt[b];
      }
      if (threadIdx.x == 63) sh[KB_HIST_THREADS - 1] = li;  // valid elements of the sub-chunk
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KB_SUB_PER; ++u) {
      if (k[u] < 0) continue;
      const int b = k[u] >> KB_SHIFT;
      const uint32_t slot = lstart[b] + rk[u];
      const uint32_t row = (uint32_t)k[u] & (KB_ROWS - 1);
      st_pos[slot] = cur[b] + rk[u];
      st_r[slot] = NA >= 2 ? kb_record(row, v[0][u], v[1 % NS][u]) : (uint64_t)row;
#pragma unroll
      for (int a = 2; a < NA; ++a) st_v[a - 2][slot] = v[a][u];
    }
    __syncthreads();
    const uint32_t nvalid = sh[KB_HIST_THREADS - 1];  // total of the lcnt scan
    for (uint32_t j = threadIdx.x; j < nvalid; j += KB_HIST_THREADS) {
      const uint32_t pos = st_pos[j];
      sr[pos] = st_r[j];
#pragma unroll
      for (int a = 2; a < NA; ++a) sv[(int64_t)pos * NV + a - 2] = st_v[a - 2][j];  // element-major
    }
    __syncthreads();  // nvalid read, stage drained before the counters change
    for (int b = b0; b < b1; ++b) {  // advance the cursors, clear the sub-chunk counts
      cur[b] += lcnt[b];
      lcnt[b] = 0;
    }
    __syncthreads();
  }
}

// bucket b: its range summed per row in LDS, rows [b * KB_ROWS, ...) written once, zero
// rows included (NA == 0: counts the containers per row)
template <int NA>
__global__ __launch_bounds__(KB_ACC_THREADS) void kb_accum(
    int64_t n, int64_t n_keys, int nb, const uint32_t* __restrict__ tot,
    const uint64_t* __restrict__ sr, const uint64_t* __restrict__ sv, uint64_t* __restrict__ o0,
    uint64_t* __restrict__ o1, uint64_t* __restrict__ o2, uint64_t* __restrict__ o3) {
  constexpr int NACC = NA > 0 ? NA : 1;
  constexpr int NV = kb_nv(NA);
  __shared__ unsigned long long acc[NACC][KB_ROWS];
  __shared__ uint32_t sh[KB_ACC_THREADS];
  uint64_t* out[4] = {o0, o1, o2, o3};
  const int b = blockIdx.x;
  for (int r = threadIdx.x; r < KB_ROWS; r += KB_ACC_THREADS)
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a][r] = 0ull;
  uint32_t s = 0;  // base = tot[0] + ... + tot[b - 1]
  for (int j = threadIdx.x; j < b; j += KB_ACC_THREADS) s += tot[j];
  const uint32_t base = block_incl_scan<KB_ACC_THREADS>(s, sh);  // syncs; base of the last
  const uint32_t start = sh[KB_ACC_THREADS - 1];
  (void)base;
  const uint32_t end = start + tot[b];
  auto add_elem = [&](uint64_t rec, const uint64_t* vals) {  // one record into the LDS rows
    const uint32_t r = (uint32_t)rec & (KB_ROWS - 1);
    if (NA == 0) {
      atomicAdd(&acc[0][r], 1ull);
    } else {
      atomicAdd(&acc[0][r], (unsigned long long)(((uint32_t)rec) >> KB_SHIFT));
      atomicAdd(&acc[1][r], (unsigned long long)((rec >> 32) << KB_MEM_SHIFT));
#pragma unroll
      for (int a = 2; a < NA; ++a) atomicAdd(&acc[a][r], (unsigned long long)vals[a - 2]);
    }
  };
  // [start, end) in three parts: the 16-B aligned middle as pairs (one 16-B load of 2
  // records, NV of 16-B loads of their limit values), the head and tail element by element
  // (64-bit: end may be close to 2^32)
  const int64_t a0 = ((int64_t)start + 1) & ~(int64_t)1, a1 = (int64_t)end & ~(int64_t)1;
  if (a0 >= a1) {
    for (int64_t i = (int64_t)start + threadIdx.x; i < (int64_t)end; i += KB_ACC_THREADS) {
      uint64_t vals[NV];
#pragma unroll
      for (int a = 0; a < NV; ++a) vals[a] = NA > 2 ? sv[i * NV + a] : 0ull;
      add_elem(sr[i], vals);
    }
  } else {
    if (threadIdx.x < 2) {  // head [start, a0) and tail [a1, end): at most 1 each
      const int64_t i = threadIdx.x == 0 ? (int64_t)start : a1;
      if (threadIdx.x == 0 ? i < a0 : i < (int64_t)end) {
        uint64_t vals[NV];
#pragma unroll
        for (int a = 0; a < NV; ++a) vals[a] = NA > 2 ? sv[i * NV + a] : 0ull;
        add_elem(sr[i], vals);
      }
    }
    constexpr int QU = KB_UNROLL;  // pairs per thread in flight
    for (int64_t q0 = a0 + 2 * (int64_t)threadIdx.x; q0 < a1; q0 += 2LL * KB_ACC_THREADS * QU) {
      u64x2 w[QU];
      u64x2 v[NV][QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int64_t i = q0 + 2LL * KB_ACC_THREADS * u;
        const bool ok = i < a1;
        w[u] = ok ? __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(sr + i)) : u64x2{0, 0};
#pragma unroll
        for (int h = 0; h < NV; ++h)
          v[h][u] = NA > 2 && ok ? __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(sv + i * NV) + h)
                                 : u64x2{0, 0};
      }
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        if (q0 + 2LL * KB_ACC_THREADS * u >= a1) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          uint64_t vals[NV];
#pragma unroll
          for (int a = 0; a < NV; ++a) {
            const int e = j * NV + a;  // the value's 8-B slot in the pair's limit words
            vals[a] = (e & 1) ? v[e >> 1][u].y : v[e >> 1][u].x;
          }
          add_elem(j ? w[u].y : w[u].x, vals);
        }
      }
    }
  }
  __syncthreads();
  const int64_t row0 = (int64_t)b * KB_ROWS;
  for (int r = threadIdx.x; r < KB_ROWS; r += KB_ACC_THREADS) {
    if (row0 + r >= n_keys) break;
#pragma unroll
    for (int a = 0; a < NACC; ++a) out[a][row0 + r] = acc[a][r];
  }
}

// the escape list, added to its rows after the accumulation: the cpu requests' high parts
// and the memory requests the records could not hold
constexpr unsigned KB_ESC_WG = 64;  // kb_escape workgroups (one arrival atomic each)
// esc_n[0]: the list's length; esc_n[1]: this launch's arrivals — the last workgroup to
// finish zeroes both, so the next call's sweep starts from an empty list
__global__ __launch_bounds__(256) void kb_escape(uint32_t* __restrict__ esc_n,
                                                 const int32_t* __restrict__ esc_row,
                                                 const uint64_t* __restrict__ esc_cpu,
                                                 const uint64_t* __restrict__ esc_mem,
                                                 uint64_t* __restrict__ o0, uint64_t* __restrict__ o1) {
  const uint32_t cnt = __hip_atomic_load(esc_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < cnt; i += gridDim.x * 256u) {
    const int32_t r = esc_row[i];
    if (esc_cpu[i]) add_u64(o0 + r, esc_cpu[i]);
    if (esc_mem[i]) add_u64(o1 + r, esc_mem[i]);
  }
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(esc_n + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
          gridDim.x - 1u) {
    __hip_atomic_store(esc_n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(esc_n + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- one-sweep path (NA = 0 counts / 2 requests) --------------------------------------
// kb_sweep: tile g = containers [g * tile, ...) (tile <= KB_SW_TILE: keyed_sweep_tile), 8
// per thread (16-B loads of quads).  Each valid container's rank within its bucket comes
// from an LDS counter (two 16-bit counters per word), one exclusive scan of the counts
// gives the bucket starts, the records are counting-sorted into an LDS stage and leave as
// ONE contiguous run of nvalid records (16-B stores: whole lines) into the tile's own
// region sr[g * KB_SW_TILE ...], the starts into the tile's table entries (kb_tab_at:
// entry (g, b), entry (g, nb) = nvalid).  No global histogram, no scan launch, and the keys are read once.
constexpr int KB_SW_WAVES = KB_SW_THREADS / 64;
constexpr int KB_SW_CNT_WORDS = (int)(KB_NB_MAX / 2);  // two 16-bit bucket counts per word

__device__ __forceinline__ uint32_t kb_half(const uint32_t* w, int b) {
  return (w[b >> 1] >> (16 * (b & 1))) & 0xffffu;
}

// The tiles' bucket starts (the sweep's table): 16-bit entries (a tile holds < 2^16
// records) in blocks of KB_TB buckets — entry (g, b) at [b / KB_TB][g][b % KB_TB] — so a
// gather workgroup, whose bucket pair lies in one or two blocks, reads 64-B pieces of
// them, and an XCD's groups (a contiguous run of buckets) read about 1/8 of the table
// (round 5's [g][nb + 1] u32 rows: every XCD read the whole 4.8 MB table at C4)
constexpr int KB_TB = 32;
__device__ __forceinline__ int64_t kb_tab_at(int64_t G, int64_t g, int b) {
  return ((int64_t)(b / KB_TB) * G + g) * KB_TB + (b % KB_TB);
}

// Persistent and software-pipelined (round 5): one workgroup per CU walks the tiles
// g = blockIdx.x, + gridDim.x, ...; the next tile's loads (range-checked buffer loads, so
// their count is static) go out before the current tile's ranks, scan, scatter and
// stores, so the CU's HBM traffic does not stop for the LDS work.  Round 4's sweep took one
// 16384-container tile per workgroup launch — load, then work, then store, every phase
// alone on the CU: C4 keyed 0.3327 -> 0.3257 ms (sweep 255 -> 223 us, the gather 83 ->
// 112 us over twice the segments).
template <int NA>
__global__ __launch_bounds__(KB_SW_THREADS) void kb_sweep(
    int64_t n, int64_t n_keys, const int32_t* __restrict__ key, const uint64_t* __restrict__ a0,
    const uint64_t* __restrict__ a1, int nb, uint32_t* __restrict__ tab, uint64_t* __restrict__ sr,
    uint32_t* __restrict__ esc_n, int32_t* __restrict__ esc_row, uint64_t* __restrict__ esc_cpu,
    uint64_t* __restrict__ esc_mem, int64_t tile, int64_t G) {
  static_assert(NA == 0 || NA == 2, "one-sweep path: counts or requests");
  constexpr int NS = NA > 0 ? NA : 1;
  constexpr int PER = KB_SW_PER;
  __shared__ uint64_t st[KB_SW_TILE];  // the tile's records, bucket order
  __shared__ uint32_t cnt2[KB_SW_CNT_WORDS];
  __shared__ uint32_t wtot[KB_SW_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nw = (nb + 1) / 2;
  // tile g's loads: quads of consecutive containers (16-B buffer loads through descriptors
  // that end at the tile's end: outside, they read 0 and the validity test drops them)
  int32_t kn[PER];
  uint64_t vn[NS][PER];
  auto issue = [&](int64_t g) {
    const int64_t t0 = g * tile, t1 = min(t0 + tile, n);
    const int32_t len = (int32_t)(t1 > t0 ? t1 - t0 : 0);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(key + t0), (short)0, 4 * len, 0x00020000);
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
      const int32_t o = 4 * (q * KB_SW_THREADS + tid);
      const i32x4 kk = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, 4 * o, 0, 2));
      kn[4 * q] = kk.x;
      kn[4 * q + 1] = kk.y;
      kn[4 * q + 2] = kk.z;
      kn[4 * q + 3] = kk.w;
    }
    if constexpr (NA == 2) {
      const uint64_t* in[2] = {a0, a1};
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(in[a] + t0), (short)0, 8 * len, 0x00020000);
#pragma unroll
        for (int q = 0; q < PER / 4; ++q) {
          const int32_t o = 4 * (q * KB_SW_THREADS + tid);
          const u64x2 lo = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rv, 8 * o, 0, 2));
          const u64x2 hi = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(rv, 8 * o + 16, 0, 2));
          vn[a][4 * q] = lo.x;
          vn[a][4 * q + 1] = lo.y;
          vn[a][4 * q + 2] = hi.x;
          vn[a][4 * q + 3] = hi.y;
        }
      }
    }
  };
  int64_t g = blockIdx.x;
  KCC_TLK(512 + blockIdx.x, 0);
  if (g < G) issue(g);
  for (; g < G; g += gridDim.x) {
    if (g == (int64_t)blockIdx.x + gridDim.x) KCC_TLK(512 + blockIdx.x, 1);  // first tile done
    const int64_t t0 = g * tile, t1 = min(t0 + tile, n);
    int32_t k[PER];
    uint64_t v[NS][PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      k[u] = kn[u];
#pragma unroll
      for (int a = 0; a < NS; ++a) v[a][u] = NA == 2 ? vn[a][u] : 0ull;
    }
    if (g + gridDim.x < G) issue(g + gridDim.x);  // in flight during this tile's work
    for (int w = tid; w < nw; w += KB_SW_THREADS) cnt2[w] = 0;
    __syncthreads();  // counters zeroed (and the previous tile's stage read)
    uint64_t rec[PER];
    uint32_t br[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t c = t0 + 4 * ((int64_t)(u / 4) * KB_SW_THREADS + tid) + (u & 3);
      const bool valid = c < t1 && k[u] >= 0 && (int64_t)k[u] < n_keys;
      const int b = valid ? k[u] >> KB_SHIFT : 0;
      const uint32_t sh = 16u * (uint32_t)(b & 1);
      const uint32_t rk = valid ? (atomicAdd(&cnt2[b >> 1], 1u << sh) >> sh) & 0xffffu : 0u;
      br[u] = valid ? (uint32_t)b << 16 | rk : 0xffffffffu;
      const uint32_t row = (uint32_t)k[u] & (KB_ROWS - 1);
      if constexpr (NA == 2) {
        rec[u] = kb_record(row, v[0][u], v[1][u]);
        if (valid) {
          const bool mem_ok = kb_mem_ok(v[1][u]);
          if (!mem_ok || (v[0][u] >> KB_CPU_BITS) != 0) {  // rare: what the record cannot hold
            const uint32_t e = atomicAdd(esc_n, 1u);
            esc_row[e] = k[u];
            esc_cpu[e] = v[0][u] & ~KB_CPU_LO;
            esc_mem[e] = mem_ok ? 0ull : v[1][u];
          }
        }
      } else {
        rec[u] = row;
      }
    }
    __syncthreads();
    uint32_t c4[4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int w = 2 * tid + j;
      const uint32_t x = w < nw ? cnt2[w] : 0u;
      c4[2 * j] = x & 0xffffu;
      c4[2 * j + 1] = x >> 16;
    }
    const uint32_t s4 = c4[0] + c4[1] + c4[2] + c4[3];
    const uint32_t incl = wave_incl_scan32(s4);
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    uint32_t wbase = 0, nvalid = 0;
#pragma unroll
    for (int w = 0; w < KB_SW_WAVES; ++w) {
      const uint32_t t = wtot[w];
      wbase += w < wv ? t : 0u;
      nvalid += t;
    }
    {
      uint32_t run = wbase + incl - s4;
      uint32_t st4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st4[j] = run;
        run += c4[j];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int w = 2 * tid + j;
        if (w < nw) cnt2[w] = st4[2 * j] | st4[2 * j + 1] << 16;
      }
      // (4 tid .. 4 tid + 3 lie in one block: one 8-B store; the entry nb = nvalid)
      static_assert(KB_TB % 4 == 0, "a thread's four entries in one block");
      if (4 * tid <= nb) {
        // (32-bit block offset: the table holds < 2^32 entries, keyed_counts_words)
        uint16_t* const t16 = reinterpret_cast<uint16_t*>(tab) + (uint32_t)g * KB_TB +
                              (uint32_t)(4 * tid / KB_TB) * (uint32_t)(G * KB_TB) + (4 * tid) % KB_TB;
        uint32_t e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = 4 * tid + j == nb ? nvalid : st4[j];
        if (4 * tid + 3 <= nb) {
          *reinterpret_cast<uint2*>(t16) = make_uint2(e[0] | e[1] << 16, e[2] | e[3] << 16);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (4 * tid + j <= nb) t16[j] = (uint16_t)e[j];
        }
      }
      if (tid == 0 && nb >= 4 * KB_SW_THREADS)  // (the entry nb past every thread's four)
        reinterpret_cast<uint16_t*>(tab)[kb_tab_at(G, g, nb)] = (uint16_t)nvalid;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      if (br[u] == 0xffffffffu) continue;
      st[kb_half(cnt2, (int)(br[u] >> 16)) + (br[u] & 0xffffu)] = rec[u];
    }
    __syncthreads();
    // the stage leaves as one contiguous run: a fixed number of 16-B streaming stores per
    // thread, through a descriptor that ends at nvalid records (past it they are dropped;
    // an odd last record goes as a pair with the zero slot after it, which is in range of
    // the tile's region but past nvalid: harmless)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(sr + g * KB_SW_TILE), (short)0, 8 * (int)((nvalid + 1u) & ~1u), 0x00020000);
#pragma unroll
    for (int h = 0; h < KB_SW_TILE / (2 * KB_SW_THREADS); ++h) {
      const uint32_t j = 2u * (uint32_t)(h * KB_SW_THREADS + tid);
      const u64x2 pr = *reinterpret_cast<const u64x2*>(&st[j]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, pr), rs, (int)(8 * j), 0, 2);
    }
  }
  KCC_TLK(512 + blockIdx.x, 2);
}

// kb_gather: bucket group b's records — segment [entry (g, b0), entry (g, b0 + nbk)) of every tile
// g — summed into LDS rows (64-bit LDS atomics), its rows written once.  `parts` workgroups
// share a group (tiles dealt round-robin): each sums its tiles; the last to arrive adds the
// others' rows and writes the outputs, and only the others publish theirs (part_acc).
// XCD-aware placement: workgroup i runs on XCD i mod KB_XCDS, and the slots of one XCD are
// a contiguous run of groups (both parts of a group included), so neighbouring groups — whose
// segments of a tile are neighbours in its run and share the lines at their ends, and whose
// table entries share lines — read them through one L2 (round 5's placement spread neighbours
// over the 8 XCDs: each line at a segment end and each table line was fetched by several L2s,
// 1.34x the records' bytes).
// A wave works on two sub-batches of KB_GA_U2 segments at once, the first summed while the
// second's loads are in flight (a segment is a few hundred bytes: one per wave would be
// latency-bound).
constexpr int KB_GA_THREADS = 1024;
constexpr int KB_GA_WAVES = KB_GA_THREADS / 64;
// segments per sub-batch (two per wave at once: 2 x 8 x 128 records, as round 5's one
// batch of 16 x 128)
constexpr int KB_GA_U2 = 8;
static_assert((KB_GA_U2 & (KB_GA_U2 - 1)) == 0 && KB_GA_U2 <= 64,
              "a sub-batch's table entries are read by lanes lane & (KB_GA_U2 - 1)");
constexpr int KB_GA_CH = 2048;  // tiles per table chunk in LDS (a barrier each: 1024 measured slower)
constexpr int KB_XCDS = 8;      // gfx950: 8 XCDs, workgroups dealt round-robin
// buckets per gather workgroup: a tile's segments of KB_GA_BPG adjacent buckets are
// contiguous in its run, so a workgroup reads them as one segment (half the segments, their
// partial lines and their latency batches, for twice the LDS rows)
constexpr int KB_GA_BPG = 2;
constexpr int KB_GA_ROWS = KB_GA_BPG * KB_ROWS;  // LDS rows per gather workgroup
static_assert(KB_SW_TILE < 0xffff, "a segment's length and split point pack in 16 bits each; table entries are u16");
static_assert(2 * KB_GA_ROWS * 8 + 2 * KB_GA_CH * 4 + 64 <= 160 * 1024,
              "kb_gather<2>'s LDS (rows of both arrays + the segment tables) fits one CU");
// Tiles are read newest-first (the last-written records first, while the memory-side cache
// may hold them): measured equal (0.3427 / 0.3432 ms), kept.
[[maybe_unused]] constexpr uint32_t KB_GA_SPIN_MAX = 1u << 22;  // polls before the wait gives up

template <int NA>
__global__ __launch_bounds__(KB_GA_THREADS) void kb_gather(
    int64_t G, int64_t n_keys, int nb, int parts, uint32_t stride, const uint32_t* __restrict__ tab,
    const uint64_t* __restrict__ sr, uint64_t* __restrict__ part_acc, uint32_t* __restrict__ arrive,
    unsigned long long* __restrict__ faults, uint64_t* __restrict__ o0, uint64_t* __restrict__ o1) {
  constexpr int NACC = NA > 0 ? NA : 1;
  __shared__ unsigned long long acc[NACC][KB_GA_ROWS];
  __shared__ uint32_t seg_off[KB_GA_CH];  // start within the tile
  __shared__ uint32_t seg_len[KB_GA_CH];  // length | (where the group's second bucket starts) << 16
  __shared__ uint32_t last_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // this workgroup's slot: XCD x = blockIdx.x mod KB_XCDS holds slots [x q + min(x, r), ...)
  const uint32_t W = gridDim.x, x = blockIdx.x % KB_XCDS, jx = blockIdx.x / KB_XCDS;
  const uint32_t q = W / KB_XCDS, rr = W % KB_XCDS;
  const uint32_t slot = x * q + (x < rr ? x : rr) + jx;
  // b: the bucket group (buckets KB_GA_BPG b .. + nbk - 1)
  const int b = (int)(slot / (uint32_t)parts), part = (int)(slot % (uint32_t)parts);
  const int b0 = KB_GA_BPG * b, nbk = nb - b0 < KB_GA_BPG ? nb - b0 : KB_GA_BPG;
  KCC_TLK(blockIdx.x, 0);
  for (int r = tid; r < KB_GA_ROWS; r += KB_GA_THREADS)
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a][r] = 0ull;
  // this part's tiles: g = part, part + parts, ...
  const int64_t my_tiles = G > part ? (G - part + parts - 1) / parts : 0;
#ifdef KCC_DIAG_GA_NOATOM
  uint64_t dg = 0;  // timing build: the records summed into a register (wrong sums)
  auto add_rec = [&](uint64_t rec, uint32_t hi) { dg += rec + hi; };
#else
  auto add_rec = [&](uint64_t rec, uint32_t hi) {  // hi: KB_ROWS for the group's second bucket
    const uint32_t r = ((uint32_t)rec & (KB_ROWS - 1)) + hi;
    if constexpr (NA == 0) {
      atomicAdd(&acc[0][r], 1ull);
    } else {
      atomicAdd(&acc[0][r], (unsigned long long)(((uint32_t)rec) >> KB_SHIFT));
      atomicAdd(&acc[1][r], (unsigned long long)((rec >> 32) << KB_MEM_SHIFT));
    }
  };
#endif
  for (int64_t c0 = 0; c0 < my_tiles; c0 += KB_GA_CH) {
    const int ch = (int)min((int64_t)KB_GA_CH, my_tiles - c0);
    __syncthreads();  // the previous chunk's table entries are consumed
    // the chunk's table entries: every thread's loads issued before any is used (one round
    // trip per chunk, not one per KB_GA_THREADS entries)
    constexpr int TQ = KB_GA_CH / KB_GA_THREADS;
    uint32_t e0[TQ], e1[TQ], e2[TQ];
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const int i = tid + q * KB_GA_THREADS;
      const int64_t g = (int64_t)part + (my_tiles - 1 - (c0 + (i < ch ? i : 0))) * parts;
      const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tab);
      e0[q] = t16[kb_tab_at(G, g, b0)];
      e1[q] = t16[kb_tab_at(G, g, b0 + nbk)];
      e2[q] = t16[kb_tab_at(G, g, KB_GA_BPG > 1 && nbk > 1 ? b0 + 1 : b0)];
    }
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const int i = tid + q * KB_GA_THREADS;
      if (i < ch) {
        seg_off[i] = e0[q];
        // (tile runs < 2^16 records: 0xffff is "no second bucket", past every index)
        seg_len[i] = (e1[q] - e0[q]) | (KB_GA_BPG > 1 && nbk > 1 ? e2[q] - e0[q] : 0xffffu) << 16;
      }
    }
    __syncthreads();
    if (c0 == 0) KCC_TLK(blockIdx.x, 1);
    // sub-batch t = segments [KB_GA_U2 t, KB_GA_U2 (t + 1)) of the chunk; wave wv takes
    // t = wv, wv + KB_GA_WAVES, ...  Every load is issued whatever the segment's length (lanes
    // past it re-read the segment's first record, a line the wave reads anyway), so each
    // sub-batch issues the same instructions and the waits stay static
    const int nsb = (ch + KB_GA_U2 - 1) / KB_GA_U2;
    uint64_t ra[KB_GA_U2][2], rb[KB_GA_U2][2];
    uint32_t la[KB_GA_U2], fa[KB_GA_U2], lb[KB_GA_U2], fb[KB_GA_U2];
    auto load_sb = [&](int t, uint64_t (&r)[KB_GA_U2][2], uint32_t (&len)[KB_GA_U2],
                       uint32_t (&first)[KB_GA_U2]) {
      // the sub-batch's table entries: one LDS read per array by lanes 0..U2-1, then
      // wave-uniform (SGPR) lengths and starts
      const int ib = KB_GA_U2 * t, il = ib + (lane & (KB_GA_U2 - 1));
      const bool lok = t < nsb && il < ch;
      const uint32_t vlen = lok ? seg_len[il] : 0xffff0000u;  // length | mid << 16
      const uint32_t voff = lok ? seg_off[il] : 0u;
#pragma unroll
      for (int u = 0; u < KB_GA_U2; ++u) {
        const bool ok = t < nsb && ib + u < ch;  // (wave-uniform)
        const uint32_t gi = (uint32_t)(c0 + (ok ? ib + u : 0));
        const uint32_t g = (uint32_t)part + ((uint32_t)my_tiles - 1u - gi) * (uint32_t)parts;
        // (registers, not LDS: an LDS read between the adds would wait for every LDS atomic
        // issued before it)
        len[u] = (uint32_t)__builtin_amdgcn_readlane((int)vlen, u);
        first[u] = g * stride + (uint32_t)__builtin_amdgcn_readlane((int)voff, u);
        const uint64_t* __restrict__ seg = sr + first[u];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t o = (uint32_t)lane + 64u * h;
          // (default policy: a non-temporal load measured equal, r06e; the neighbouring
          // groups' reads of a shared end line hit in the XCD's L2)
          r[u][h] = seg[o < (len[u] & 0xffffu) ? o : 0u];
        }
      }
    };
    auto sum_sb = [&](uint64_t (&r)[KB_GA_U2][2], uint32_t (&len)[KB_GA_U2],
                      uint32_t (&first)[KB_GA_U2]) {
#pragma unroll
      for (int u = 0; u < KB_GA_U2; ++u) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t o = (uint32_t)lane + 64u * h;
          if (o < (len[u] & 0xffffu)) add_rec(r[u][h], o >= (len[u] >> 16) ? (uint32_t)KB_ROWS : 0u);
        }
      }
      // the rest of long segments (skewed keys), 64 records a step
#pragma unroll 1
      for (int u = 0; u < KB_GA_U2; ++u)
        for (uint32_t o = 128u + (uint32_t)lane; o < (len[u] & 0xffffu); o += 64u)
          add_rec(sr[first[u] + o], o >= (len[u] >> 16) ? (uint32_t)KB_ROWS : 0u);
    };
    // two sub-batches loaded at once, the first summed while the second arrives (the next
    // pair's loads kept in flight across iterations measured equal, r06d: the compiler's
    // loop-carried registers wait for them at the loop head)
    for (int t = wv; t < nsb; t += 2 * KB_GA_WAVES) {
      load_sb(t, ra, la, fa);
      load_sb(t + KB_GA_WAVES, rb, lb, fb);  // (past nsb: a harmless re-read, summed as empty)
      sum_sb(ra, la, fa);
      sum_sb(rb, lb, fb);
    }
  }
  __syncthreads();
  KCC_TLK(blockIdx.x, 2);
#ifdef KCC_DIAG_GA_NOATOM
  if (dg == 0x123456789ull) acc[0][0] = dg;  // (keeps the sums alive)
#endif
  const int64_t row0 = (int64_t)b0 * KB_ROWS;
  uint64_t* out[2] = {o0, o1};
  if (parts == 1) {
    for (int r = tid; r < KB_GA_ROWS; r += KB_GA_THREADS) {
      if (row0 + r >= n_keys) break;
#pragma unroll
      for (int a = 0; a < NACC; ++a) out[a][row0 + r] = acc[a][r];
    }
    return;
  }
  // several parts: arrive first; every part but the last publishes its rows and then raises
  // the group's ready count, the last waits for that count, adds the others' rows and writes
  // the outputs (round 5 had every part publish before arriving: the last part's rows went
  // to part_acc for nothing, 3x the output's bytes written).  The hand-off is the node-prep
  // one (kcc_kernels.hip np_wait_rows): agent-scope stores, each wave's vmcnt(0) before the
  // barrier, then the count; agent-scope loads after it.  A waiting part is resident and its
  // peers have arrived (they are past their sums), so the wait is short; it is bounded anyway
  uint32_t* const ready = arrive + (nb + KB_GA_BPG - 1) / KB_GA_BPG;
  if (tid == 0)
    last_s = __hip_atomic_fetch_add(arrive + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (uint32_t)parts - 1u;
  __syncthreads();
  KCC_TLK(blockIdx.x, 3);
  const int64_t pstride = (int64_t)NACC * KB_GA_ROWS;
  if (!last_s) {
    uint64_t* mine = part_acc + ((int64_t)b * parts + part) * pstride;
    for (int r = tid; r < KB_GA_ROWS; r += KB_GA_THREADS)
#pragma unroll
      for (int a = 0; a < NACC; ++a)
        __hip_atomic_store(mine + a * KB_GA_ROWS + r, (uint64_t)acc[a][r], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(ready + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    KCC_TLK(blockIdx.x, 4);
    return;
  }
  if (tid == 0) {
    uint32_t spins = 0;
#ifdef KCC_DIAG_RED_GIVEUP  // fault-path build: the wait gives up at once, as a timed-out one
    if (faults) atomicAdd(faults + FAULT_RED, 1ull);
    spins = KB_GA_SPIN_MAX;
#endif
    while (spins < KB_GA_SPIN_MAX &&
           __hip_atomic_load(ready + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
           (uint32_t)parts - 1u) {
      if (++spins >= KB_GA_SPIN_MAX) {  // never on a healthy device: the sums are not trusted
        if (faults) atomicAdd(faults + FAULT_RED, 1ull);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    __hip_atomic_store(arrive + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ready + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  KCC_TLK(blockIdx.x, 5);
  // the others' rows: each part's loads all issued before they are added (one round trip
  // per part, not one per KB_GA_THREADS rows)
  constexpr int RQ = KB_GA_ROWS / KB_GA_THREADS;
  static_assert(KB_GA_ROWS % KB_GA_THREADS == 0, "whole row rounds");
  uint64_t t[RQ][NACC];
#pragma unroll
  for (int q = 0; q < RQ; ++q)
#pragma unroll
    for (int a = 0; a < NACC; ++a) t[q][a] = acc[a][tid + q * KB_GA_THREADS];
  for (int p = 0; p < parts; ++p) {
    if (p == part) continue;
    const uint64_t* src = part_acc + ((int64_t)b * parts + p) * pstride;
    uint64_t v[RQ][NACC];
#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
      for (int a = 0; a < NACC; ++a)
        v[q][a] = __hip_atomic_load(src + a * KB_GA_ROWS + tid + q * KB_GA_THREADS, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
      for (int a = 0; a < NACC; ++a) t[q][a] += v[q][a];
  }
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int r = tid + q * KB_GA_THREADS;
    if (row0 + r < n_keys)
#pragma unroll
      for (int a = 0; a < NACC; ++a) out[a][row0 + r] = t[q][a];
  }
  KCC_TLK(blockIdx.x, 6);
}

}  // namespace

static int keyed_cus() {  // (thread-safe once: a function-local static's initializer)
  static const int cus = [] {
    int dev = 0, c = 0;
    return hipGetDevice(&dev) == hipSuccess &&
                   hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                   c > 0
               ? c
               : 256;
  }();
  return cus;
}

// Containers per scatter workgroup: about KB_TILE, cut so the tiles make whole rounds of
// one workgroup per CU (the scatter's LDS and registers hold one per CU): 1209 tiles of
// 32768 at C4 were 4.7 rounds, the last one 70 % full.
int64_t keyed_tile(int64_t n) {
  const int64_t cus = keyed_cus();
  if (n <= 0) return KB_TILE;
  const int64_t rounds = (n + KB_TILE * cus - 1) / (KB_TILE * cus);
  const int64_t t = (n + rounds * cus - 1) / (rounds * cus);
  return (t + 3) / 4 * 4;  // quads: 16-B loads
}
int64_t keyed_tiles(int64_t n) {
  const int64_t t = keyed_tile(n);
  return (n + t - 1) / t;
}
int64_t keyed_buckets(int64_t n_keys) { return (n_keys + KB_ROWS - 1) / KB_ROWS; }
bool keyed_bucketed(int64_t n_keys, int64_t n) {  // (record indices, padded tiles, < 2^32)
  return n_keys > 0 && keyed_buckets(n_keys) <= KB_NB_MAX && n < ((int64_t)1 << 32) - KB_SW_TILE &&
         keyed_sweep_tiles(n) * KB_SW_TILE < ((int64_t)1 << 32);
}
int64_t keyed_sweep_tile(int64_t n) {
  const int64_t cus = keyed_cus();
  if (n <= KB_SW_TILE * cus) return KB_SW_TILE;
  const int64_t rounds = (n + KB_SW_TILE * cus - 1) / (KB_SW_TILE * cus);
  const int64_t t = (n + rounds * cus - 1) / (rounds * cus);
  return (t + 3) / 4 * 4;  // (quads: 16-B loads; <= KB_SW_TILE, a multiple of 4)
}
int64_t keyed_sweep_tiles(int64_t n) {
  const int64_t t = keyed_sweep_tile(n);
  return n > 0 ? (n + t - 1) / t : 0;
}

// gather workgroups per bucket group (one workgroup per CU: its LDS rows): as many as one
// round of them holds, 1 to 4 (C4: 123 groups of two buckets, 2 parts; round 4 with one
// bucket per workgroup, 245 buckets: 1 part 0.339-0.340 ms, 2 parts 0.372 ms)
constexpr int KB_GA_PARTS_MAX = 4;
int keyed_sweep_parts(int64_t nb) {
  const int64_t cus = keyed_cus(), ng = (nb + KB_GA_BPG - 1) / KB_GA_BPG;
  if (ng <= 0) return 1;
  const int64_t p = cus / ng;
  return (int)(p < 1 ? 1 : p > KB_GA_PARTS_MAX ? KB_GA_PARTS_MAX : p);
}
int64_t keyed_counts_words(int64_t n_keys, int64_t n) {
  const int64_t nb = keyed_buckets(n_keys);
  const int64_t a = keyed_tiles(n) * nb;
  const int64_t b = (nb / KB_TB + 1) * keyed_sweep_tiles(n) * KB_TB / 2;  // (u16 entries, blocked)
  return a > b ? a : b;
}
int64_t keyed_sr_slots(int64_t n) {
  const int64_t t = keyed_sweep_tiles(n) * KB_SW_TILE;
  return t > n ? t : n;
}
int64_t keyed_part_words(int64_t n_keys, int na) {  // (bucket groups x parts x arrays x rows)
  const int64_t ng = (keyed_buckets(n_keys) + KB_GA_BPG - 1) / KB_GA_BPG;
  return ng * KB_GA_PARTS_MAX * (na > 0 ? na : 1) * (int64_t)KB_GA_ROWS;
}

// the one-sweep path (NA = 0 / 2): kb_sweep, kb_gather, kb_escape
template <int NA>
static hipError_t run_sweep(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* const* in,
                            uint64_t* const* out, const KeyedWork& kw, hipStream_t s) {
  const int nb = (int)keyed_buckets(n_keys);
  const int64_t G = keyed_sweep_tiles(n), tile = keyed_sweep_tile(n);
  const int parts = keyed_sweep_parts(nb);
  if (G > 0x7fffffff || (int64_t)nb * parts > 0x7fffffff) return hipErrorInvalidValue;
  if (G > 0) {  // one persistent workgroup per CU at most
    const int64_t wg = G < keyed_cus() ? G : keyed_cus();
    hipLaunchKernelGGL(kb_sweep<NA>, dim3((unsigned)wg), dim3(KB_SW_THREADS), 0, s, n, n_keys, key,
                       in[0], in[1], nb, kw.counts, kw.sr, kw.esc_n, kw.esc_row, kw.esc_cpu, kw.esc_mem,
                       tile, G);
  }
  const int ng = (nb + KB_GA_BPG - 1) / KB_GA_BPG;  // bucket groups
  hipLaunchKernelGGL(kb_gather<NA>, dim3((unsigned)(ng * parts)), dim3(KB_GA_THREADS), 0, s, G, n_keys,
                     nb, parts, (uint32_t)KB_SW_TILE, kw.counts, kw.sr, kw.part_acc, kw.arrive,
                     kw.faults, out[0], out[1]);
  if (NA >= 2 && n > 0)  // (few workgroups: each adds to one arrival counter; the list is short)
    hipLaunchKernelGGL(kb_escape, dim3(KB_ESC_WG), dim3(256), 0, s, kw.esc_n, kw.esc_row, kw.esc_cpu,
                       kw.esc_mem, out[0], out[1]);
  return hipGetLastError();
}

template <int NA>
static hipError_t run_bucketed(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* const* in,
                               uint64_t* const* out, const KeyedWork& kw, hipStream_t s) {
  const int nb = (int)keyed_buckets(n_keys);
  if (n == 0) {
    hipError_t e = hipMemsetAsync(kw.tot, 0, sizeof(uint32_t) * (size_t)nb, s);
    if (e != hipSuccess) return e;
  } else {
    const int64_t tile = keyed_tile(n), G = keyed_tiles(n);
    hipLaunchKernelGGL(kb_hist, dim3((unsigned)G), dim3(KB_HIST_THREADS), nb * sizeof(uint32_t), s, n,
                       n_keys, key, nb, kw.counts, tile);
    hipLaunchKernelGGL(kb_scan, dim3((unsigned)nb), dim3(KB_SCAN_THREADS), 0, s, G, nb, kw.counts,
                       kw.tot, kw.esc_n);
    hipLaunchKernelGGL(kb_scatter<NA>, dim3((unsigned)G), dim3(KB_HIST_THREADS),
                       (3 * nb + KB_HIST_THREADS) * sizeof(uint32_t), s, n, n_keys, key, in[0], in[1],
                       in[2], in[3], nb, kw.counts, kw.tot, kw.sr, kw.sv, kw.esc_n, kw.esc_row,
                       kw.esc_cpu, kw.esc_mem, tile);
  }
  hipLaunchKernelGGL(kb_accum<NA>, dim3((unsigned)nb), dim3(KB_ACC_THREADS), 0, s, n, n_keys, nb,
                     kw.tot, kw.sr, kw.sv, out[0], out[1], out[2], out[3]);
  if (NA >= 2 && n > 0)
    hipLaunchKernelGGL(kb_escape, dim3(KB_ESC_WG), dim3(256), 0, s, kw.esc_n, kw.esc_row, kw.esc_cpu,
                       kw.esc_mem, out[0], out[1]);
  return hipGetLastError();
}

hipError_t launch_reduce_keyed(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* cpu,
                               const int64_t* mem, const uint64_t* cpul, const int64_t* meml,
                               uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                               int64_t* lim_mem, const KeyedWork* kw, hipStream_t s) {
  if (kw && keyed_bucketed(n_keys, n)) {
    const uint64_t* in[4] = {cpu, reinterpret_cast<const uint64_t*>(mem), cpul,
                             reinterpret_cast<const uint64_t*>(meml)};
    uint64_t* out[4] = {used_cpu, reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                        reinterpret_cast<uint64_t*>(lim_mem)};
    if (cpul) return run_bucketed<4>(n_keys, n, key, in, out, *kw, s);
    return run_sweep<2>(n_keys, n, key, in, out, *kw, s);
  }
  if (n_keys > 0) {  // the sums start from zero (CC:257-260)
    hipError_t e = hipMemsetAsync(used_cpu, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess) e = hipMemsetAsync(used_mem, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess && cpul) e = hipMemsetAsync(lim_cpu, 0, 8 * (size_t)n_keys, s);
    if (e == hipSuccess && cpul) e = hipMemsetAsync(lim_mem, 0, 8 * (size_t)n_keys, s);
    if (e != hipSuccess) return e;
  }
  if (n <= 0 || n_keys <= 0) return hipSuccess;
  const int64_t grid = (n + KY_BLOCK - 1) / KY_BLOCK;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  if (cpul)
    hipLaunchKernelGGL(reduce_keyed_kernel<4>, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n,
                       n_keys, key, cpu, reinterpret_cast<const uint64_t*>(mem), cpul,
                       reinterpret_cast<const uint64_t*>(meml), used_cpu,
                       reinterpret_cast<uint64_t*>(used_mem), lim_cpu,
                       reinterpret_cast<uint64_t*>(lim_mem));
  else
    hipLaunchKernelGGL(reduce_keyed_kernel<2>, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n,
                       n_keys, key, cpu, reinterpret_cast<const uint64_t*>(mem), nullptr, nullptr,
                       used_cpu, reinterpret_cast<uint64_t*>(used_mem), nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_count_keyed(int64_t n_keys, int64_t n, const int32_t* key, int64_t* count,
                              const KeyedWork* kw, hipStream_t s) {
  if (kw && keyed_bucketed(n_keys, n)) {
    const uint64_t* in[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t* out[4] = {reinterpret_cast<uint64_t*>(count), nullptr, nullptr, nullptr};
    return run_sweep<0>(n_keys, n, key, in, out, *kw, s);
  }
  if (n_keys > 0) {
    hipError_t e = hipMemsetAsync(count, 0, 8 * (size_t)n_keys, s);
    if (e != hipSuccess) return e;
  }
  if (n <= 0 || n_keys <= 0) return hipSuccess;
  const int64_t grid = (n + KY_BLOCK - 1) / KY_BLOCK;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(count_keyed_kernel, dim3((unsigned)grid), dim3(KY_THREADS), 0, s, n, n_keys,
                     key, reinterpret_cast<uint64_t*>(count));
  return hipGetLastError();
}

}  // namespace kcc

#ifdef KCC_TIMELINE
// (timeline builds only) copy the keyed kernels' stamps to host[1024][8] and zero them
extern "C" int kcc_debug_timeline_keyed(void* host) {
  static uint64_t zero[1024][8];
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(kcc::kcc_tlk), sizeof(zero)) != hipSuccess) return -3;
  return hipMemcpyToSymbol(HIP_SYMBOL(kcc::kcc_tlk), zero, sizeof(zero)) == hipSuccess ? 0 : -3;
}
#endif
