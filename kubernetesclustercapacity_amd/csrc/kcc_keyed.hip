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
// Two implementations; keys < 0 or >= n_keys are skipped (pods whose
// node is not a listed row):
//  - bucketed (n_keys <= KB_NB_MAX * KB_ROWS, the default): rows are cut into buckets of
//    KB_ROWS; kb_hist counts each tile's containers per bucket (LDS histogram), kb_scan
//    turns the counts into scatter offsets, kb_scatter moves every container's (row in
//    bucket, values) into its bucket's contiguous range (LDS cursors), and kb_accum sums
//    each bucket in LDS (64-bit LDS atomics) and writes its rows once.  No global
//    atomics; ~64 B of HBM traffic per container.
//  - direct atomics (fallback): each lane takes KY_IPL consecutive containers, merges
//    runs of equal keys in registers (a pod's containers are consecutive in a List) and
//    issues one 64-bit device atomic per array and run — device-scope atomics to random
//    rows execute past the L2s at ~14 G/s, so this is the slow path.
#include "kcc_internal.h"

namespace kcc {
namespace {

constexpr int KY_THREADS = 256;
constexpr int KY_IPL = 4;                             // containers per lane
constexpr int KY_BLOCK = KY_THREADS * KY_IPL;         // containers per workgroup

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

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
                                                           uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t kb_h[];
  for (int b = threadIdx.x; b < nb; b += KB_HIST_THREADS) kb_h[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * KB_TILE;
  const int64_t t1 = min(t0 + (int64_t)KB_TILE, n);
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
                                                          uint32_t* __restrict__ tot) {
  __shared__ uint32_t sh[KB_SCAN_THREADS];
  const int b = blockIdx.x;
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

// tile g: every valid container to its bucket's range (row in bucket, values).  The tile
// goes in sub-chunks of KB_SUB: each element's rank within its bucket (LDS counters),
// a scan of the sub-chunk's bucket counts, and a counting sort into an LDS stage, so that
// the global writes leave in bucket order — a bucket's elements of one sub-chunk land on
// consecutive addresses (its range in the bucket is this workgroup's, contiguous), and a
// wave's stores coalesce instead of touching 64 lines.
// sub-chunk size by value count: the stage (NA x 8 B + 6 B per element) plus up to 51 KB
// of bucket cursors must fit 160 KB of LDS (4096: 0.38 ms at C4 vs 0.46 ms for 2048)
constexpr int kb_sub(int na) { return na > 2 ? 2048 : 4096; }

template <int NA>
__global__ __launch_bounds__(KB_HIST_THREADS) void kb_scatter(
    int64_t n, int64_t n_keys, const int32_t* __restrict__ key, const uint64_t* __restrict__ a0,
    const uint64_t* __restrict__ a1, const uint64_t* __restrict__ a2, const uint64_t* __restrict__ a3,
    int nb, const uint32_t* __restrict__ counts, const uint32_t* __restrict__ tot,
    uint16_t* __restrict__ sk, uint64_t* __restrict__ sv) {
  constexpr int NS = NA > 0 ? NA : 1;
  constexpr int KB_SUB = kb_sub(NA);
  constexpr int KB_SUB_PER = KB_SUB / KB_HIST_THREADS;
  // dynamic LDS: cur[nb], lcnt[nb], lstart[nb], scan scratch[KB_HIST_THREADS]
  extern __shared__ uint32_t kb_dyn[];
  uint32_t* cur = kb_dyn;
  uint32_t* lcnt = cur + nb;
  uint32_t* lstart = lcnt + nb;
  uint32_t* sh = lstart + nb;
  __shared__ uint64_t st_v[NS][KB_SUB];
  __shared__ uint32_t st_pos[KB_SUB];
  __shared__ uint16_t st_k[KB_SUB];
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
  const int64_t t0 = (int64_t)blockIdx.x * KB_TILE;
  const int64_t t1 = min(t0 + (int64_t)KB_TILE, n);
  // sub-chunk loads run one sub-chunk ahead: issued before this one's scan, stage and
  // writes, consumed at the top of the next iteration
  int32_t kn[KB_SUB_PER];
  uint64_t vn[NS][KB_SUB_PER];
  auto load_sub = [&](int64_t c0) {
#pragma unroll
    for (int u = 0; u < KB_SUB_PER; ++u) {
      const int64_t c = c0 + (int64_t)u * KB_HIST_THREADS + threadIdx.x;
      const bool ok = c < t1;
      kn[u] = ok ? __builtin_nontemporal_load(key + c) : -1;
#pragma unroll
      for (int a = 0; a < NA; ++a) vn[a][u] = ok ? __builtin_nontemporal_load(in[a] + c) : 0;
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
      st_pos[slot] = cur[b] + rk[u];
      st_k[slot] = (uint16_t)(k[u] & (KB_ROWS - 1));
#pragma unroll
      for (int a = 0; a < NA; ++a) st_v[a][slot] = v[a][u];
    }
    __syncthreads();
    const uint32_t nvalid = sh[KB_HIST_THREADS - 1];  // total of the lcnt scan
    for (uint32_t j = threadIdx.x; j < nvalid; j += KB_HIST_THREADS) {
      const uint32_t pos = st_pos[j];
      sk[pos] = st_k[j];
#pragma unroll
      for (int a = 0; a < NA; ++a) sv[(int64_t)pos * NA + a] = st_v[a][j];  // element-major
    }
    __syncthreads();  // nvalid read, stage drained before the counters change
    for (int b = b0; b < b1; ++b) {  // advance the cursors, clear the sub-chunk counts
      cur[b] += lcnt[b];
      lcnt[b] = 0;
    }
    __syncthreads();
  }
}

// bucket b: its range summed per row in LDS, rows [b * KB_ROWS, ...) written once
// (NA == 0: counts the containers per row)
template <int NA>
__global__ __launch_bounds__(KB_ACC_THREADS) void kb_accum(
    int64_t n, int64_t n_keys, int nb, const uint32_t* __restrict__ tot,
    const uint16_t* __restrict__ sk, const uint64_t* __restrict__ sv, uint64_t* __restrict__ o0,
    uint64_t* __restrict__ o1, uint64_t* __restrict__ o2, uint64_t* __restrict__ o3) {
  constexpr int NACC = NA > 0 ? NA : 1;
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
  for (int64_t i0 = (int64_t)start + threadIdx.x; i0 < (int64_t)end;
       i0 += KB_ACC_THREADS * KB_UNROLL) {  // 64-bit: end may be close to 2^32
    uint32_t r[KB_UNROLL];
    uint64_t v[NACC][KB_UNROLL];
#pragma unroll
    for (int u = 0; u < KB_UNROLL; ++u) {
      const int64_t i = i0 + (int64_t)u * KB_ACC_THREADS;
      const bool ok = i < end;
      r[u] = ok ? (uint32_t)__builtin_nontemporal_load(sk + i) : 0xffffffffu;
#pragma unroll
      for (int a = 0; a < NACC; ++a)
        v[a][u] = NA == 0 ? 1ull : (ok ? __builtin_nontemporal_load(sv + i * NA + a) : 0ull);
    }
#pragma unroll
    for (int u = 0; u < KB_UNROLL; ++u)
      if (r[u] != 0xffffffffu)
#pragma unroll
        for (int a = 0; a < NACC; ++a) atomicAdd(&acc[a][r[u]], (unsigned long long)v[a][u]);
  }
  __syncthreads();
  const int64_t row0 = (int64_t)b * KB_ROWS;
  for (int r = threadIdx.x; r < KB_ROWS; r += KB_ACC_THREADS) {
    if (row0 + r >= n_keys) break;
#pragma unroll
    for (int a = 0; a < NACC; ++a) out[a][row0 + r] = acc[a][r];
  }
}

}  // namespace

int64_t keyed_tiles(int64_t n) { return (n + KB_TILE - 1) / KB_TILE; }
int64_t keyed_buckets(int64_t n_keys) { return (n_keys + KB_ROWS - 1) / KB_ROWS; }
bool keyed_bucketed(int64_t n_keys, int64_t n) {
  return n_keys > 0 && keyed_buckets(n_keys) <= KB_NB_MAX && n < ((int64_t)1 << 32);
}

template <int NA>
static hipError_t run_bucketed(int64_t n_keys, int64_t n, const int32_t* key, const uint64_t* const* in,
                               uint64_t* const* out, const KeyedWork& kw, hipStream_t s) {
  const int nb = (int)keyed_buckets(n_keys);
  const int64_t G = keyed_tiles(n);
  if (n > 0) {
    hipLaunchKernelGGL(kb_hist, dim3((unsigned)G), dim3(KB_HIST_THREADS), nb * sizeof(uint32_t), s, n,
                       n_keys, key, nb, kw.counts);
    hipLaunchKernelGGL(kb_scan, dim3((unsigned)nb), dim3(KB_SCAN_THREADS), 0, s, G, nb, kw.counts,
                       kw.tot);
    hipLaunchKernelGGL(kb_scatter<NA>, dim3((unsigned)G), dim3(KB_HIST_THREADS),
                       (3 * nb + KB_HIST_THREADS) * sizeof(uint32_t), s, n, n_keys, key, in[0], in[1],
                       in[2], in[3], nb, kw.counts, kw.tot, kw.sk, kw.sv);
  } else {
    hipError_t e = hipMemsetAsync(kw.tot, 0, sizeof(uint32_t) * (size_t)nb, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kb_accum<NA>, dim3((unsigned)nb), dim3(KB_ACC_THREADS), 0, s, n, n_keys, nb,
                     kw.tot, kw.sk, kw.sv, out[0], out[1], out[2], out[3]);
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
    return cpul ? run_bucketed<4>(n_keys, n, key, in, out, *kw, s)
                : run_bucketed<2>(n_keys, n, key, in, out, *kw, s);
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
    return run_bucketed<0>(n_keys, n, key, in, out, *kw, s);
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
