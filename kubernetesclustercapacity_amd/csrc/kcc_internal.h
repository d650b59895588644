// kcc_internal.h — launch interface between the C-ABI layer (kcc_abi.cpp) and the
// gfx950 kernels (kcc_kernels.hip).  Internal: not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kcc {

// ---- (a) segmented request reduce -------------------------------------------
// One wavefront owns a contiguous range of reduce_range() containers and walks it in
// tiles of RED_TILE (RED_IPL containers per lane: two 16-B loads per lane per array).
#ifndef KCC_RED_TILES_PER_WAVE
#define KCC_RED_TILES_PER_WAVE 16  // longest wave range (tiles)
#endif
#ifndef KCC_RED_TARGET_WAVES
#define KCC_RED_TARGET_WAVES 8192  // shorten ranges until this many waves exist
#endif
#ifndef KCC_RED_PREFETCH
#define KCC_RED_PREFETCH 1  // tiles in flight ahead of the one being reduced (1 or 2)
#endif
constexpr int RED_IPL = 4;
constexpr int RED_TILE = 64 * RED_IPL;  // 256
constexpr int RED_TILES_PER_WAVE = KCC_RED_TILES_PER_WAVE;
constexpr int RED_WAVES_PER_BLOCK = 4;

// Containers per wave range: whole tiles, long (<= 16 tiles) for big inputs, short
// enough for small ones (a node shard of an 8-GPU run) that ~KCC_RED_TARGET_WAVES
// waves exist and every SIMD has several in flight.
inline int32_t reduce_range(int64_t n_containers) {
  int64_t t = (n_containers + (int64_t)RED_TILE * KCC_RED_TARGET_WAVES - 1) /
              ((int64_t)RED_TILE * KCC_RED_TARGET_WAVES);
  if (t < 1) t = 1;
  if (t > RED_TILES_PER_WAVE) t = RED_TILES_PER_WAVE;
  return (int32_t)(t * RED_TILE);
}
inline int64_t reduce_n_waves(int64_t n_containers) {
  const int64_t r = reduce_range(n_containers);
  return (n_containers + r - 1) / r;
}
// workspace bound for wave_node (shortest range)
inline int64_t reduce_max_waves(int64_t n_containers) {
  return (n_containers + RED_TILE - 1) / RED_TILE + 1;
}

// Zeroes the per-node outputs and records, for every wave range, the node that owns
// the range's first container (wave_node[n_waves]).
hipError_t launch_reduce_mark(int64_t n_nodes, int64_t n_containers, const int64_t* node_ptr,
                              int64_t* wave_node, uint64_t* used_cpu, int64_t* used_mem,
                              uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s);

hipError_t launch_reduce(int64_t n_nodes, int64_t n_containers, const int64_t* node_ptr,
                         const uint64_t* cpu_req, const int64_t* mem_req,
                         const uint64_t* cpu_lim, const int64_t* mem_lim,
                         const int64_t* wave_node, uint64_t* used_cpu, int64_t* used_mem,
                         uint64_t* lim_cpu, int64_t* lim_mem, hipStream_t s);

// ---- (b) fit -----------------------------------------------------------------
// Node stream of the fit kernel: groups of FIT_GROUP nodes, field-major inside the
// group (224 B).  fc/fm/Pb arrive through the scalar cache (SGPR operands of the VALU),
// cl by one uniform-address vector load (it is a v_cndmask operand, and gfx9 allows a
// single SGPR/VCC read per VALU instruction).  Rows outside the fast-path bounds, and
// the padding of the last group, hold all-zero fields (contribute exactly 0: x' = 2^52
// >= Pb = 0 selects cl = 0) and are listed in slow_list for the exact path.
constexpr int FIT_GROUP = 8;
constexpr double FIT_BIAS = 4503599627370496.0;  // 2^52: integers in [2^52, 2^53) have ulp 1
struct __attribute__((aligned(32))) FitGroup {
  double fc[FIT_GROUP];   // free CPU (millicores), exact in f64 on the fast path (< 2^50)
  double fm[FIT_GROUP];   // free memory (bytes), exact in f64 on the fast path (< 2^50)
  double Pb[FIT_GROUP];   // 2^52 + allocatable pods (|P| <= 2^20: exact), the biased compare operand
  int32_t cl[FIT_GROUP];  // clamp value allocatable pods - podCount (CC:135)
};
static_assert(sizeof(FitGroup) == 224, "FitGroup must be 224 B");
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

// One 32-B record per spec, in the kernel's internal (partitioned) order: specs that
// satisfy the fast-path bounds first, the rest after (so at most one wavefront mixes
// both).  rc == 0 marks a spec for the exact path (a fast-path rc is > 0).
struct __attribute__((aligned(32))) SpecRec {
  uint64_t c;    // cpu request (millicores)
  int64_t m;     // memory request (bytes)
  double rc;     // smallest f64 >= 1/c (see fit_kernel); 0 marks a spec off the fast path
  double rm;     // smallest f64 >= 1/m
};
static_assert(sizeof(SpecRec) == 32, "SpecRec must be 32 B");

struct SpecPrep {
  SpecRec* rec;
  int32_t* perm;  // internal index -> caller index
};

// counters: [0] (node, spec) pairs on the exact path, [1] rows in slow_list.
// spec_prep zeroes partial[0..2S) and counters[0..1]; node_prep appends to slow_list.
hipError_t launch_spec_prep(int64_t n_specs, const uint64_t* spec_cpu,
                            const int64_t* spec_mem, SpecPrep sp, int64_t* partial,
                            unsigned long long* counters, hipStream_t s);

hipError_t launch_node_prep(int64_t n_nodes, const uint64_t* alloc_cpu,
                            const int64_t* alloc_mem, const int64_t* alloc_pods,
                            const int64_t* pod_count, const uint64_t* used_cpu,
                            const int64_t* used_mem, FitGroup* fast, SlowNode* slow,
                            int64_t* slow_list, unsigned long long* counters, hipStream_t s);

// partial[0..S) += Σ_i q(i,s), partial[S..2S) += #div-by-zero rows (internal order).
hipError_t launch_fit(int64_t n_nodes, const FitGroup* fast, const SlowNode* slow,
                      const int64_t* slow_list, int64_t n_specs, SpecPrep sp, int64_t* partial,
                      unsigned long long* counters, hipStream_t s);

hipError_t launch_fit_finalize(int64_t n_specs, const int64_t* partial,
                               const int32_t* perm, int64_t* totals, int32_t* spec_err,
                               hipStream_t s);

}  // namespace kcc
