// valu_probe.hip — issue throughput of the VALU instructions the fit kernel is built
// from, on gfx950, at full occupancy (8 waves per SIMD).  Each kernel runs ITERS
// iterations of 16 independent instructions of one kind (8 chains, no memory traffic
// inside the loop); cycles per wave64 instruction per SIMD =
// elapsed * clock / (wave-instructions per SIMD).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_probe scripts/probe/valu_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int ITERS = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define DECL(T, init)                                                                  \
  T v0 = (T)(init), v1 = (T)(init + 1), v2 = (T)(init + 2), v3 = (T)(init + 3),        \
    v4 = (T)(init + 4), v5 = (T)(init + 5), v6 = (T)(init + 6), v7 = (T)(init + 7);
#define SUM (v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7)

__global__ __launch_bounds__(256) void k_fma_f64(double* out, double a, double b) {
  DECL(double, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v##k) : "s"(a), "v"(b));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM;
}

__global__ __launch_bounds__(256) void k_mul_f64(double* out, double a, double b) {
  DECL(double, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(v##k) : "s"(a));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_min_f64(double* out, double a, double b) {
  DECL(double, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_min_f64 %0, %1, %0" : "+v"(v##k) : "v"(b));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a;
}

__global__ __launch_bounds__(256) void k_cmp_f64(double* out, double a, double b) {
  DECL(double, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_cmp_nle_f64_e64 s[2:3], %0, %1" ::"s"(a), "v"(v##k) : "s2", "s3");
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_mul_f32(double* out, double a, double b) {
  float fa = (float)a;
  DECL(float, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(v##k) : "s"(fa));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_pk_mul_f32(double* out, double a, double b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 s = {(float)a, (float)a};
  f2 v0 = {(float)threadIdx.x, 1.f}, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4,
     v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(v##k) : "s"(s));
    REP8(F) REP8(F)
#undef F
  }
  f2 t = SUM;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y + b;
}

__global__ __launch_bounds__(256) void k_add_u32(double* out, double a, double b) {
  uint32_t sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v##k) : "s"(sa));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_min3_u32(double* out, double a, double b) {
  uint32_t sa = (uint32_t)a;
  uint32_t w = threadIdx.x * 7u;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_min3_u32 %0, %1, %2, %0" : "+v"(v##k) : "s"(sa), "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_cmp_u32(double* out, double a, double b) {
  uint32_t sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_cmp_eq_u32_e64 s[2:3], %0, %1" ::"s"(sa), "v"(v##k) : "s2", "s3");
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_cndmask(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u;
  DECL(uint32_t, threadIdx.x)
  asm volatile("v_cmp_gt_u32 vcc, 64, %0" ::"v"(v0) : "vcc");
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(v##k) : "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a + b;
}

__global__ __launch_bounds__(256) void k_add3_u32(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 5u;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_add3_u32 %0, %1, %1, %0" : "+v"(v##k) : "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a + b;
}

// the fit's current inner step (2 fma_f64, min_f64, cmp_f64, cndmask) and the
// denormal-integer variant (mul_f32, mul_f64, min3_u32, cmp_u32, cndmask), 4 nodes per
// iteration each, plus the accumulate — to time the mix, not just the parts
__global__ __launch_bounds__(256) void k_mix_f64(double* out, double a, double b) {
  double rc = b, rm = b * 0.5, bias = 4503599627370496.0, pb = a;
  uint32_t acc = 0, cl = threadIdx.x, zero = 0;
  for (int i = 0; i < ITERS; ++i) {
#define F(k)                                                                           \
  {                                                                                    \
    double qc, qm, x;                                                                  \
    uint32_t c;                                                                        \
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(qc) : "s"(a), "v"(rc), "v"(bias)); \
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(qm) : "s"(a), "v"(rm), "v"(bias)); \
    asm volatile("v_min_f64 %0, %1, %2" : "=v"(x) : "v"(qc), "v"(qm));                 \
    asm volatile("v_cmp_nle_f64_e32 vcc, %1, %2\n\tv_cndmask_b32 %0, %3, %4, vcc"     \
                 : "=v"(c) : "s"(pb), "v"(x), "v"(cl), "v"(zero) : "vcc");            \
    acc += c;                                                                          \
  }
    F(0) F(1) F(2) F(3)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_mix_denorm(double* out, double a, double b) {
  float rcf = (float)b;
  double rm = b * 0.5;
  uint32_t fc = 12345u, P = 110u, acc = 0, cl = threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#define F(k)                                                                           \
  {                                                                                    \
    float qc;                                                                          \
    double qm;                                                                         \
    uint32_t m3, c;                                                                    \
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(qc) : "s"(fc), "v"(rcf));               \
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(qm) : "s"(a), "v"(rm));                 \
    asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(m3) : "v"(qc), "v"((uint32_t)__double_as_longlong(qm)), "s"(P)); \
    asm volatile("v_cmp_eq_u32_e32 vcc, %1, %2\n\tv_cndmask_b32 %0, %2, %3, vcc"      \
                 : "=v"(c) : "s"(P), "v"(m3), "v"(cl) : "vcc");                         \
    acc += c;                                                                          \
  }
    F(0) F(1) F(2) F(3)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}


__global__ __launch_bounds__(256) void k_cndmask_sgpr(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u;
  DECL(uint32_t, threadIdx.x)
  asm volatile("v_cmp_gt_u32_e64 s[4:5], 64, %0" ::"v"(v0) : "s4", "s5");
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_cndmask_b32_e64 %0, %1, %0, s[4:5]" : "+v"(v##k) : "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a + b;
}

__global__ __launch_bounds__(256) void k_cmp_e32(double* out, double a, double b) {
  uint32_t sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1" ::"s"(sa), "v"(v##k) : "vcc");
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_addc(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u;
  DECL(uint32_t, threadIdx.x)
  asm volatile("v_cmp_gt_u32 vcc, 64, %0" ::"v"(v0) : "vcc");
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_addc_co_u32 %0, s[6:7], %1, %0, vcc" : "+v"(v##k) : "v"(w) : "s6", "s7");
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a + b;
}

__global__ __launch_bounds__(256) void k_min_u32(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_min_u32 %0, %1, %0" : "+v"(v##k) : "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + a + b;
}

__global__ __launch_bounds__(256) void k_mad_u24(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u, sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(v##k) : "s"(sa), "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_mul_u24(double* out, double a, double b) {
  uint32_t sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(v##k) : "s"(sa));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

__global__ __launch_bounds__(256) void k_med3_i32(double* out, double a, double b) {
  uint32_t w = threadIdx.x * 3u, sa = (uint32_t)a;
  DECL(uint32_t, threadIdx.x)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_med3_i32 %0, %1, %2, %0" : "+v"(v##k) : "s"(sa), "v"(w));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b;
}

// denormal operands at full rate?  (the fit would feed integers as f32/f64 denormals)
__global__ __launch_bounds__(256) void k_mul_f32_denorm(double* out, double a, double b) {
  float fa = __uint_as_float(12345u);  // denormal
  DECL(float, threadIdx.x * 0.001f + 1.0f)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(v##k) : "s"(fa));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b + a;
}

__global__ __launch_bounds__(256) void k_mul_f64_denorm(double* out, double a, double b) {
  double da = __longlong_as_double(123456789ll);  // denormal
  DECL(double, threadIdx.x * 0.001 + 1.0)
  for (int i = 0; i < ITERS; ++i) {
#define F(k) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(v##k) : "s"(da));
    REP8(F) REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = SUM + b + a;
}

// packed f32 multiply of two integer-valued f32 denormals (an SGPR pair: two nodes'
// free CPU) by a normal per-lane reciprocal, in round-toward--inf (f32 and f64)
__global__ __launch_bounds__(256) void k_pk_mul_denorm_rd(double* out, double a, double b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 10\n\ts_nop 1" ::: "memory");
  f2 s = {__uint_as_float(96000u), __uint_as_float(12345u)};
  const f2 r = {(float)b, 0.f};
  f2 acc = {0.f, 0.f};
  for (int i = 0; i < ITERS; ++i) {
#define F(k)                                                                         \
  {                                                                                  \
    f2 q;                                                                            \
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(q) : "s"(s), "v"(r)); \
    acc.x = __uint_as_float(__float_as_uint(acc.x) ^ __float_as_uint(q.x));          \
  }
    REP8(F) REP8(F)
#undef F
  }
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 0\n\ts_nop 1" ::: "memory");
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + a;
}

__global__ __launch_bounds__(256) void k_mul_f64_denorm_rd(double* out, double a, double b) {
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 10\n\ts_nop 1" ::: "memory");
  double da = __longlong_as_double(123456789012ll);
  uint32_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
#define F(k)                                                                   \
  {                                                                            \
    double q;                                                                  \
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(q) : "s"(da), "v"(b));          \
    acc ^= (uint32_t)__double_as_longlong(q);                                  \
  }
    REP8(F) REP8(F)
#undef F
  }
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 0\n\ts_nop 1" ::: "memory");
  out[blockIdx.x * 256 + threadIdx.x] = acc + a;
}

typedef void (*kern_t)(double*, double, double);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 32 waves/CU = 8 per SIMD
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * blocks * 256));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct {
    const char* name;
    kern_t k;
    double per_iter;  // units per loop iteration (instructions, or nodes for the mixes)
  } ks[] = {{"v_fma_f64", k_fma_f64, 16},      {"v_mul_f64", k_mul_f64, 16},
            {"v_min_f64", k_min_f64, 16},      {"v_cmp_f64", k_cmp_f64, 16},
            {"v_mul_f32", k_mul_f32, 16},      {"v_pk_mul_f32", k_pk_mul_f32, 16},
            {"v_add_u32", k_add_u32, 16},      {"v_min3_u32", k_min3_u32, 16},
            {"v_cmp_u32", k_cmp_u32, 16},      {"v_cndmask_b32", k_cndmask, 16},
            {"v_add3_u32", k_add3_u32, 16},    {"mix_f64 (per node)", k_mix_f64, 4},
            {"mix_denorm (per node)", k_mix_denorm, 4},
            {"v_cndmask_b32_e64 sgpr-mask", k_cndmask_sgpr, 16}, {"v_cmp_eq_u32_e32", k_cmp_e32, 16},
            {"v_addc_co_u32 (vcc in)", k_addc, 16}, {"v_min_u32", k_min_u32, 16},
            {"v_mad_u32_u24", k_mad_u24, 16}, {"v_mul_u32_u24", k_mul_u24, 16},
            {"v_med3_i32", k_med3_i32, 16}, {"v_mul_f32 denormal", k_mul_f32_denorm, 16},
            {"v_mul_f64 denormal", k_mul_f64_denorm, 16},
            {"v_pk_mul_f32 denormal RD (+v_xor)", k_pk_mul_denorm_rd, 16},
            {"v_mul_f64 denormal RD (+v_xor)", k_mul_f64_denorm_rd, 16}};
  const double clk_ghz = prop.clockRate / 1e6;
  printf("{\"cus\": %d, \"clock_ghz_nominal\": %.3f, \"waves_per_simd\": 8}\n", cus, clk_ghz);
  for (auto& k : ks) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 3.0, 0.5);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 3.0, 0.5);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double per_simd = 8.0 * ITERS * k.per_iter;  // 8 waves per SIMD
    const double cyc = best * 1e-3 * clk_ghz * 1e9 / per_simd;
    printf("{\"what\": \"%s\", \"ms\": %.4f, \"cycles_per_unit_per_SIMD_at_nominal_clock\": %.3f}\n",
           k.name, best, cyc);
  }
  CHECK(hipFree(out));
  return 0;
}
