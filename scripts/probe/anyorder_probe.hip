// Diagnostic: can two kernels of one stream overlap on gfx950?  Kernel A (a few
// workgroups spinning ~30 us) then kernel B launched (1) plainly, (2) with
// hipExtAnyOrderLaunch (the AQL barrier bit cleared), (3) on a second stream of higher
// priority; then kernel C plainly.  Each workgroup stamps its start and end
// (s_memrealtime, 100 MHz).  Overlap = B's first start before A's last end.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/anyorder_probe scripts/probe/anyorder_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__global__ void spin(uint64_t* t, int work, uint32_t* sink, const uint32_t* flag) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x + (flag ? flag[0] : 0u);
  for (int i = 0; i < work; ++i) a = a * 1664525u + 1013904223u;
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x] = t0;
    t[2 * blockIdx.x + 1] = t1;
  }
  if (a == 0x12345u) sink[0] = a;
}

struct Span {
  uint64_t first_start, last_start, first_end, last_end;
};
static Span span(const std::vector<uint64_t>& h, int g) {
  Span s{~0ull, 0, ~0ull, 0};
  for (int i = 0; i < g; ++i) {
    s.first_start = std::min(s.first_start, h[2 * i]);
    s.last_start = std::max(s.last_start, h[2 * i]);
    s.first_end = std::min(s.first_end, h[2 * i + 1]);
    s.last_end = std::max(s.last_end, h[2 * i + 1]);
  }
  return s;
}

static std::vector<uint64_t> get(const uint64_t* d, int g) {
  std::vector<uint64_t> h(2 * g);
  (void)hipMemcpy(h.data(), d, 8 * 2 * g, hipMemcpyDeviceToHost);
  return h;
}

int main() {
  uint64_t* t[4];
  for (auto& p : t) (void)hipMalloc(&p, 8 * 2 * 4096);
  uint32_t* sink;
  (void)hipMalloc(&sink, 4);
  hipStream_t s0, s1;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  (void)hipStreamCreateWithPriority(&s0, hipStreamNonBlocking, lo);
  (void)hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, hi);
  hipEvent_t e1, e2;
  (void)hipEventCreateWithFlags(&e1, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&e2, hipEventDisableTiming);
  printf("stream priorities: least %d greatest %d\n", lo, hi);
  // part 1: A (64 WGs, ~30 us) then B (512 WGs, ~10 us): plain / any-order / second stream
  const int ga = 64, gb = 512, wa = 1800, wb = 600;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL(spin, dim3(ga), dim3(256), 0, s0, t[0], wa, sink, nullptr);
      if (mode == 0)
        hipLaunchKernelGGL(spin, dim3(gb), dim3(256), 0, s0, t[1], wb, sink, nullptr);
      else if (mode == 1)
        hipExtLaunchKernelGGL(spin, dim3(gb), dim3(256), 0, s0, nullptr, nullptr,
                              hipExtAnyOrderLaunch, t[1], wb, sink, (const uint32_t*)nullptr);
      else
        hipLaunchKernelGGL(spin, dim3(gb), dim3(256), 0, s1, t[1], wb, sink, nullptr);
      hipLaunchKernelGGL(spin, dim3(ga), dim3(256), 0, s0, t[2], wb, sink, nullptr);
      (void)hipDeviceSynchronize();
    }
    const Span A = span(get(t[0], ga), ga), B = span(get(t[1], gb), gb), C = span(get(t[2], ga), ga);
    const double z = (double)A.first_start;
    printf("%-22s A [0, first end %7.2f, last end %7.2f] us  B [%7.2f .. %7.2f, end %7.2f]  C start %7.2f\n",
           mode == 0 ? "plain" : mode == 1 ? "hipExtAnyOrderLaunch" : "second stream (prio)",
           (A.first_end - z) / 100.0, (A.last_end - z) / 100.0, (B.first_start - z) / 100.0,
           (B.last_start - z) / 100.0, (B.last_end - z) / 100.0, (C.first_start - z) / 100.0);
  }
  // part 2: the fork/join a step would use.  s0: K1 -> [e1] ; s1: wait e1, K2 -> [e2] ;
  // s0: K3 ; wait e2 ; K4.   K2 || K3 expected; gaps = starts minus the producers' ends.
  for (int mode = 0; mode < 2; ++mode) {
    double g2 = 0, g3 = 0, g4 = 0, tot = 0;
    const int reps = 8;
    for (int rep = 0; rep < reps + 2; ++rep) {
      hipLaunchKernelGGL(spin, dim3(256), dim3(256), 0, s0, t[0], 600, sink, nullptr);
      if (mode == 1) {
        (void)hipEventRecord(e1, s0);
        (void)hipStreamWaitEvent(s1, e1, 0);
        hipLaunchKernelGGL(spin, dim3(256), dim3(1024), 0, s1, t[1], 600, sink, nullptr);
        (void)hipEventRecord(e2, s1);
      } else {
        hipLaunchKernelGGL(spin, dim3(256), dim3(1024), 0, s0, t[1], 600, sink, nullptr);
      }
      hipLaunchKernelGGL(spin, dim3(512), dim3(256), 0, s0, t[2], 1200, sink, nullptr);
      if (mode == 1) (void)hipStreamWaitEvent(s0, e2, 0);
      hipLaunchKernelGGL(spin, dim3(64), dim3(256), 0, s0, t[3], 60, sink, nullptr);
      (void)hipDeviceSynchronize();
      if (rep < 2) continue;
      const Span K1 = span(get(t[0], 256), 256), K2 = span(get(t[1], 256), 256),
                 K3 = span(get(t[2], 512), 512), K4 = span(get(t[3], 64), 64);
      g2 += ((double)K2.first_start - (double)K1.last_end) / 100.0;
      g3 += ((double)K3.first_start - (double)K1.last_end) / 100.0;
      g4 += ((double)K4.first_start - (double)std::max(K2.last_end, K3.last_end)) / 100.0;
      tot += ((double)K4.last_end - (double)K1.first_start) / 100.0;
    }
    printf("%-26s K2 start - K1 end %6.2f us, K3 start - K1 end %6.2f us, K4 start - max(K2, K3 end) %6.2f us, K1 start..K4 end %7.2f us\n",
           mode == 0 ? "one stream (serial)" : "fork/join over 2 streams", g2 / reps, g3 / reps,
           g4 / reps, tot / reps);
  }
  return 0;
}
