// cluster_capacity — C++ mirror of the reference's main() (CC:48-150) over libkcc.
//
// Same flags, parsing, error exits and verdict text as
// src/KubeAPI/ClusterCapacity.go; the node/pod listing comes from a cluster file
// (-cluster) instead of client-go, and the two hot loops (CC:262-294, CC:105-140) run
// on the GPU through the C-ABI (kcc_capacity).  Additions: -specs <file> (a batch of
// what-if specs, one "cpuRequests memRequests replicas" per line), -v (per-node
// report of CC:107-117/137), -device/-gpus.
#include <cctype>
#include <cerrno>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "kcc.h"
#include "kcc_host.hpp"

using namespace kcchost;

namespace {

const char* kInvalidBytes =
    "byte quantity must be a positive integer with a unit of measurement like M, MB, MiB, G, "
    "GiB, or GB";
const char* kRule =
    "==============================================================================================================";

struct Flags {
  std::map<std::string, std::string> v = {
      {"kubeconfig", ""},         {"cluster", ""},          {"cpuRequests", "100m"},
      {"cpuLimits", "200m"},      {"memRequests", "100mb"}, {"memLimits", "200mb"},
      {"replicas", "1"},          {"specs", ""},            {"device", "0"},
      {"gpus", "1"},              {"v", "false"},           {"schedulerRequests", "false"}};
};

// Go flag package syntax: -name=value, -name value, --name=value; bool -v.
bool parseFlags(int argc, char** argv, Flags& f) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.size() < 2 || a[0] != '-') {
      std::fprintf(stderr, "unexpected argument %s\n", a.c_str());
      return false;
    }
    a = a.substr(a[1] == '-' ? 2 : 1);
    std::string name = a, val;
    const size_t eq = a.find('=');
    bool has = false;
    if (eq != std::string::npos) {
      name = a.substr(0, eq);
      val = a.substr(eq + 1);
      has = true;
    }
    if (!f.v.count(name)) {
      std::fprintf(stderr, "flag provided but not defined: -%s\n", name.c_str());
      return false;
    }
    if ((name == "v" || name == "schedulerRequests") && !has) {
      val = "true";
    } else if (!has) {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "flag needs an argument: -%s\n", name.c_str());
        return false;
      }
      val = argv[++i];
    }
    f.v[name] = val;
  }
  return true;
}

struct Spec {
  std::string cpuStr, memStr, repStr;
  uint64_t cpu = 0;
  int64_t mem = 0, replicas = 0;
};

bool goAtoiStrict(const std::string& s, int64_t& out) {
  char* end = nullptr;
  errno = 0;
  if (s.empty()) return false;
  const long long v = std::strtoll(s.c_str(), &end, 10);
  if (errno || *end || std::isspace((unsigned char)s[0])) return false;
  out = v;
  return true;
}

// CC:64-83: parse one spec exactly like the flags; exits like the reference on error.
// Go fmt "%.2f" (CC:117): NaN prints "NaN" and infinities "+Inf" / "-Inf" (an
// unhealthy node's zero row divides 0 by 0, CC:112-115); finite values format like C's.
std::string goF2(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "+Inf" : "-Inf";
  char b[64];
  std::snprintf(b, sizeof b, "%.2f", x);
  return b;
}

void parseSpec(Spec& s, bool verbose_errors) {
  s.cpu = convertCPUToMilis(s.cpuStr);
  const auto mem = ToBytes(s.memStr);
  if (!mem.second) {
    std::printf("ERROR : Invalid input memRequests = %" PRId64 " %s ...exiting\n", mem.first,
                kInvalidBytes);
    std::exit(1);
  }
  s.mem = mem.first;
  if (!goAtoiStrict(s.repStr, s.replicas)) {
    std::printf("ERROR : Invalid input replicas = 0 strconv.Atoi: parsing \"%s\": invalid syntax "
                "...exiting\n", s.repStr.c_str());
    std::exit(1);
  }
  (void)verbose_errors;
}

int fail(kcc_ctx* ctx, int rc) {
  std::fprintf(stderr, "kcc error %d: %s\n", rc, ctx ? kcc_last_error(ctx) : kcc_create_error());
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  Flags f;
  if (!parseFlags(argc, argv, f)) return 2;
  const bool verbose = f.v["v"] == "true";
  // opt-in (NOT the reference's semantics): pod requests as the
  // scheduler counts them — init containers, sidecars, overhead
  const bool schedReq = f.v["schedulerRequests"] == "true";

  Spec one{f.v["cpuRequests"], f.v["memRequests"], f.v["replicas"]};
  const uint64_t cpuLimits = convertCPUToMilis(f.v["cpuLimits"]);            // CC:65
  parseSpec(one, true);                                                      // CC:64, 67-71, 79-83
  const auto memLim = ToBytes(f.v["memLimits"]);                             // CC:73-77
  if (!memLim.second) {
    std::printf("ERROR : Invalid input memLimits = %" PRId64 " %s ...exiting\n", memLim.first,
                kInvalidBytes);
    return 1;
  }
  std::printf("\nCPU limits, requests, Memory limits, requests and replicas parsed from input : "
              "%" PRIu64 " %" PRIu64 " %" PRId64 " %" PRId64 " %" PRId64 "\n",
              cpuLimits, one.cpu, memLim.first, one.mem, one.replicas);  // CC:85

  std::vector<Spec> specs;
  if (!f.v["specs"].empty()) {
    std::ifstream sf(f.v["specs"]);
    if (!sf) {
      std::fprintf(stderr, "cannot open spec file %s\n", f.v["specs"].c_str());
      return 1;
    }
    std::string line;
    while (std::getline(sf, line)) {
      std::istringstream is(line);
      Spec s;
      if (!(is >> s.cpuStr >> s.memStr >> s.repStr) || s.cpuStr[0] == '#') continue;
      parseSpec(s, false);
      specs.push_back(s);
    }
  } else {
    specs.push_back(one);
  }

  // cluster access (CC:88-99): a cluster file replaces kubeconfig + client-go
  const std::string path = !f.v["cluster"].empty() ? f.v["cluster"] : f.v["kubeconfig"];
  if (path.empty()) {
    std::fprintf(stderr, "no cluster: pass -cluster <file> (client-go is not part of this build)\n");
    return 1;
  }
  Cluster cl;
  std::string err;
  if (!loadCluster(path, cl, err)) {
    std::fprintf(stderr, "panic: %s\n", err.c_str());
    return 2;
  }
  kcc_ctx* ctx = nullptr;
  int rc = kcc_create(&ctx, std::atoi(f.v["device"].c_str()), std::atoi(f.v["gpus"].c_str()));
  if (rc) return fail(nullptr, rc);
  std::vector<node> rows;
  rc = getHealthyNodes(ctx, cl, rows);  // node cpu / memory strings parsed on the device
  if (rc) return fail(ctx, rc);
  EngineInputs in;
  rc = buildInputs(ctx, cl, rows, in);  // container cpu strings parsed on the device
  if (rc) return fail(ctx, rc);
  const int64_t n = (int64_t)rows.size(), nc = (int64_t)in.cpu_req.size();

  // -schedulerRequests: the per-node request sums of the opt-in model, fed to the fit
  std::vector<uint64_t> suc;
  std::vector<int64_t> sum_;
  if (schedReq) {
    suc.resize((size_t)n);
    sum_.resize((size_t)n);
    const int64_t np = (int64_t)in.ovh_cpu.size(), ni = (int64_t)in.init_mem.size();
    rc = kcc_reduce_requests_pods(ctx, n, np, nc, ni, in.node_pod_ptr.data(), in.pod_ptr.data(),
                                  in.cpu_req.data(), in.mem_req.data(), in.init_ptr.data(),
                                  ni ? in.init_cpu.data() : nullptr,
                                  ni ? in.init_mem.data() : nullptr,
                                  ni ? in.init_rst.data() : nullptr,
                                  np ? in.ovh_cpu.data() : nullptr,
                                  np ? in.ovh_mem.data() : nullptr, suc.data(), sum_.data());
    if (rc) return fail(ctx, rc);
  }

  if (verbose) {  // CC:107-117, 137 — per-node sums and fit, one row at a time
    std::vector<uint64_t> uc(n), lc(n);
    std::vector<int64_t> um(n), lm(n);
    rc = kcc_reduce_requests(ctx, n, nc, in.node_ptr.data(), in.cpu_req.data(), in.mem_req.data(),
                             in.cpu_lim.data(), in.mem_lim.data(), uc.data(), um.data(), lc.data(),
                             lm.data());
    if (rc) return fail(ctx, rc);
    if (schedReq) {
      uc = suc;
      um = sum_;
    }
    // every row's "Max replicas" (CC:137) for the first spec in one device call
    std::vector<int64_t> qs(n);
    std::vector<int32_t> es(n);
    rc = kcc_fit_rows(ctx, n, in.alloc_cpu.data(), in.alloc_mem.data(), in.alloc_pods.data(),
                      in.pod_count.data(), uc.data(), um.data(), specs[0].cpu, specs[0].mem,
                      qs.data(), es.data());
    if (rc) return fail(ctx, rc);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t q = qs[i];
      const int32_t e = es[i];
      std::printf("\n{%s %" PRIu64 " %" PRId64 " %" PRId64 "} - Current non-terminated pods : %" PRId64,
                  rows[i].name.c_str(), rows[i].allocatableCPU, rows[i].allocatableMemory,
                  rows[i].allocatablePods, in.pod_count[i]);
      std::printf("\nSum of CPU Limits, Requests and Memory Limits, Requests for all pods : %" PRIu64
                  " %" PRIu64 " %" PRId64 " %" PRId64, lc[i], uc[i], lm[i], um[i]);
      std::printf("\nTotal allocatbale CPU and Memory : %" PRIu64 ", %" PRId64, rows[i].allocatableCPU,
                  rows[i].allocatableMemory);
      const double ac = (double)rows[i].allocatableCPU, am = (double)rows[i].allocatableMemory;
      std::printf("\nCPU Limits, Requests and Memory Limits, Requests used percentage till now : "
                  "%s %s %s %s", goF2((double)lc[i] * 100 / ac).c_str(),
                  goF2((double)uc[i] * 100 / ac).c_str(), goF2((double)lm[i] * 100 / am).c_str(),
                  goF2((double)um[i] * 100 / am).c_str());
      if (e) {
        std::fprintf(stderr, "panic: runtime error: integer divide by zero\n");
        kcc_destroy(ctx);
        return 2;
      }
      std::printf("\nMax replicas : %" PRId64 "\n", q);
    }
  }

  std::vector<uint64_t> sc(specs.size());
  std::vector<int64_t> sm(specs.size()), totals(specs.size());
  std::vector<int32_t> serr(specs.size());
  for (size_t s = 0; s < specs.size(); ++s) {
    sc[s] = specs[s].cpu;
    sm[s] = specs[s].mem;
  }
  if (schedReq)
    rc = kcc_fit(ctx, n, in.alloc_cpu.data(), in.alloc_mem.data(), in.alloc_pods.data(),
                 in.pod_count.data(), suc.data(), sum_.data(), (int64_t)specs.size(), sc.data(),
                 sm.data(), totals.data(), serr.data());
  else
    rc = kcc_capacity(ctx, n, nc, in.node_ptr.data(), in.cpu_req.data(), in.mem_req.data(),
                      in.alloc_cpu.data(), in.alloc_mem.data(), in.alloc_pods.data(),
                      in.pod_count.data(), (int64_t)specs.size(), sc.data(), sm.data(),
                      totals.data(), serr.data());
  if (rc) return fail(ctx, rc);
  kcc_destroy(ctx);

  if (f.v["specs"].empty()) {  // CC:142-149, verbatim text
    if (serr[0]) {
      std::fprintf(stderr, "panic: runtime error: integer divide by zero\n");
      return 2;
    }
    std::printf("%s\n", kRule);
    std::printf("\n\t Total possible replicas for the pod with required input specs : %" PRId64,
                totals[0]);
    if (totals[0] >= specs[0].replicas)
      std::printf("\n\t So you can go ahead with deployment of %" PRId64
                  " pod replicas in the Kubernetes cluster!!\n\n", specs[0].replicas);
    else
      std::printf("\n\t Unfortunately Kubernetes cluster can't scehdule %" PRId64
                  " replicas. Please try again by reducing the number of replicas or/and cpu/memory "
                  "resource requests. Exiting!!\n\n", specs[0].replicas);
    std::printf("%s\n", kRule);
    return 0;
  }
  // batch: one line per spec
  for (size_t s = 0; s < specs.size(); ++s) {
    if (serr[s])
      std::printf("%s %s %s panic: integer divide by zero\n", specs[s].cpuStr.c_str(),
                  specs[s].memStr.c_str(), specs[s].repStr.c_str());
    else
      std::printf("%s %s %s total=%" PRId64 " %s\n", specs[s].cpuStr.c_str(), specs[s].memStr.c_str(),
                  specs[s].repStr.c_str(), totals[s], totals[s] >= specs[s].replicas ? "yes" : "no");
  }
  return 0;
}
