// kcc_host.hpp — C++ host mirror of the reference's host side around the hot path.
//
// The reference host is Go (src/KubeAPI/ClusterCapacity.go = CC, src/bytefmt/bytes.go =
// BF); Go is absent from this image, so the part a user drives — flag parsing, the
// quantity helpers, node/pod selection and the verdict — is restated here in C++ with
// the same names, argument meaning and error behaviour, on top of the C-ABI of
// include/kcc.h.  client-go is replaced by a cluster description file (there is no
// apiserver here); the selection rules of getHealthyNodes / getNonTerminatedPodsForNode
// are kept.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "kcc.h"

namespace kcchost {

// CC:301-319.  Prints "\nError converting string to int for <s>\n" and returns 0 on an
// Atoi failure, like the reference; `ok` (optional) reports it.
uint64_t convertCPUToMilis(const std::string& cpu, bool* ok = nullptr, bool print = true);

// BF:75-105.  Returns (bytes, true) or (0, false) — the Go (int64, error) pair.
std::pair<int64_t, bool> ToBytes(const std::string& s);

// CC:159-164
inline int64_t findMin(int64_t x, int64_t y) { return x <= y ? x : y; }

// CC:41-46
struct node {
  std::string name;
  uint64_t allocatableCPU = 0;
  int64_t allocatableMemory = 0;
  int64_t allocatablePods = 0;
};

struct Container {
  std::string cpuRequest = "0", cpuLimit = "0";  // Quantity.String() (canonical)
  int64_t memRequest = 0, memLimit = 0;          // Quantity.Value()
  bool init = false, restartable = false;        // an init container (restartPolicy Always)
};

struct Pod {
  std::string nodeName, ns, name, phase;
  std::vector<Container> containers;
  bool getFails = false;  // the per-pod Get of CC:264 returns NotFound (CC:267-271)
  uint64_t overheadCPU = 0;  // spec.overhead (millicores, bytes): opt-in model only
  int64_t overheadMem = 0;
};

struct NodeObj {
  std::string name, cpu, memory;  // Status.Allocatable cpu / memory (Quantity.String())
  int64_t pods = 0;               // Status.Allocatable.Pods().Value()
  std::vector<std::string> conditions;  // Status.Conditions[j].Status
};

struct Cluster {
  std::vector<NodeObj> nodes;
  std::vector<Pod> pods;
};

// Cluster description file (one object per line, '#' comments):
//   node <name> <cpu> <memory> <pods> <cond0> <cond1> <cond2> <cond3>
//   pod <nodeName|-> <namespace> <name> <phase> [missing]
//   container <cpuRequest> <cpuLimit> <memRequestBytes> <memLimitBytes>   (of the last pod)
//   initcontainer <cpuRequest> <cpuLimit> <memRequestBytes> <memLimitBytes> [always]
//   overhead <cpuMillis> <memBytes>                                         (of the last pod)
// (init containers and overhead are read only by -schedulerRequests; the
// reference's sums ignore them, CC:277.)
// "-" as nodeName means "" (an unscheduled pod).  Returns false with a message on error.
bool loadCluster(const std::string& path, Cluster& out, std::string& err);

// CC:166-230 — rows in node order; an unhealthy node keeps a zero row (CC:221-226).
// (The reference's make([]node, n, 3) panics for n > 3, CC:176: not reproduced.)
// The nodes' cpu and memory strings are converted on the device (kcc_parse_cpu_millis,
// kcc_parse_bytes on `ctx`, one batch each).  Returns a KCC_E* code (0 on success).
int getHealthyNodes(kcc_ctx* ctx, const Cluster& c, std::vector<node>& healthy,
                    bool print = true);

// CC:232-253 — indices of the pods on `nodeName` whose phase is not Pending,
// Succeeded, Failed or Unknown.
std::vector<size_t> getNonTerminatedPodsForNode(const Cluster& c, const std::string& nodeName);

// The same selection for every node at once (one cluster-wide pass, grouped by
// spec.nodeName): nodeName -> pod indices in list order.
std::map<std::string, std::vector<size_t>> nonTerminatedPodsByNode(const Cluster& c);

// Per-row inputs of the engine: CSR containers (requests), podCount = len(pods).
struct EngineInputs {
  std::vector<int64_t> node_ptr{0};
  std::vector<uint64_t> cpu_req, cpu_lim;
  std::vector<int64_t> mem_req, mem_lim;
  std::vector<uint64_t> alloc_cpu;
  std::vector<int64_t> alloc_mem, alloc_pods, pod_count;
  // opt-in scheduler request model: the summed pods in CSR form
  std::vector<int64_t> node_pod_ptr{0}, pod_ptr{0}, init_ptr{0};
  std::vector<uint64_t> init_cpu, ovh_cpu;
  std::vector<int64_t> init_mem, ovh_mem;
  std::vector<uint8_t> init_rst;
};
// The container cpu strings (limits and requests, CC:279-283) are converted on the device
// in one kcc_parse_cpu_millis batch on `ctx`; each failed string prints
// the reference's "Error converting string to int" line, in the reference's order
// (per container: limit, then request).  Returns a KCC_E* code (0 on success).
int buildInputs(kcc_ctx* ctx, const Cluster& c, const std::vector<node>& rows, EngineInputs& in);

}  // namespace kcchost
