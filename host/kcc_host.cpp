// kcc_host.cpp — see kcc_host.hpp.  Reference: CC = src/KubeAPI/ClusterCapacity.go,
// BF = src/bytefmt/bytes.go of AshutoshNirkhe/KubernetesClusterCapacity.
#include "kcc_host.hpp"

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace kcchost {

namespace {

// Go strconv.Atoi (ParseInt(s, 10, 0) on 64-bit): [+-]digits, within int64.
bool goAtoi(const std::string& s, int64_t& out) {
  size_t i = 0;
  bool neg = false;
  if (s.empty()) return false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == s.size()) return false;
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    const uint64_t d = (uint64_t)(s[i] - '0');
    if (v > (lim - d) / 10) return false;  // ErrRange
    v = v * 10 + d;
  }
  out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

}  // namespace

uint64_t convertCPUToMilis(const std::string& cpu_in, bool* ok, bool print) {
  std::string cpu = cpu_in;
  bool flag = true;
  if (!cpu.empty() && cpu.back() == 'm') {  // strings.HasSuffix / TrimSuffix
    cpu.pop_back();
    flag = false;
  }
  int64_t cpuMili = 0;
  if (goAtoi(cpu, cpuMili)) {
    if (flag) cpuMili = (int64_t)((uint64_t)cpuMili * 1000u);  // Go int multiply wraps
    if (ok) *ok = true;
  } else {
    cpuMili = 0;
    if (print) std::printf("\nError converting string to int for %s\n", cpu.c_str());
    if (ok) *ok = false;
  }
  return (uint64_t)cpuMili;  // CC:318
}

std::pair<int64_t, bool> ToBytes(const std::string& in) {
  // strings.TrimSpace + strings.ToUpper
  size_t b = 0, e = in.size();
  while (b < e && std::isspace((unsigned char)in[b])) ++b;
  while (e > b && std::isspace((unsigned char)in[e - 1])) --e;
  std::string s = in.substr(b, e - b);
  for (char& ch : s) ch = (char)std::toupper((unsigned char)ch);
  size_t i = 0;  // strings.IndexFunc(s, unicode.IsLetter)
  while (i < s.size() && !(std::isalpha((unsigned char)s[i]) || (unsigned char)s[i] >= 0x80)) ++i;
  if (i == s.size()) return {0, false};
  const std::string num = s.substr(0, i), mult = s.substr(i);
  // strconv.ParseFloat on a letter-free string: [sign] digits [. digits]
  size_t k = (!num.empty() && (num[0] == '+' || num[0] == '-')) ? 1 : 0;
  size_t digits = 0;
  bool dot = false;
  for (; k < num.size(); ++k) {
    if (std::isdigit((unsigned char)num[k])) ++digits;
    else if (num[k] == '.' && !dot) dot = true;
    else return {0, false};
  }
  if (digits == 0) return {0, false};
  const double bytes = std::strtod(num.c_str(), nullptr);  // correctly rounded, like Go
  if (std::isinf(bytes) || !(bytes > 0)) return {0, false};
  double unit;
  if (mult == "T" || mult == "TB" || mult == "TIB") unit = 1099511627776.0;
  else if (mult == "G" || mult == "GB" || mult == "GIB") unit = 1073741824.0;
  else if (mult == "M" || mult == "MB" || mult == "MIB" || mult == "MI") unit = 1048576.0;
  else if (mult == "K" || mult == "KB" || mult == "KIB" || mult == "KI") unit = 1024.0;
  else if (mult == "B") unit = 1.0;
  else return {0, false};
  const double v = bytes * unit;
  // Go int64(float64) on amd64 (CVTTSD2SQ): out of range -> 0x8000000000000000
  if (std::isnan(v) || v >= 9223372036854775808.0 || v < -9223372036854775808.0)
    return {INT64_MIN, true};
  return {(int64_t)v, true};
}

bool loadCluster(const std::string& path, Cluster& out, std::string& err) {
  std::ifstream f(path);
  if (!f) {
    err = "cannot open cluster file " + path;
    return false;
  }
  std::string line;
  int ln = 0;
  while (std::getline(f, line)) {
    ++ln;
    const size_t hash = line.find('#');
    if (hash != std::string::npos) line.resize(hash);
    std::istringstream is(line);
    std::string kind;
    if (!(is >> kind)) continue;
    auto bad = [&](const char* what) {
      err = path + ":" + std::to_string(ln) + ": " + what;
      return false;
    };
    if (kind == "node") {
      NodeObj n;
      if (!(is >> n.name >> n.cpu >> n.memory >> n.pods)) return bad("node <name> <cpu> <memory> <pods> <c0..c3>");
      std::string c;
      while (is >> c) n.conditions.push_back(c);
      if (n.conditions.size() < 4) return bad("a node needs 4 condition statuses (CC:212-213)");
      out.nodes.push_back(n);
    } else if (kind == "pod") {
      Pod p;
      if (!(is >> p.nodeName >> p.ns >> p.name >> p.phase)) return bad("pod <node|-> <ns> <name> <phase>");
      if (p.nodeName == "-") p.nodeName.clear();
      std::string extra;
      if (is >> extra) p.getFails = extra == "missing";
      out.pods.push_back(p);
    } else if (kind == "container") {
      if (out.pods.empty()) return bad("container before any pod");
      Container c;
      if (!(is >> c.cpuRequest >> c.cpuLimit >> c.memRequest >> c.memLimit))
        return bad("container <cpuReq> <cpuLim> <memReqBytes> <memLimBytes>");
      out.pods.back().containers.push_back(c);
    } else if (kind == "initcontainer") {
      if (out.pods.empty()) return bad("initcontainer before any pod");
      Container c;
      c.init = true;
      if (!(is >> c.cpuRequest >> c.cpuLimit >> c.memRequest >> c.memLimit))
        return bad("initcontainer <cpuReq> <cpuLim> <memReqBytes> <memLimBytes> [always]");
      std::string pol;
      if (is >> pol) c.restartable = pol == "always";
      out.pods.back().containers.push_back(c);
    } else if (kind == "overhead") {
      if (out.pods.empty()) return bad("overhead before any pod");
      if (!(is >> out.pods.back().overheadCPU >> out.pods.back().overheadMem))
        return bad("overhead <cpuMillis> <memBytes>");
    } else {
      return bad("unknown record");
    }
  }
  return true;
}

namespace {
// One packed batch (Arrow layout, 4-byte padded) of strings for kcc_parse_*.
void pack(const std::vector<const std::string*>& strs, std::string& chars,
          std::vector<int64_t>& off) {
  chars.clear();
  off.assign(1, 0);
  for (const std::string* s : strs) {
    chars += *s;
    off.push_back((int64_t)chars.size());
  }
  chars.resize((chars.size() + 4) & ~(size_t)3, '\0');
}
}  // namespace

int getHealthyNodes(kcc_ctx* ctx, const Cluster& c, std::vector<node>& healthy, bool print) {
  const size_t noOfNodes = c.nodes.size();
  if (print) std::printf("\nThere are total %zu nodes in the cluster\n\n", noOfNodes);
  healthy.assign(noOfNodes, node{});  // zero rows stay for unhealthy nodes (CC:221-226)
  // both conversions of every node in one device batch each (CC:196-197, CC:202-206);
  // the prints below keep the reference's per-node order
  std::vector<uint64_t> cpu(noOfNodes);
  std::vector<int64_t> mem(noOfNodes);
  std::vector<int8_t> cst(noOfNodes), mst(noOfNodes);
  if (noOfNodes > 0) {
    std::vector<const std::string*> cs, ms;
    for (const NodeObj& n : c.nodes) {
      cs.push_back(&n.cpu);
      ms.push_back(&n.memory);
    }
    std::string chars;
    std::vector<int64_t> off;
    pack(cs, chars, off);
    int rc = kcc_parse_cpu_millis(ctx, (int64_t)noOfNodes, chars.data(), off.back(), off.data(),
                                  cpu.data(), cst.data());
    if (rc) return rc;
    pack(ms, chars, off);
    rc = kcc_parse_bytes(ctx, (int64_t)noOfNodes, chars.data(), off.back(), off.data(), mem.data(),
                         mst.data());
    if (rc) return rc;
  }
  for (size_t i = 0; i < noOfNodes; ++i) {
    const NodeObj& n = c.nodes[i];
    if (cst[i] != KCC_PARSE_OK && print) {  // CC:315-316, the string without its 'm'
      std::string s = n.cpu;
      if (!s.empty() && s.back() == 'm') s.pop_back();
      std::printf("\nError converting string to int for %s\n", s.c_str());
    }
    const int64_t memAlloc = mst[i] == KCC_PARSE_OK ? mem[i] : 0;  // CC:203-206
    if (mst[i] == KCC_PARSE_UNSUPPORTED)  // a float64-edge literal Quantity never prints
      std::fprintf(stderr, "node %s: memory %s is outside the device parser's exact domain; "
                   "using 0\n", n.name.c_str(), n.memory.c_str());
    bool flagHealthy = true;
    for (int j = 0; j < 4; ++j) {  // CC:212-219
      if (n.conditions[j] != "False") {
        if (print) std::printf("Skipping node %s as it is not healthy\n", n.name.c_str());
        flagHealthy = false;
        break;
      }
    }
    if (flagHealthy) {
      healthy[i].name = n.name;
      healthy[i].allocatableCPU = cpu[i];
      healthy[i].allocatableMemory = memAlloc;
      healthy[i].allocatablePods = n.pods;
    }
  }
  return KCC_OK;
}

std::map<std::string, std::vector<size_t>> nonTerminatedPodsByNode(const Cluster& c) {
  std::map<std::string, std::vector<size_t>> out;
  for (size_t i = 0; i < c.pods.size(); ++i) {  // pods in list order within each node
    const Pod& p = c.pods[i];
    if (p.phase == "Pending" || p.phase == "Succeeded" || p.phase == "Failed" ||
        p.phase == "Unknown")
      continue;
    out[p.nodeName].push_back(i);
  }
  return out;
}

std::vector<size_t> getNonTerminatedPodsForNode(const Cluster& c, const std::string& nodeName) {
  std::vector<size_t> out;
  for (size_t i = 0; i < c.pods.size(); ++i) {  // field selector of CC:236
    const Pod& p = c.pods[i];
    if (p.nodeName != nodeName) continue;
    if (p.phase == "Pending" || p.phase == "Succeeded" || p.phase == "Failed" ||
        p.phase == "Unknown")
      continue;
    out.push_back(i);
  }
  return out;
}

int buildInputs(kcc_ctx* ctx, const Cluster& c, const std::vector<node>& rows, EngineInputs& in) {
  in = EngineInputs{};
  std::string chars;          // limit, request, limit, request, ... (CC:279-283 order)
  std::vector<int64_t> off{0};
  // one cluster-wide pass (the List of CC:236 with the phase selector)
  // grouped by spec.nodeName, instead of one List per node row; a zero row (name "")
  // gets the pods whose nodeName is "", like the reference's per-row List
  const std::map<std::string, std::vector<size_t>> by_node = nonTerminatedPodsByNode(c);
  const std::vector<size_t> none;
  std::vector<const std::string*> init_cpu_str;  // after the app strings: same error order
  for (const node& r : rows) {  // CC:105: every row, zero rows included (name "")
    const auto it = by_node.find(r.name);
    const std::vector<size_t>& pods = it == by_node.end() ? none : it->second;
    for (size_t pi : pods) {
      const Pod& p = c.pods[pi];
      if (p.getFails) continue;  // NotFound: skipped by the sum (CC:267-268), still counted
      for (const Container& ct : p.containers) {  // CC:277-293 (app containers only)
        if (ct.init) continue;
        chars += ct.cpuLimit;
        off.push_back((int64_t)chars.size());
        chars += ct.cpuRequest;
        off.push_back((int64_t)chars.size());
        in.mem_req.push_back(ct.memRequest);
        in.mem_lim.push_back(ct.memLimit);
      }
      for (const Container& ct : p.containers) {  // opt-in model: init containers
        if (!ct.init) continue;
        init_cpu_str.push_back(&ct.cpuRequest);
        in.init_mem.push_back(ct.memRequest);
        in.init_rst.push_back(ct.restartable ? 1 : 0);
      }
      in.pod_ptr.push_back((int64_t)in.mem_req.size());
      in.init_ptr.push_back((int64_t)in.init_mem.size());
      in.ovh_cpu.push_back(p.overheadCPU);
      in.ovh_mem.push_back(p.overheadMem);
    }
    in.node_ptr.push_back((int64_t)in.mem_req.size());
    in.node_pod_ptr.push_back((int64_t)in.ovh_cpu.size());
    in.alloc_cpu.push_back(r.allocatableCPU);
    in.alloc_mem.push_back(r.allocatableMemory);
    in.alloc_pods.push_back(r.allocatablePods);
    in.pod_count.push_back((int64_t)pods.size());  // len(pods), CC:106/135
  }
  const int64_t ns = (int64_t)off.size() - 1;
  std::vector<uint64_t> millis((size_t)ns);
  std::vector<int8_t> st((size_t)ns);
  chars.resize((chars.size() + 4) & ~(size_t)3, '\0');  // 4-byte padded buffer
  if (ns > 0) {
    const int rc = kcc_parse_cpu_millis(ctx, ns, chars.data(), off[ns], off.data(), millis.data(),
                                        st.data());
    if (rc) return rc;
  }
  in.cpu_lim.resize((size_t)ns / 2);
  in.cpu_req.resize((size_t)ns / 2);
  for (int64_t k = 0; k < ns; ++k) {
    if (st[k] != KCC_PARSE_OK) {  // CC:315-316 prints the string without its 'm'
      std::string s = chars.substr((size_t)off[k], (size_t)(off[k + 1] - off[k]));
      if (!s.empty() && s.back() == 'm') s.pop_back();
      std::printf("\nError converting string to int for %s\n", s.c_str());
    }
    (k & 1 ? in.cpu_req : in.cpu_lim)[(size_t)k / 2] = millis[k];
  }
  if (!init_cpu_str.empty()) {  // opt-in model only; the reference never reads them
    std::string ichars;
    std::vector<int64_t> ioff;
    pack(init_cpu_str, ichars, ioff);
    const int64_t ni = (int64_t)init_cpu_str.size();
    in.init_cpu.resize((size_t)ni);
    std::vector<int8_t> ist((size_t)ni);
    const int rc = kcc_parse_cpu_millis(ctx, ni, ichars.data(), ioff[ni], ioff.data(),
                                        in.init_cpu.data(), ist.data());
    if (rc) return rc;
    for (int64_t k = 0; k < ni; ++k)
      if (ist[k] != KCC_PARSE_OK) {  // as convertCPUToMilis reports it (CC:315-316)
        std::string s = *init_cpu_str[(size_t)k];
        if (!s.empty() && s.back() == 'm') s.pop_back();
        std::printf("\nError converting string to int for %s\n", s.c_str());
        in.init_cpu[(size_t)k] = 0;
      }
  }
  return KCC_OK;
}

}  // namespace kcchost

// C entry points for tests (ctypes) — the parsers only; no device work.
extern "C" {
uint64_t kcchost_convert_cpu_to_milis(const char* s, int* ok) {
  bool b = false;
  const uint64_t v = kcchost::convertCPUToMilis(s, &b, false);
  if (ok) *ok = b ? 1 : 0;
  return v;
}
int kcchost_to_bytes(const char* s, int64_t* out) {
  const auto r = kcchost::ToBytes(s);
  *out = r.first;
  return r.second ? 0 : -1;
}
}
