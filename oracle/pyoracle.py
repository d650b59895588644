"""Independent pure-Python (big-int) restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and the C-oracle cross-check), never by
the product package.  It is written separately from oracle/kcc_oracle.c (explicit
two's-complement masking instead of C unsigned wrap) so that the two restatements
check each other (SURVEY.md §4 item 2, §8c "Cross-check").

Reference: AshutoshNirkhe/KubernetesClusterCapacity
  CC = src/KubeAPI/ClusterCapacity.go, BF = src/bytefmt/bytes.go
Parity pinning: no reference tests/goldens exist; pinned by the
hand-derived KATs in tests/test_oracle_kat.py.  Pure-Python loops: small cases only.
"""
from __future__ import annotations

import math
import re

M64 = (1 << 64) - 1
I64_MIN = -(1 << 63)


def u64(x: int) -> int:
    return x & M64


def i64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def go_div_i64(x: int, y: int) -> int:
    """Go int64 '/', truncating toward zero, wrapping MinInt64 / -1."""
    if y == 0:
        raise ZeroDivisionError("integer divide by zero")
    q = abs(x) // abs(y)
    if (x < 0) != (y < 0):
        q = -q
    return i64(q)


def find_min(x: int, y: int) -> int:  # CC:159-164
    return x if x <= y else y


def reduce_requests(node_ptr, cpu_req, mem_req, cpu_lim=None, mem_lim=None):
    """CC:255-299 (adds CC:290-293) for every node of a CSR container list."""
    n = len(node_ptr) - 1
    out = []
    for i in range(n):
        cr = cl = mr = ml = 0
        for c in range(node_ptr[i], node_ptr[i + 1]):
            cr = u64(cr + int(cpu_req[c]))
            mr = i64(mr + int(mem_req[c]))
            if cpu_lim is not None:
                cl = u64(cl + int(cpu_lim[c]))
            if mem_lim is not None:
                ml = i64(ml + int(mem_lim[c]))
        out.append((cr, mr, cl, ml))
    return out


def fit_one(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
            spec_cpu, spec_mem) -> int:
    """CC:119-136 for one node row and one spec.  Raises ZeroDivisionError where Go
    panics."""
    alloc_cpu, used_cpu, spec_cpu = u64(alloc_cpu), u64(used_cpu), u64(spec_cpu)
    alloc_mem, used_mem, spec_mem = i64(alloc_mem), i64(used_mem), i64(spec_mem)
    if alloc_cpu <= used_cpu:
        qc = 0
    else:
        if spec_cpu == 0:
            raise ZeroDivisionError("integer divide by zero")
        qc = i64((alloc_cpu - used_cpu) // spec_cpu)  # int(uint64) reinterprets
    if alloc_mem <= used_mem:
        qm = 0
    else:
        qm = go_div_i64(i64(alloc_mem - used_mem), spec_mem)
    q = find_min(qc, qm)
    if q >= i64(alloc_pods):
        q = i64(alloc_pods - pod_count)
    return q


def fit(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
        spec_cpu, spec_mem):
    """CC:101-140 for every spec: returns (totals, errs)."""
    totals, errs = [], []
    for s in range(len(spec_cpu)):
        tot = 0
        err = 0
        try:
            for i in range(len(alloc_cpu)):
                tot = i64(tot + fit_one(int(alloc_cpu[i]), int(alloc_mem[i]),
                                        int(alloc_pods[i]), int(pod_count[i]),
                                        int(used_cpu[i]), int(used_mem[i]),
                                        int(spec_cpu[s]), int(spec_mem[s])))
        except ZeroDivisionError:
            tot, err = 0, 1
        totals.append(tot)
        errs.append(err)
    return totals, errs


# ---- host-side parsers (out of the hot path; define the engine's int64 inputs) ----

_ATOI = re.compile(r"[+-]?[0-9]+\Z")


def go_atoi(s: str):
    if not _ATOI.match(s):
        return None
    v = int(s)
    if v < I64_MIN or v > (1 << 63) - 1:
        return None
    return v


def convert_cpu_to_milis(cpu: str):
    """CC:301-319.  Returns (value, ok)."""
    flag = True
    if cpu.endswith("m"):
        cpu = cpu[:-1]
        flag = False
    v = go_atoi(cpu)
    if v is None:
        return 0, False
    if flag:
        v = i64(v * 1000)
    return u64(v), True


_FLOAT = re.compile(r"[+-]?([0-9]+\.?[0-9]*|\.[0-9]+)\Z")
_UNITS = {
    "T": 1 << 40, "TB": 1 << 40, "TIB": 1 << 40,
    "G": 1 << 30, "GB": 1 << 30, "GIB": 1 << 30,
    "M": 1 << 20, "MB": 1 << 20, "MIB": 1 << 20, "MI": 1 << 20,
    "K": 1 << 10, "KB": 1 << 10, "KIB": 1 << 10, "KI": 1 << 10,
    "B": 1,
}


def to_bytes(s: str):
    """BF:75-105.  Returns (value, ok)."""
    s = s.strip().upper()
    i = next((k for k, ch in enumerate(s) if ch.isalpha()), -1)
    if i == -1:
        return 0, False
    num, mult = s[:i], s[i:]
    if not _FLOAT.match(num):
        return 0, False
    b = float(num)  # Python float() is correctly rounded, like Go ParseFloat
    if math.isinf(b) or b <= 0:
        return 0, False
    if mult not in _UNITS:
        return 0, False
    v = b * float(_UNITS[mult])
    if math.isnan(v) or v >= 2.0 ** 63 or v < -(2.0 ** 63):
        return I64_MIN, True  # amd64 CVTTSD2SQ overflow value
    return int(v), True


def pod_requests(pod_ptr, cpu_req, mem_req, init_ptr=None, init_cpu=None, init_mem=None,
                 restartable=None, ovh_cpu=None, ovh_mem=None):
    """SURVEY §8f row 4 — OPT-IN scheduler request model, NOT the reference's semantics
    (the reference sums app containers only, CC:276-294).  The kube-scheduler's pod
    request (pkg/api/v1/resource PodRequests, sidecar-aware form; absent here, parity
    unpinned beyond hand-derived cases), restated with k8s' "absent resource" rule for
    max: an empty init list leaves the app sum unchanged.  Returns [(cpu, mem)]."""
    out = []
    for p in range(len(pod_ptr) - 1):
        app = [0, 0]
        for c in range(pod_ptr[p], pod_ptr[p + 1]):
            app = [app[0] + int(cpu_req[c]), app[1] + int(mem_req[c])]
        side = [0, 0]
        init = [None, None]
        if init_ptr is not None:
            for k in range(init_ptr[p], init_ptr[p + 1]):
                r = [int(init_cpu[k]), int(init_mem[k])]
                if restartable is not None and restartable[k]:
                    app = [app[0] + r[0], app[1] + r[1]]
                    side = [side[0] + r[0], side[1] + r[1]]
                    cand = side
                else:
                    cand = [r[0] + side[0], r[1] + side[1]]
                # compare in the wrapped domain (cpu unsigned, memory signed)
                cand = [u64(cand[0]), i64(cand[1])]
                init = [cand[j] if init[j] is None or cand[j] > init[j] else init[j]
                        for j in range(2)]
        app = [u64(app[0]), i64(app[1])]
        req = [app[j] if init[j] is None or app[j] >= init[j] else init[j] for j in range(2)]
        if ovh_cpu is not None:
            req[0] += int(ovh_cpu[p])
        if ovh_mem is not None:
            req[1] += int(ovh_mem[p])
        out.append((u64(req[0]), i64(req[1])))
    return out
