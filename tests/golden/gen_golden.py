"""Generate the committed golden fixtures tests/golden/*.npz.

Inputs are seeded synthetic clusters (kubernetesclustercapacity_amd.synth) plus
hand-built edge rows; expected outputs come from the pure-Python big-int
restatement oracle/pyoracle.py (independent of the C oracle and of the kernels).
The reference itself cannot run here (Go absent, no reference fixtures exist:
SURVEY.md §4/§8c), so these vectors are pinned through the KATs in
tests/test_oracle_kat.py, which both oracles pass.

Run:  python tests/golden/gen_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from kubernetesclustercapacity_amd import synth  # noqa: E402
from oracle import pyoracle  # noqa: E402

U64 = 1 << 64


def edge_case():
    """Hand-built rows covering every branch of CC:119-136."""
    rows = [  # alloc_cpu, alloc_mem, alloc_pods, podCount, containers [(cpu, mem)]
        (4000, 16_723_480_576, 110, 12, [(1850, 3_221_225_472)]),      # K2
        (64000, 274_877_906_944, 110, 30, []),                          # K3 clamp
        (64000, 274_877_906_944, 110, 130, []),                         # K4 negative clamp
        (4000, 1 << 30, 110, 5, [(4000, 1 << 30)]),                     # K5 full
        (0, 0, 0, 3, []),                                               # K6 zero row
        (4000, 1 << 34, 110, 1, [(U64 - 100, 0)]),                      # K8 wrapped request
        (U64 - 1, (1 << 63) - 1, 1 << 40, 0, []),                       # huge quotients
        (8000, 1 << 36, 0, 0, []),                                      # allocPods 0
        (8000, 1 << 36, -4, 2, []),                                     # allocPods < 0
        (8000, (1 << 63) - 1, 250, 7, [(10, -1)]),                      # mem overflow -> MinInt64
        (1 << 40, 1 << 50, 65536, 0, []),                               # P at fast bound
        (1 << 40, 1 << 50, 65537, 0, []),                               # P above fast bound
        (2**31 - 1, 2**53 - 1, 110, 0, []),                             # fast-path edges
        (2**31, 2**53, 110, 0, []),                                     # just past them
        (5, 5, 110, 200, [(1, 1), (1, 1), (1, 1)]),                     # tiny free
        (100, 100, 3, 1 << 30, []),                                     # |clamp| > 2^20
        (2**21 - 1, 2**50 - 1, 110, 0, []),                             # fit fast-path edges
        (2**21, 2**50, 110, 0, []),                                     # just past them
        (2**21 - 1, 2**50 - 1, 1 << 20, 0, []),                         # P at its bound
        (2**21 - 1, 2**50 - 1, (1 << 20) + 1, 0, []),                   # P past it
        (4_194_302, 2**51 - 2, 2, 1, []),                               # 2 x (spec edge)
        (2**50 - 1, 2**50 - 1, 300, 0, []),                             # f64 quotient bounds
        (2**50, 2**50 - 1, 300, 0, []),                                 # free CPU past it
        (2**51 - 2, 2**49 + 3, 7, 2, []),
    ]
    alloc_cpu = np.array([r[0] for r in rows], np.uint64)
    alloc_mem = np.array([r[1] for r in rows], np.int64)
    alloc_pods = np.array([r[2] for r in rows], np.int64)
    pod_count = np.array([r[3] for r in rows], np.int64)
    cpu, mem, ptr = [], [], [0]
    for r in rows:
        for c, m in r[4]:
            cpu.append(c)
            mem.append(m)
        ptr.append(len(cpu))
    cpu = np.array(cpu, np.uint64)
    mem = np.array(mem, np.int64)
    spec_cpu = np.array([200, 100, 1, 3, 7, 8000, 0, 1 << 23, 2**63, 50, 1, 2**23 - 1,
                         2**22 - 1, 2**22, 2**21 - 1, 1, 2**51 - 1, 2**51, 2**49 + 1],
                        np.uint64)
    spec_mem = np.array([262_144_000, 104_857_600, 1, 1 << 20, -1, 1 << 35, 1 << 20, 0,
                         -(1 << 63), 2**37, 2**37 - 1, 3, 2**51 - 1, 7, 2**50 - 1, 2**51,
                         5, 2**40 + 1, 2**49 + 1],
                        np.int64)
    return dict(alloc_cpu=alloc_cpu, alloc_mem=alloc_mem, alloc_pods=alloc_pods,
                pod_count=pod_count, node_ptr=np.array(ptr, np.int64), cpu_req=cpu,
                mem_req=mem, cpu_lim=cpu * np.uint64(3), mem_lim=mem * 3,
                spec_cpu=spec_cpu, spec_mem=spec_mem)


def cluster_case(n, pods, n_specs, seed, skew=False, adversarial=False, unhealthy=0.01):
    c = synth.make_cluster(n, pods, seed=seed, skew=skew, adversarial=adversarial,
                           unhealthy=unhealthy, chunk=128)
    sc, sm = synth.make_specs(n_specs, seed=seed, adversarial=adversarial)
    return dict(alloc_cpu=c.alloc_cpu, alloc_mem=c.alloc_mem, alloc_pods=c.alloc_pods,
                pod_count=c.pod_count, node_ptr=c.node_ptr, cpu_req=c.cpu_req,
                mem_req=c.mem_req, cpu_lim=c.cpu_lim, mem_lim=c.mem_lim,
                spec_cpu=sc, spec_mem=sm)


def expected(d):
    sums = pyoracle.reduce_requests(d["node_ptr"].tolist(), d["cpu_req"].tolist(),
                                    d["mem_req"].tolist(), d["cpu_lim"].tolist(),
                                    d["mem_lim"].tolist())
    used_cpu = np.array([s[0] for s in sums], np.uint64)
    used_mem = np.array([s[1] for s in sums], np.int64)
    lim_cpu = np.array([s[2] for s in sums], np.uint64)
    lim_mem = np.array([s[3] for s in sums], np.int64)
    tot, err = pyoracle.fit(d["alloc_cpu"], d["alloc_mem"], d["alloc_pods"], d["pod_count"],
                            used_cpu, used_mem, d["spec_cpu"], d["spec_mem"])
    return dict(exp_used_cpu=used_cpu, exp_used_mem=used_mem, exp_lim_cpu=lim_cpu,
                exp_lim_mem=lim_mem, exp_totals=np.array(tot, np.int64),
                exp_err=np.array(err, np.int32))


CASES = {
    "edge": edge_case,
    "small": lambda: cluster_case(300, 6_000, 64, 11),
    "adversarial": lambda: cluster_case(300, 6_000, 64, 12, adversarial=True),
    "skew": lambda: cluster_case(200, 4_000, 32, 13, skew="zipf"),  # SURVEY §8d Zipf(1.2)
    "sparse": lambda: cluster_case(2_000, 300, 16, 14, unhealthy=0.2),   # mostly empty nodes
}


def parse_case():
    """tests/golden/parse.npz: the hand KAT strings and seeded corpora of
    tests/test_parse.py, packed; expected values/statuses from oracle/pyoracle.py."""
    from kubernetesclustercapacity_amd import quantity
    from tests import test_parse as tp
    d = {}
    for key, strs, fn in (("cpu", tp.CPU_KATS + tp.fuzz_corpus(600, 31), pyoracle.convert_cpu_to_milis),
                          ("mem", tp.BYTES_KATS + tp.fuzz_corpus(600, 32) + tp.decimal_corpus(1200, 33),
                           pyoracle.to_bytes)):
        buf, off = quantity.pack_strings(strs)
        res = [fn(x.decode("latin-1")) for x in strs]
        d[f"{key}_buf"], d[f"{key}_off"] = buf, off
        d[f"{key}_val"] = np.array([r[0] for r in res], np.uint64 if key == "cpu" else np.int64)
        d[f"{key}_st"] = np.array([1 if r[1] else 0 for r in res], np.int8)
    return d


def main():
    """No argument: every fixture; otherwise only the named ones (parse, edge, small, ...)."""
    want = set(sys.argv[1:]) or {"parse", *CASES}
    if "parse" in want:
        path = os.path.join(HERE, "parse.npz")
        np.savez_compressed(path, **parse_case())
        print(f"{path}")
    for name, fn in CASES.items():
        if name not in want:
            continue
        d = fn()
        d.update(expected(d))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"{path}: nodes={d['alloc_cpu'].size} containers={d['cpu_req'].size} "
              f"specs={d['spec_cpu'].size}")


if __name__ == "__main__":
    main()
