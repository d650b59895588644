"""Parity of variants/ builds (scripts/ab_variants.py build ...) on one seeded case of
tests/test_gpu_parity.py against the C oracle — for bisecting a kernel change on the GPU.

  python scripts/variant_parity.py NAME ... [--n 20000 --pods 400000 --s 300 --seed 1]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--pods", type=int, default=400000)
    ap.add_argument("--s", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from kubernetesclustercapacity_amd import _lib, synth
    from oracle import coracle
    c = synth.make_cluster(a.n, a.pods, seed=a.seed)
    sc, sm = synth.make_specs(a.s, seed=a.seed)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    P = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    for nm in a.names:
        L = _lib.load(os.path.join(ROOT, "variants", f"libkcc_{nm}.so"))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0
        t = np.zeros(a.s, np.int64)
        e = np.zeros(a.s, np.int32)
        rc = L.kcc_fit(h, a.n, P(c.alloc_cpu), P(c.alloc_mem), P(c.alloc_pods), P(c.pod_count),
                       P(uc), P(um), a.s, P(sc), P(sm), P(t), P(e))
        bad = np.nonzero(t != ot)[0]
        print(f"{nm}: rc={rc} mismatches={bad.size}"
              + (f" first={bad[:5].tolist()} got={t[bad[:3]].tolist()} want={ot[bad[:3]].tolist()}"
                 if bad.size else ""), flush=True)
        L.kcc_destroy(h)


if __name__ == "__main__":
    main()
