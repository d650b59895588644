"""Run the golden fit fixtures and a seeded adversarial cluster against one libkcc build
(GPU): python scripts/probe/dbg_variant.py variants/libkcc_X.so ..."""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.init()
from kubernetesclustercapacity_amd import _lib, synth  # noqa: E402
from oracle import coracle  # noqa: E402

for path in sys.argv[1:]:
    _lib._LIB = _lib.load(path)
    from kubernetesclustercapacity_amd import CapacityEngine
    bad = []
    with CapacityEngine(0, 1) as eng:
        for g in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz"))):
            if g.endswith("parse.npz"):
                continue
            d = np.load(g)
            t, e = eng.total_possible_max_replicas(d["alloc_cpu"], d["alloc_mem"], d["alloc_pods"],
                                                   d["pod_count"], d["exp_used_cpu"],
                                                   d["exp_used_mem"], d["spec_cpu"], d["spec_mem"])
            nbad = int((t != d["exp_totals"]).sum())
            bad.append((os.path.basename(g), d["spec_cpu"].size, nbad))
        c = synth.make_cluster(20_000, 400_000, seed=3, chunk=4096, adversarial=True)
        for S in (1, 63, 64, 65, 300, 1500, 5000):
            sc, sm = synth.make_specs(S, seed=S, adversarial=True)
            t, e = eng.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                                c.alloc_pods, c.pod_count, sc, sm)
            uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
            ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, 8)
            bad.append((f"synth S={S}", S, int((t != ot).sum())))
    print(os.path.basename(path), bad, flush=True)
