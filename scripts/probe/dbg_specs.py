"""Debug: one capacity call per spec count, mismatching specs vs the C oracle."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kubernetesclustercapacity_amd import synth, CapacityEngine  # noqa: E402
from oracle import coracle  # noqa: E402

eng = CapacityEngine(0, 1)
c = synth.make_cluster(2_500, 50_000, seed=11, chunk=1024)
uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
for s in [int(a) for a in sys.argv[1:]]:
    sc, sm = synth.make_specs(s, seed=11)
    sc[::3] = sc[0]
    sm[::5] = sm[1]
    sc[1::7] = sc[2]
    for rep in range(2):
        t, e = eng.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                            c.alloc_pods, c.pod_count, sc, sm)
        ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, 8)
        bad = np.nonzero(t != ot)[0]
        print(s, rep, "bad", len(bad), bad[:12], "err", int((e != oe).sum()))
        for i in bad[:6]:
            print("   i", i, "c", sc[i], "m", sm[i], "got", t[i], "want", ot[i], "diff", int(t[i]) - int(ot[i]))
