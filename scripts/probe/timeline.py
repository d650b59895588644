"""Diagnostic: per-workgroup phase timeline of the small fit-side kernels (a
-DKCC_TIMELINE build, variants/libkcc_tl.so), C4 inputs.  Stamps are s_memrealtime
(100 MHz); printed in microseconds relative to the first spec_prep workgroup."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from kubernetesclustercapacity_amd import _lib, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "tl"
L = _lib.load(os.path.join(ROOT, "variants", f"libkcc_{name}.so"))
L.kcc_debug_timeline.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
cl = synth.config_cluster("C4")
sc, sm = synth.config_specs("C4")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
ac, am, ap, pc = T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)
s_cpu, s_mem = T(sc), T(sm)
n, S, nc = cl.n_nodes, sc.size, cl.n_containers
uc = torch.empty(n, dtype=torch.int64, device=dev)
um = torch.empty(n, dtype=torch.int64, device=dev)
part = torch.empty(2 * S, dtype=torch.int64, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
h = C.c_void_p()
assert L.kcc_create(C.byref(h), 0, 1) == 0
assert L.kcc_reserve(h, n, nc, S) == 0
buf = np.zeros((4096, 4), np.uint64)


def step():
    assert L.kcc_reduce_requests_async(h, n, nc, P(ptr), P(cpu), P(mem), None, None, P(uc), P(um),
                                       None, None, None) == 0
    assert L.kcc_fit_prepare_async(h, n, P(ac), P(am), P(ap), P(pc), P(uc), P(um), S, P(s_cpu),
                                   P(s_mem), P(part), None) == 0
    assert L.kcc_fit_run_async(h, n, S, P(part), None) == 0


for _ in range(3):
    step()
torch.cuda.synchronize()
assert L.kcc_debug_timeline(buf.ctypes.data) == 0
step()
assert L.kcc_debug_timeline(buf.ctypes.data) == 0
t = buf.astype(np.float64)
t0 = t[0:300, 0][t[0:300, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731


def show(label, rows, k0, k1):
    r = rows[(rows[:, k0] > 0) & (rows[:, k1] > 0)]
    if not len(r):
        print(f"{label:34s} (none)")
        return
    d = (r[:, k1] - r[:, k0]) / 100.0
    print(f"{label:34s} n={len(r):4d} start {us(r[:, k0].min()):8.2f}..{us(r[:, k0].max()):8.2f}"
          f"  end {us(r[:, k1].min()):8.2f}..{us(r[:, k1].max()):8.2f}"
          f"  dur min/med/max {d.min():6.2f}/{np.median(d):6.2f}/{d.max():6.2f} us")


sp = t[0:257]
sp = t[0:300]
show("spec_rank wgs", sp, 0, 1)
show("node_prep entry -> after prologue", t[3072:4096], 2, 0)
show("node_prep (after prologue -> end)", t[3072:4096], 0, 1)
show("clamp_agg accumulate", t[2048:3072], 0, 1)
show("clamp_agg suffixes+write", t[2048:3072], 1, 2)

np_rows = t[3072:3072 + 512]
np.save(os.path.join(ROOT, "gpurun_out", "tl_node_prep.npy"), np.stack([us(np_rows[:, 2]), us(np_rows[:, 0]), us(np_rows[:, 1])], 1))
