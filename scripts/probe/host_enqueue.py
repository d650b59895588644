"""Host-side cost of one step's enqueue (kcc_capacity_async through ctypes) against the
GPU's time per step, on rank 0's shard of C4 split `shard` ways: if the enqueue takes as
long as the step, the step is host-bound and device-side gains cannot show.
  python scripts/probe/host_enqueue.py [shard]"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from kubernetesclustercapacity_amd import _lib, synth  # noqa: E402

shard = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
n_all = synth.CONFIGS["C4"]["n_nodes"]
cl = synth.config_cluster("C4", node_lo=0, node_hi=n_all // shard, limits=False)
sc, sm = synth.config_specs("C4")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
args = [T(x) for x in (cl.node_ptr, cl.cpu_req, cl.mem_req, cl.alloc_cpu, cl.alloc_mem,
                       cl.alloc_pods, cl.pod_count)]
n, S, nc = cl.n_nodes, sc.size, cl.n_containers
uc = torch.empty(n, dtype=torch.int64, device=dev)
um = torch.empty(n, dtype=torch.int64, device=dev)
s_cpu, s_mem = T(sc), T(sm)
tot = torch.empty(S, dtype=torch.int64, device=dev)
err = torch.empty(S, dtype=torch.int32, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
stream = torch.cuda.Stream(dev)
sh = C.c_void_p(stream.cuda_stream)
L = _lib.load(os.path.join(ROOT, "kubernetesclustercapacity_amd", "libkcc.so"))
h = C.c_void_p()
assert L.kcc_create(C.byref(h), 0, 1) == 0
assert L.kcc_reserve(h, n, nc, S) == 0
pa = [P(a) for a in args]


def step():
    assert L.kcc_capacity_async(h, n, nc, None, *pa, P(uc), P(um), S, P(s_cpu), P(s_mem),
                                P(tot), P(err), sh) == 0


for _ in range(20):
    step()
torch.cuda.synchronize()
for reps in (200,):
    enq = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    t0 = time.perf_counter()
    for _ in range(reps):
        a = time.perf_counter()
        step()
        enq.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    e1.record(stream)
    e1.synchronize()
    t2 = time.perf_counter()
    print(f"shard {shard}: enqueue per step median {np.median(enq) * 1e6:.1f} us "
          f"(p90 {np.percentile(enq, 90) * 1e6:.1f}); host loop {(t1 - t0) / reps * 1e6:.1f} us/step; "
          f"GPU events {e0.elapsed_time(e1) / reps * 1e3:.1f} us/step; wall to drain {(t2 - t0) / reps * 1e6:.1f} us/step")
    # the GPU alone: a graph-free burst enqueued ahead (host far ahead of the device)
L.kcc_destroy(h)
