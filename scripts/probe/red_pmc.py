"""Diagnostic: run the segmented reduce of each named variants/ build REPS times in a row
(C4 inputs, shared outputs), for rocprofv3 --pmc passes; dispatches are in name order."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from kubernetesclustercapacity_amd import _lib, synth  # noqa: E402

REPS = 10
dev = torch.device("cuda", 0)
cl = synth.config_cluster("C4")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
n, nc = cl.n_nodes, cl.n_containers
uc = torch.empty(n, dtype=torch.int64, device=dev)
um = torch.empty(n, dtype=torch.int64, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
for nm in sys.argv[1:]:
    L = _lib.load(os.path.join(ROOT, "variants", f"libkcc_{nm}.so"))
    h = C.c_void_p()
    assert L.kcc_create(C.byref(h), 0, 1) == 0
    assert L.kcc_reserve(h, n, nc, 16) == 0
    for _ in range(REPS):
        assert L.kcc_reduce_requests_async(h, n, nc, P(ptr), P(cpu), P(mem), None, None,
                                           P(uc), P(um), None, None, None) == 0
    torch.cuda.synchronize()
    print(nm, "done", flush=True)
