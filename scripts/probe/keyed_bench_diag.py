"""Probe: bench-like sequence (warmup + timed steps of the pipelined call, then the keyed
reduce repeated) with both outputs checked against the C oracle after each phase."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
torch.cuda.init()
from kubernetesclustercapacity_amd import CapacityEngine, synth  # noqa: E402
from oracle import coracle  # noqa: E402

dev = torch.device("cuda", 0)
cl = synth.make_cluster(1_000_000, 20_000_000, seed=20261019, node_lo=0, node_hi=1_000_000)
sc, sm = synth.config_specs("C4")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
n, S = cl.n_nodes, sc.size
a = [T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)]
uc = torch.empty(n, dtype=torch.int64, device=dev)
um = torch.empty(n, dtype=torch.int64, device=dev)
partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
oc, om, _, _ = coracle.reduce_requests(cl.node_ptr, cl.cpu_req, cl.mem_req)


def check(name, c, m):
    gc, gm = c.cpu().numpy().view(np.uint64), m.cpu().numpy()
    bc, bm = np.flatnonzero(gc != oc), np.flatnonzero(gm != om)
    print(f"{name}: cpu rows off {bc.size} {bc[:5]}, mem rows off {bm.size} {bm[:5]}", flush=True)


stream = torch.cuda.Stream(dev)
with CapacityEngine(0, 1) as eng:
    eng.reserve(n, cpu.numel(), S)
    with torch.cuda.stream(stream):
        for it in range(5):
            eng.capacity_partial_async(cl.node_ptr, ptr, cpu, mem, *a, uc, um, T(sc), T(sm),
                                       partial, stream=stream)
            torch.cuda.synchronize()
            check(f"step {it}", uc, um)
    node_of = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int32),
                                      torch.diff(ptr))
    g = torch.Generator(device=dev)
    g.manual_seed(20261016)
    perm = torch.randperm(cpu.numel(), device=dev, generator=g)
    key, kc, km = node_of[perm].contiguous(), cpu[perm].contiguous(), mem[perm].contiguous()
    o1 = torch.empty(n, dtype=torch.int64, device=dev)
    o2 = torch.empty(n, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # without this the first call reads inputs still being made
    with torch.cuda.stream(stream):
        for it in range(4):
            eng.reduce_requests_keyed_async(n, key, kc, km, o1, o2, stream=stream)
            torch.cuda.synchronize()
            check(f"keyed {it}", o1, o2)
    print("node_of check:", bool(torch.equal(torch.bincount(node_of, minlength=n).cpu(),
                                             torch.from_numpy(np.diff(cl.node_ptr)))))
