"""Probe: the pipelined step's per-node outputs (used_cpu/used_mem written by
kcc_capacity_partial_async into POISONED buffers) and the keyed device API, both against
the C oracle at C4.  Prints which rows differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
torch.cuda.init()
from kubernetesclustercapacity_amd import CapacityEngine, synth  # noqa: E402
from oracle import coracle  # noqa: E402

dev = torch.device("cuda", 0)
cl = synth.make_cluster(1_000_000, 20_000_000, seed=20261019)
sc, sm = synth.config_specs("C4")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
n, S = cl.n_nodes, sc.size
a = [T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)]
uc = torch.full((n,), 0x5555555555555555, dtype=torch.int64, device=dev)
um = torch.full((n,), 0x5555555555555555, dtype=torch.int64, device=dev)
partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
oc, om, _, _ = coracle.reduce_requests(cl.node_ptr, cl.cpu_req, cl.mem_req)
with CapacityEngine(0, 1) as eng:
    eng.reserve(n, cpu.numel(), S)
    eng.capacity_partial_async(cl.node_ptr, ptr, cpu, mem, *a, uc, um, T(sc), T(sm), partial)
    torch.cuda.synchronize()
    gc, gm = uc.cpu().numpy().view(np.uint64), um.cpu().numpy()
    bad = np.flatnonzero((gc != oc) | (gm != om))
    print("pipelined step: rows differing from the oracle:", bad.size, bad[:10])
    if bad.size:
        cnt = np.diff(cl.node_ptr)
        print("  their container counts:", cnt[bad[:10]], "last nonempty row:",
              np.flatnonzero(cnt)[-1], "n:", n)
    node_of = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int32),
                                      torch.diff(ptr))
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    perm = torch.randperm(cpu.numel(), device=dev, generator=g)
    key, kc, km = node_of[perm].contiguous(), cpu[perm].contiguous(), mem[perm].contiguous()
    kc_out = torch.empty(n, dtype=torch.int64, device=dev)
    km_out = torch.empty(n, dtype=torch.int64, device=dev)
    eng.reduce_requests_keyed_async(n, key, kc, km, kc_out, km_out)
    torch.cuda.synchronize()
    gc, gm = kc_out.cpu().numpy().view(np.uint64), km_out.cpu().numpy()
    bad = np.flatnonzero((gc != oc) | (gm != om))
    print("keyed (device API, random order): rows differing:", bad.size, bad[:10])
