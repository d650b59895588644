"""Diagnostic: per-workgroup phase timeline of the one-sweep keyed reduce (kb_sweep,
kb_gather) from a -DKCC_TIMELINE build (variants/libkcc_NAME.so).  Stamps are s_memrealtime
(100 MHz), printed in microseconds from the sweep's first workgroup entry.

  python scripts/probe/keyed_timeline.py [NAME] [--config C4]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from kubernetesclustercapacity_amd import _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("name", nargs="?", default="tlk")
ap.add_argument("--config", default="C4")
a = ap.parse_args()
L = _lib.load(os.path.join(ROOT, "variants", f"libkcc_{a.name}.so"))
L.kcc_debug_timeline_keyed.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
cl = synth.config_cluster(a.config)
T = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
n, nc = cl.n_nodes, cl.n_containers
g = torch.Generator(device=dev)
g.manual_seed(20261016)
perm = torch.randperm(nc, device=dev, generator=g)
node_of = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int32), torch.diff(ptr))
key, kc, km = node_of[perm].contiguous(), cpu[perm].contiguous(), mem[perm].contiguous()
del perm, node_of
oc = torch.empty(n, dtype=torch.int64, device=dev)
om = torch.empty(n, dtype=torch.int64, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
h = C.c_void_p()
assert L.kcc_create(C.byref(h), 0, 1) == 0
buf = np.zeros((1024, 8), np.uint64)


def call():
    assert L.kcc_reduce_requests_keyed_async(h, n, nc, P(key), P(kc), P(km), None, None, P(oc), P(om),
                                             None, None, None) == 0


for _ in range(5):
    call()
torch.cuda.synchronize()
assert L.kcc_debug_timeline_keyed(buf.ctypes.data) == 0
for rep in range(3):
    call()
    torch.cuda.synchronize()
    assert L.kcc_debug_timeline_keyed(buf.ctypes.data) == 0
    t = buf.astype(np.float64)
    sw, ga = t[512:1024], t[0:512]
    sw = sw[sw[:, 0] > 0]
    t0 = sw[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731
    pct = lambda v: " ".join(f"{np.percentile(v, q):7.1f}" for q in (0, 10, 50, 90, 100))  # noqa: E731
    print(f"--- call {rep}: {a.config}, {nc} containers -> {n} rows (percentiles 0/10/50/90/100, us)")
    print(f"sweep  start        {pct(us(sw[:, 0]))}")
    print(f"sweep  first tile   {pct(us(sw[sw[:, 1] > 0][:, 1]))}")
    print(f"sweep  end          {pct(us(sw[:, 2]))}")
    g_ = ga[ga[:, 0] > 0]
    print(f"gather workgroups {len(g_)}")
    print(f"gather start        {pct(us(g_[:, 0]))}")
    print(f"gather table ready  {pct(us(g_[:, 1]))}   (dur {pct((g_[:, 1] - g_[:, 0]) / 100)})")
    print(f"gather sums done    {pct(us(g_[:, 2]))}   (dur {pct((g_[:, 2] - g_[:, 1]) / 100)})")
    print(f"gather arrived      {pct(us(g_[:, 3]))}")
    pub = g_[g_[:, 4] > 0]
    if len(pub):
        print(f"gather published    {pct(us(pub[:, 4]))}   (dur {pct((pub[:, 4] - pub[:, 3]) / 100)})")
    last = g_[g_[:, 5] > 0]
    if len(last):
        print(f"gather last waited  {pct(us(last[:, 5]))}   (wait {pct((last[:, 5] - last[:, 3]) / 100)})")
        print(f"gather last end     {pct(us(last[:, 6]))}   (dur {pct((last[:, 6] - last[:, 5]) / 100)})")
