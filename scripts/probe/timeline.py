"""Diagnostic: per-workgroup phase timeline of the small fit-side kernels (a
-DKCC_TIMELINE build, variants/libkcc_NAME.so).  Stamps are s_memrealtime (100 MHz),
printed in microseconds relative to node_prep's first workgroup entry.

  python scripts/probe/timeline.py [NAME] [--config C4] [--shard 8]
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
ap.add_argument("name", nargs="?", default="tl")
ap.add_argument("--config", default="C4")
ap.add_argument("--shard", type=int, default=1)
ap.add_argument("--pipeline", action="store_true",
                help="time kcc_capacity_partial_async (the bench's step, incl. the clamp in the "
                     "fit by size) instead of reduce + fit_prepare + fit_run")
ap.add_argument("--dump", default=None, help="save the raw stamp buffer (.npy) here")
a = ap.parse_args()
L = _lib.load(os.path.join(ROOT, "variants", f"libkcc_{a.name}.so"))
L.kcc_debug_timeline.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
n_all = synth.CONFIGS[a.config]["n_nodes"]
cl = synth.config_cluster(a.config, node_lo=0, node_hi=n_all // a.shard)
sc, sm = synth.config_specs(a.config)
T = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)  # noqa: E731
ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
ac, am, ap_, pc = T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)
s_cpu, s_mem = T(sc), T(sm)
n, S, nc = cl.n_nodes, sc.size, cl.n_containers
uc = torch.empty(n, dtype=torch.int64, device=dev)
um = torch.empty(n, dtype=torch.int64, device=dev)
part = torch.empty(2 * S, dtype=torch.int64, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
h = C.c_void_p()
assert L.kcc_create(C.byref(h), 0, 1) == 0
assert L.kcc_reserve(h, n, nc, S) == 0
buf = np.zeros((8192, 8), np.uint64)


def step():
    if a.pipeline:
        assert L.kcc_capacity_partial_async(h, n, nc, None, P(ptr), P(cpu), P(mem), P(ac), P(am),
                                            P(ap_), P(pc), P(uc), P(um), S, P(s_cpu), P(s_mem),
                                            P(part), 1, None) == 0
        return
    assert L.kcc_reduce_requests_async(h, n, nc, P(ptr), P(cpu), P(mem), None, None, P(uc), P(um),
                                       None, None, None) == 0
    assert L.kcc_fit_prepare_async(h, n, P(ac), P(am), P(ap_), P(pc), P(uc), P(um), S, P(s_cpu),
                                   P(s_mem), P(part), None) == 0
    assert L.kcc_fit_run_async(h, n, S, P(part), None) == 0


for _ in range(3):
    step()
torch.cuda.synchronize()
assert L.kcc_debug_timeline(buf.ctypes.data) == 0
step()
assert L.kcc_debug_timeline(buf.ctypes.data) == 0
t = buf.astype(np.float64)
if a.dump:
    np.save(a.dump, buf)
npr = t[0:1024]
# t0: node_prep's first entry, or (node prep inside the reduce launch) the reduce's first
t0 = npr[:, 2][npr[:, 2] > 0].min() if (npr[:, 2] > 0).any() else t[4096:8192, 0][t[4096:8192, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
print(f"config {a.config} shard 1/{a.shard}: {n} nodes, {S} specs")


def show(label, rows, k0, k1):
    r = rows[(rows[:, k0] > 0) & (rows[:, k1] > 0)]
    if not len(r):
        print(f"{label:36s} (none)")
        return
    d = (r[:, k1] - r[:, k0]) / 100.0
    print(f"{label:36s} n={len(r):4d} start {us(r[:, k0].min()):7.2f}..{us(r[:, k0].max()):7.2f}"
          f"  end {us(r[:, k1].min()):7.2f}..{us(r[:, k1].max()):7.2f}"
          f"  dur min/med/max {d.min():6.2f}/{np.median(d):6.2f}/{d.max():6.2f}")


if not (npr[:, 0] > 0).any():  # node prep inside the reduce launch (np_rows stamps)
    show("np_rows entry -> ranks' flag", npr, 2, 6)
    show("np_rows flag -> rows' waves done", npr, 6, 3)
    show("np_rows waves -> rows computed", npr, 3, 4)
    show("np_rows computed -> stream position", npr, 4, 5)
    show("np_rows position -> stream written", npr, 5, 1)
    show("np_rows whole", npr, 2, 1)
    rr = t[4096:8192]
    show("reduce workgroups (wave 0)", rr, 0, 1)
show("node_prep entry -> prologue done", npr, 2, 0)
show("  entry -> table loads in LDS", npr, 2, 6)
show("  member masks (LDS atomics)", npr, 6, 7)
show("  prefix counts", npr, 7, 0)
show("node_prep pass loads + phase 1", npr, 0, 3)
show("node_prep phase 2 (+barrier)", npr, 3, 4)
show("node_prep stream + records (+barrier)", npr, 4, 5)
show("node_prep last pass -> end (C flush)", npr, 5, 1)
show("node_prep whole", npr, 2, 1)
fr = t[2048:2048 + 2048]  # (the reduce's slots start at 4096)
show("fit entry -> first claim", fr, 0, 1)
show("  entry -> spec records in", fr, 0, 5)
show("  spec records -> stream length", fr, 5, 1)
show("fit loop", fr, 1, 2)
show("fit slow rows + atomics", fr, 2, 3)
show("fit whole", fr, 0, 3)
cr = t[1024:2048]
show("clamp_apply entry -> tab loaded", cr, 0, 1)
show("clamp_apply consume bin", cr, 1, 2)
show("clamp_apply suffixes", cr, 2, 3)
show("clamp_apply specs (wave 0)", cr, 3, 4)
show("clamp_apply whole", cr, 0, 4)
# clamp_apply: consume time against the bin's record count (column 5)
ok = (cr[:, 1] > 0) & (cr[:, 2] > 0)
recs, dur = cr[ok, 5], (cr[ok, 2] - cr[ok, 1]) / 100.0
order = np.argsort(-recs)[:8]
print("clamp_apply heaviest bins (records, consume us):",
      [(int(recs[i]), round(float(dur[i]), 2)) for i in order])
print("clamp_apply records total", int(recs.sum()), "median", float(np.median(recs)))
# fit: loop end times per XCD (blockIdx & 7) and claims per workgroup (column 4)
ok = (fr[:, 1] > 0) & (fr[:, 2] > 0)
idx = np.nonzero(ok)[0]
ends = us(fr[ok, 2])
claims = fr[ok, 4]
for x in range(8):
    sel = (idx & 7) == x
    if sel.any():
        print(f"fit xcd {x}: wgs {int(sel.sum())} loop end min/med/max {ends[sel].min():7.2f}/"
              f"{np.median(ends[sel]):7.2f}/{ends[sel].max():7.2f}  claims min/med/max "
              f"{int(claims[sel].min())}/{int(np.median(claims[sel]))}/{int(claims[sel].max())}")
# fit: per segment (column bx, sub-queue = XCD) loop end spread; gx columns of 256 specs
gx = (S + 255) // 256
r_ = idx >> 3
bx_ = r_ % gx
seg_end = {}
for k in range(len(idx)):
    seg_end.setdefault((int(bx_[k]), int(idx[k] & 7)), []).append(ends[k])
lo_ = np.array([min(v) for v in seg_end.values()])
hi_ = np.array([max(v) for v in seg_end.values()])
md_ = np.array([np.median(v) for v in seg_end.values()])
print(f"fit segments {len(seg_end)}: within-segment spread med/max {np.median(hi_ - lo_):.2f}/{(hi_ - lo_).max():.2f}"
      f"  segment median ends min/med/max {md_.min():.2f}/{np.median(md_):.2f}/{md_.max():.2f}")
# reduce: wave 0 of each workgroup (slots 4096 + workgroup), start/end (columns 0, 1)
rr = t[4096:8192]
okr = (rr[:, 0] > 0) & (rr[:, 1] > 0)
if okr.any():
    r0 = rr[okr, 0].min()
    st_, en_ = (rr[okr, 0] - r0) / 100.0, (rr[okr, 1] - r0) / 100.0
    print(f"reduce waves {int(okr.sum())}: start max {st_.max():.2f}  end min/p10/med/p90/max "
          f"{en_.min():.2f}/{np.percentile(en_, 10):.2f}/{np.median(en_):.2f}/{np.percentile(en_, 90):.2f}/{en_.max():.2f}")
if okr.any():
    idr = np.nonzero(okr)[0]
    for x in range(8):
        sel = (idr & 7) == x
        e = en_[sel]
        print(f"reduce xcd {x}: wgs {int(sel.sum())} end min/med/max {e.min():.2f}/{np.median(e):.2f}/{e.max():.2f}")
    # by position in the grid (dispatch order): quartiles of workgroup index
    for qd in range(4):
        sel = (idr >= qd * len(rr) // 4) & (idr < (qd + 1) * len(rr) // 4)
        if sel.any():
            print(f"reduce wg quarter {qd}: end med {np.median(en_[sel]):.2f} max {en_[sel].max():.2f}")
