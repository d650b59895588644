"""A/B timing of compile-time kernel variants in ONE process (interleaved rounds).

  python scripts/ab_variants.py build  NAME="-DKNOB=.." ...   (CPU: builds variants/libkcc_NAME.so)
  python scripts/ab_variants.py run [--config C4] [--rounds 5] [--reps 10] NAME ...   (GPU)

Each variant is the same sources with -D knobs (kcc_internal.h: KCC_RED_PREFETCH,
KCC_RED_TILES_PER_WAVE, ...), loaded side by side with ctypes.  Times the segmented
reduce (reduce_requests_async) and the fit (prepare + run) on the same device tensors,
checks every variant's outputs are identical, prints one JSON line per variant.
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "variants")


def build(specs):
    os.makedirs(VDIR, exist_ok=True)
    for spec in specs:
        name, _, flags = spec.partition("=")
        out = os.path.join(VDIR, f"libkcc_{name}.so")
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "kubernetesclustercapacity_amd", "csrc"),
                        "variant", f"VOUT={out}", f"EXTRA={flags}"], check=True)
        print("built", out, flags)


def run(names, config, rounds, reps, shard=1):
    import numpy as np
    import torch

    from kubernetesclustercapacity_amd import _lib, synth

    dev = torch.device("cuda", 0)
    n_all = synth.CONFIGS[config]["n_nodes"]
    cl = synth.config_cluster(config, node_lo=0, node_hi=n_all // shard)  # rank 0 of `shard`
    sc, sm = synth.config_specs(config)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
    ac, am, ap, pc = T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)
    s_cpu, s_mem = T(sc), T(sm)
    n, S, nc = cl.n_nodes, sc.size, cl.n_containers
    libs, ctxs, outs, golden = {}, {}, {}, {}
    shared_out = dict(uc=torch.empty(n, dtype=torch.int64, device=dev),
                      um=torch.empty(n, dtype=torch.int64, device=dev),
                      part=torch.empty(2 * S, dtype=torch.int64, device=dev),
                      tot=torch.empty(S, dtype=torch.int64, device=dev),
                      err=torch.empty(S, dtype=torch.int32, device=dev))
    for nm in names:
        L = _lib.load(os.path.join(VDIR, f"libkcc_{nm}.so"))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0, L.kcc_create_error()
        assert L.kcc_reserve(h, n, nc, S) == 0
        libs[nm], ctxs[nm] = L, h
        # one output set for all variants (the same addresses: placement alone moved
        # the reduce by ~7 % between contexts); compared variant by variant below
        outs[nm] = shared_out
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    stream = torch.cuda.Stream(dev)
    sh = C.c_void_p(stream.cuda_stream)

    def reduce(nm):
        o = outs[nm]
        rc = libs[nm].kcc_reduce_requests_async(ctxs[nm], n, nc, P(ptr), P(cpu), P(mem), None,
                                                None, P(o["uc"]), P(o["um"]), None, None, sh)
        assert rc == 0

    def fit(nm):
        o = outs[nm]
        L = libs[nm]
        assert L.kcc_fit_prepare_async(ctxs[nm], n, P(ac), P(am), P(ap), P(pc), P(o["uc"]),
                                       P(o["um"]), S, P(s_cpu), P(s_mem), P(o["part"]), sh) == 0
        assert L.kcc_fit_run_async(ctxs[nm], n, S, P(o["part"]), sh) == 0

    times = {nm: {"reduce": [], "fit": []} for nm in names}
    with torch.cuda.stream(stream):
        for nm in names:  # warm up; each variant's outputs kept for the comparison (the
            reduce(nm)    # partial is in the variant's internal spec order: its finalized
            fit(nm)       # totals are compared)
            o = outs[nm]
            assert libs[nm].kcc_fit_finalize_async(ctxs[nm], S, P(o["part"]), P(o["tot"]),
                                                   P(o["err"]), sh) == 0
            torch.cuda.synchronize()
            golden[nm] = {k: v.clone() for k, v in shared_out.items()}
        torch.cuda.synchronize()
        for _ in range(rounds):
            for nm in names:
                for what, fn in (("reduce", reduce), ("fit", fit)):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(reps):
                        fn(nm)
                    e1.record(stream)
                    e1.synchronize()
                    times[nm][what].append(e0.elapsed_time(e1) / reps)
    ref = names[0]
    for nm in names:
        for k in ("uc", "um", "tot", "err"):
            if not nm.startswith("diag_"):  # diagnostic builds are timing-only
                assert torch.equal(golden[nm][k], golden[ref][k]), f"{nm} differs from {ref} in {k}"
        r = times[nm]
        print(json.dumps({"variant": nm, "config": config, "shard": shard,
                          "reduce_ms_median": float(np.median(r["reduce"])),
                          "reduce_ms_min": float(np.min(r["reduce"])),
                          "fit_ms_median": float(np.median(r["fit"])),
                          "fit_ms_min": float(np.min(r["fit"])),
                          "reduce_GBps": (nc * 16 + (n + 1) * 8 + n * 16) / (np.median(r["reduce"]) * 1e-3) / 1e9,
                          "identical_outputs": not nm.startswith("diag_")}))


def run_step(names, config, rounds, reps, shard=1):
    """The whole device step (kcc_capacity_async: reduce + spec setup + node prep + fit +
    clamp / finalize, the clamp in the fit by size) on rank 0's shard of `shard`, every
    variant's totals checked equal to the first's."""
    import numpy as np
    import torch

    from kubernetesclustercapacity_amd import _lib, synth

    dev = torch.device("cuda", 0)
    n_all = synth.CONFIGS[config]["n_nodes"]
    cl = synth.config_cluster(config, node_lo=0, node_hi=n_all // shard, limits=False)
    sc, sm = synth.config_specs(config)
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
    libs, ctxs = {}, {}
    for nm in names:
        L = _lib.load(os.path.join(VDIR, f"libkcc_{nm}.so"))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0, L.kcc_create_error()
        assert L.kcc_reserve(h, n, nc, S) == 0
        libs[nm], ctxs[nm] = L, h

    def step(nm):
        assert libs[nm].kcc_capacity_async(ctxs[nm], n, nc, None, *[P(a) for a in args], P(uc),
                                           P(um), S, P(s_cpu), P(s_mem), P(tot), P(err), sh) == 0
    times = {nm: [] for nm in names}
    golden = {}
    with torch.cuda.stream(stream):
        for nm in names:
            for _ in range(3):
                step(nm)
            torch.cuda.synchronize()
            golden[nm] = (tot.clone(), err.clone())
        for _ in range(rounds):
            for nm in names:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    step(nm)
                e1.record(stream)
                e1.synchronize()
                times[nm].append(e0.elapsed_time(e1) / reps)
    ref = names[0]
    for nm in names:
        same = bool(torch.equal(golden[nm][0], golden[ref][0]) and torch.equal(golden[nm][1], golden[ref][1]))
        assert same or nm.startswith("diag_"), f"{nm} totals differ from {ref}"
        print(json.dumps({"variant": nm, "config": config, "shard": shard,
                          "step_ms_median": float(np.median(times[nm])),
                          "step_ms_min": float(np.min(times[nm])), "identical_totals": same}))


def run_keyed(names, config, rounds, reps):
    """The keyed (list-order) reduce on the config's containers in a random order (the
    bench's keyed leg), every variant checked equal to the CSR sums."""
    import numpy as np
    import torch

    from kubernetesclustercapacity_amd import _lib, synth

    dev = torch.device("cuda", 0)
    cl = synth.config_cluster(config)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
    n, nc = cl.n_nodes, cl.n_containers
    g = torch.Generator(device=dev)
    g.manual_seed(20261016)
    perm = torch.randperm(nc, device=dev, generator=g)
    node_of = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int32), torch.diff(ptr))
    key = node_of[perm].contiguous()
    kc, km = cpu[perm].contiguous(), mem[perm].contiguous()
    del perm, node_of
    want_c = torch.zeros(n, dtype=torch.int64, device=dev).index_add_(0, torch.repeat_interleave(
        torch.arange(n, device=dev), torch.diff(ptr)), cpu)
    oc = torch.empty(n, dtype=torch.int64, device=dev)
    om = torch.empty(n, dtype=torch.int64, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    stream = torch.cuda.Stream(dev)
    sh = C.c_void_p(stream.cuda_stream)
    libs, ctxs = {}, {}
    for nm in names:
        L = _lib.load(os.path.join(VDIR, f"libkcc_{nm}.so"))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0, L.kcc_create_error()
        libs[nm], ctxs[nm] = L, h

    def keyed(nm):
        assert libs[nm].kcc_reduce_requests_keyed_async(ctxs[nm], n, nc, P(key), P(kc), P(km), None,
                                                        None, P(oc), P(om), None, None, sh) == 0
    times = {nm: [] for nm in names}
    ok = {}
    with torch.cuda.stream(stream):
        for nm in names:
            keyed(nm)
            torch.cuda.synchronize()
            ok[nm] = bool(torch.equal(oc, want_c))
        for _ in range(rounds):
            for nm in names:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    keyed(nm)
                e1.record(stream)
                e1.synchronize()
                times[nm].append(e0.elapsed_time(e1) / reps)
    alg = nc * 20 + n * 16
    for nm in names:
        ms = float(np.median(times[nm]))
        print(json.dumps({"variant": nm, "config": config, "keyed_ms_median": ms,
                          "keyed_ms_min": float(np.min(times[nm])),
                          "frac": alg / (ms * 1e-3) / 8e12, "cpu_sums_equal_csr": ok[nm]}))


def run_parse(names, config, rounds, reps):
    """The quantity-string legs (bench parse / parse.quantity): the config's container cpu
    and memory request strings, kcc_parse_cpu_millis_async and kcc_parse_quantity_async,
    every variant's outputs checked equal to the first's."""
    import numpy as np
    import torch

    from kubernetesclustercapacity_amd import _lib, quantity, synth

    dev = torch.device("cuda", 0)
    cl = synth.config_cluster(config)
    legs = {}
    for leg, fmt in (("cpu", quantity.cpu_quantity_strings), ("qty", quantity.memory_quantity_strings)):
        buf, off = fmt(cl.cpu_req if leg == "cpu" else cl.mem_req)
        b = torch.from_numpy(buf).to(dev)
        o = torch.from_numpy(off.astype(np.int64)).to(dev)
        legs[leg] = (b, o, torch.empty(o.numel() - 1, dtype=torch.int64, device=dev),
                     torch.empty(o.numel() - 1, dtype=torch.int8, device=dev))
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    stream = torch.cuda.Stream(dev)
    sh = C.c_void_p(stream.cuda_stream)
    libs, ctxs = {}, {}
    for nm in names:
        L = _lib.load(os.path.join(VDIR, f"libkcc_{nm}.so"))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0, L.kcc_create_error()
        libs[nm], ctxs[nm] = L, h

    def call(nm, leg):
        b, o, out, st = legs[leg]
        fn = libs[nm].kcc_parse_cpu_millis_async if leg == "cpu" else libs[nm].kcc_parse_quantity_async
        assert fn(ctxs[nm], o.numel() - 1, P(b), b.numel(), P(o), P(out), P(st), sh) == 0

    times = {nm: {"cpu": [], "qty": []} for nm in names}
    ref = {}
    with torch.cuda.stream(stream):
        for nm in names:
            for leg in ("cpu", "qty"):
                call(nm, leg)
                torch.cuda.synchronize()
                got = (legs[leg][2].clone(), legs[leg][3].clone())
                if leg not in ref:
                    ref[leg] = got
                assert torch.equal(got[0], ref[leg][0]) and torch.equal(got[1], ref[leg][1]), (nm, leg)
        for _ in range(rounds):
            for nm in names:
                for leg in ("cpu", "qty"):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(reps):
                        call(nm, leg)
                    e1.record(stream)
                    e1.synchronize()
                    times[nm][leg].append(e0.elapsed_time(e1) / reps)
    for nm in names:
        print(json.dumps({"variant": nm, "config": config,
                          "cpu_ms_median": float(np.median(times[nm]["cpu"])),
                          "qty_ms_median": float(np.median(times[nm]["qty"])),
                          "identical_outputs": True}))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        import argparse
        ap = argparse.ArgumentParser()
        ap.add_argument("cmd")
        ap.add_argument("names", nargs="+")
        ap.add_argument("--config", default="C4")
        ap.add_argument("--rounds", type=int, default=5)
        ap.add_argument("--reps", type=int, default=10)
        ap.add_argument("--shard", type=int, default=1, help="use rank 0's nodes of this many")
        ap.add_argument("--keyed", action="store_true", help="time the keyed reduce instead")
        ap.add_argument("--parse", action="store_true", help="time the quantity-string kernels instead")
        ap.add_argument("--step", action="store_true", help="time the whole kcc_capacity_async step")
        a = ap.parse_args()
        if a.step:
            run_step(a.names, a.config, a.rounds, a.reps, a.shard)
        elif a.parse:
            run_parse(a.names, a.config, a.rounds, a.reps)
        elif a.keyed:
            run_keyed(a.names, a.config, a.rounds, a.reps)
        else:
            run(a.names, a.config, a.rounds, a.reps, a.shard)
