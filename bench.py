"""Benchmark: node x spec fit evaluations per second (BASELINE.json metric).

One step = one pass of the hot path over the resident synthetic cluster:
  segmented request reduce (CC:290-293) -> fit prepare (spec partition, per-node
  free capacity) -> nodes x specs fit kernel (CC:119-138) -> [RCCL all-reduce of the
  per-spec partials when N > 1] -> finalize (totals + div-by-zero flags).
Inputs are resident in HBM before the timed region; value = nodes x specs of the
whole job / step time (max over ranks).

Default workload = BASELINE config C4 (1M nodes, ~20M pods / ~40M containers, 4096
specs), which fits one MI355X.  --gpus N (one process per GPU, torch.distributed.run):
the cluster is partitioned by nodes; by default each rank owns one C4-sized partition
of an N x 1M-node cluster (weak scaling: N=1 is exactly C4) and the only exchange is
the RCCL all-reduce of the per-spec partials.  --scaling strong shards the same 1M
nodes over the N ranks instead.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU accounting of the fit kernel (DESIGN.md "Roofline accounting"):
#  - VALU instructions per (node, 64-spec wavefront) on the fast path, counted in the
#    kernel's ISA (pinned by tests/test_isa.py);
#  - issue peak: one wave64 VALU instruction per SIMD per 4 cycles (PMC: every
#    SQ_INSTS_VALU costs one SQ_ACTIVE_INST_VALU quad-cycle), 256 CUs x 4 SIMDs x 2.4 GHz.
FIT_VALU_PER_NODE_WAVE = 3.0
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 4  # wave-instructions / s
METRIC = "node×spec fit evals/sec at 1M nodes × 4K specs; % of HBM roofline"
# per-launch HBM traffic of each kernel from rocprofv3 PMC passes of this same bench
# command (scripts/profile.sh + scripts/summarize_prof.py); null when absent
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(kernel):
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
        return t["kernels"][kernel]["hbm_bytes_per_launch"], t["source"]
    except (OSError, KeyError, ValueError):
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--scaling", default="weak", choices=["strong", "weak"],
                    help="weak: a C4-sized node partition per rank; strong: C4 split over ranks")
    ap.add_argument("--chunks", type=int, default=1,
                    help="node chunks of the pipelined step (reduce of chunk k overlaps the fit "
                         "of chunk k-1); 1 = reduce, then fit")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pods", action="store_true",
                    help="skip the opt-in scheduler pod-request leg (SURVEY §8f row 4)")
    ap.add_argument("--no-keyed", action="store_true",
                    help="skip the list-order (keyed) reduce leg (SURVEY §8f row 1)")
    ap.add_argument("--no-parse", action="store_true",
                    help="skip the quantity-string parse leg (SURVEY §8f row 2)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU time of the oracle's fit sample")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, production); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostic: run only rank 0's node shard of a world of this size "
                         "(no all-reduce) to estimate per-rank step time at N GPUs")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from kubernetesclustercapacity_amd import CapacityEngine, synth
    from kubernetesclustercapacity_amd.shard import node_range

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: running {world} rank(s)",
              file=sys.stderr)
    local = local % max(torch.cuda.device_count(), 1)  # rehearsal: several ranks, one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    cfg = synth.CONFIGS[args.config]
    n_total = cfg["n_nodes"] * (world if args.scaling == "weak" else 1)
    pods_total = cfg["pods"] * (world if args.scaling == "weak" else 1)
    lo, hi = node_range(n_total, rank, world)
    if args.emulate_world > 1:
        lo, hi = node_range(n_total, 0, args.emulate_world)
    t0 = time.time()
    cl = synth.make_cluster(n_total, pods_total, seed=20261015 + int(args.config[1:]),
                            node_lo=lo, node_hi=hi, skew=cfg["skew"])
    sc, sm = synth.config_specs(args.config)
    n, S, C = cl.n_nodes, sc.size, cl.n_containers
    gen_s = time.time() - t0

    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    ptr, cpu, mem = T(cl.node_ptr), T(cl.cpu_req), T(cl.mem_req)
    a_cpu, a_mem, a_pods, p_cnt = T(cl.alloc_cpu), T(cl.alloc_mem), T(cl.alloc_pods), T(cl.pod_count)
    s_cpu, s_mem = T(sc), T(sm)
    used_cpu = torch.empty(n, dtype=torch.int64, device=dev)
    used_mem = torch.empty(n, dtype=torch.int64, device=dev)
    partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
    totals = torch.empty(S, dtype=torch.int64, device=dev)
    err = torch.empty(S, dtype=torch.int32, device=dev)

    eng = CapacityEngine(local, 1)
    eng.reserve(n, C, S)
    stream = torch.cuda.Stream(dev)

    h_ptr = np.ascontiguousarray(cl.node_ptr, np.int64)

    def step():
        # reduce (side stream, node chunk k) overlapped with the fit of chunk k-1
        eng.capacity_partial_async(h_ptr, ptr, cpu, mem, a_cpu, a_mem, a_pods, p_cnt, used_cpu,
                                   used_mem, s_cpu, s_mem, partial, n_chunks=args.chunks,
                                   stream=stream)
        if world > 1:
            dist.all_reduce(partial, op=dist.ReduceOp.SUM)
        eng.fit_finalize_async(S, partial, totals, err, stream=stream)

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        # per-launch kernel durations from HIP events the library records on the stream
        # each kernel runs on, over exactly the timed steps
        eng.profile_enable(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t_end = time.perf_counter()
    red_ms_tot, red_launches, fit_ms_tot, fit_launches = eng.profile_read()
    eng.profile_enable(False)
    elapsed = t_end - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / args.steps * 1e3
    chunks = fit_launches // args.steps
    red_ms = red_ms_tot / max(red_launches, 1)   # per launch
    fit_ms = fit_ms_tot / max(fit_launches, 1)
    slow_pairs, pairs = eng.fit_slow_pairs()
    value = n_total * S / (elapsed / args.steps)
    if args.emulate_world > 1:  # per-rank rate x world (no all-reduce): an upper bound
        value = n * S * args.emulate_world / (elapsed / args.steps)

    # algorithmic bytes per launch (DESIGN.md "Roofline accounting"): a step runs
    # `chunks` reduce launches and `chunks` fit launches over node ranges of ~n/chunks
    fit_bytes = (n * 16 + chunks * (S * 48 + S * 8)) / chunks  # FitGroupA + spec records in, totals out
    red_bytes = (C * 16 + (n + 1) * 8 + n * 16) / chunks       # requests + CSR offsets in, sums out
    fit_gbs = fit_bytes / (fit_ms * 1e-3) / 1e9
    fit_valu = n / chunks * ((S + 63) // 64) * FIT_VALU_PER_NODE_WAVE / (fit_ms * 1e-3)
    red_gbs = red_bytes / (red_ms * 1e-3) / 1e9
    fit_traffic, tsrc = pmc_traffic("fit_kernel") if args.config == "C4" and world == 1 else (None, None)
    red_traffic, _ = pmc_traffic("reduce_kernel<2>") if tsrc else (None, None)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded SURVEY §8d generator, kubernetesclustercapacity_amd/synth.py)",
        "config": {
            "workload": f"{args.config}: {n_total} nodes x {pods_total} pods x {S} specs; "
                        "reduce + fit prepare + fit + finalize"
                        + (" + RCCL all-reduce" if world > 1 else ""),
            "nodes": n_total, "pods": pods_total, "containers_rank0": C, "specs": S,
            "parallelism": f"node-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm", "kernel": "fit_kernel", "achieved": fit_gbs, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": fit_gbs / HBM_PEAK_GBS, "traffic": fit_traffic,
            "traffic_source": tsrc and f"profiles/pmc_traffic.json ({tsrc}); bytes per launch",
            "bytes_per_launch": fit_bytes, "ms_per_launch": fit_ms,
            "note": "fit is VALU-bound (no contraction, 64-bit compare/divide work per eval); "
                    "HBM frac reported per the BASELINE metric; see roofline_reduce",
        },
        "roofline_valu": {
            "bound": "valu", "kernel": "fit_kernel", "achieved": fit_valu / 1e9,
            "peak": VALU_ISSUE_PEAK / 1e9, "unit": "G wave-instr/s",
            "frac": fit_valu / VALU_ISSUE_PEAK,
            "valu_per_node_wave": FIT_VALU_PER_NODE_WAVE,
            "fit_evals_per_s": n / chunks * S / (fit_ms * 1e-3),
        },
        "roofline_reduce": {
            "bound": "hbm", "kernel": "reduce_kernel<2> (its mark runs inside the spec_rank launch)",
            "achieved": red_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": red_gbs / HBM_PEAK_GBS, "bytes_per_launch": red_bytes, "ms_per_launch": red_ms,
            "traffic": red_traffic,
        },
        "pipeline": {"chunks": chunks, "reduce_ms_per_step": red_ms_tot / args.steps,
                     "fit_ms_per_step": fit_ms_tot / args.steps,
                     "note": "reduce launches run on a side stream under the fit launches; "
                             "their durations include that overlap"},
        "fast_path_fraction": 1.0 - (slow_pairs / pairs if pairs else 0.0),
        "gen_seconds": gen_s,
    }
    if args.emulate_world > 1:
        out["emulated_world"] = args.emulate_world

    # order-independent fingerprint of the per-spec totals: identical for every N
    tot_np = totals.cpu().numpy().view(np.uint64)
    out["totals_checksum"] = int(((tot_np * np.uint64(0x9E3779B97F4A7C15)) ^ (tot_np >> np.uint64(29)))
                                 .sum(dtype=np.uint64))
    out["spec_errors"] = int(err.cpu().numpy().sum())
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cl, sc, sm, totals.cpu().numpy(), err.cpu().numpy(),
                                           args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_keyed:
        out["keyed"] = keyed_leg(eng, ptr, cpu, mem, used_cpu, used_mem, n, dev, stream,
                                 args.steps, args.warmup)
    if rank == 0 and world == 1 and not args.no_pods:
        out["pods"] = pods_leg(eng, ptr, cpu, mem, n, dev, stream, args.steps, args.warmup)
    if rank == 0 and world == 1 and not args.no_parse:
        del ptr, cpu, mem
        out["parse"] = parse_leg(eng, cl, dev, stream, args.steps, args.warmup,
                                 not args.no_cpu_baseline)
    eng.close()
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def keyed_leg(eng, ptr, cpu, mem, used_cpu, used_mem, n, dev, stream, steps, warmup):
    """SURVEY §8f row 1, measured beside the step (not part of `value`): the C4 containers
    in a random order (a cluster-wide pod List, without even a pod's containers kept
    together: every container is its own run, the atomic worst case), each keyed by its
    node's row -> per-row sums (kcc_reduce_requests_keyed), checked equal to the CSR
    reduce of the step.  Algorithmic bytes per launch: C x (4 key + 16 requests) in,
    n x 16 sums out."""
    import torch

    C = cpu.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(20261016)
    perm = torch.randperm(C, device=dev, generator=g)
    node_of = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int32),
                                      torch.diff(ptr))
    key = node_of[perm].contiguous()
    kc, km = cpu[perm].contiguous(), mem[perm].contiguous()
    del perm, node_of
    oc = torch.empty(n, dtype=torch.int64, device=dev)
    om = torch.empty(n, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # the inputs above were made on torch's current stream
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            eng.reduce_requests_keyed_async(n, key, kc, km, oc, om, stream=stream)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(steps):
            eng.reduce_requests_keyed_async(n, key, kc, km, oc, om, stream=stream)
        ev1.record(stream)
        torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    diff_rows = int(((oc != used_cpu) | (om != used_mem)).sum().item())
    alg = C * 20 + n * 16
    gbs = alg / (ms * 1e-3) / 1e9
    del key, kc, km, oc, om
    return {
        "op": "per-row request sums of CC:290-293 from containers in list order (random)",
        "kernel": "kb_hist + kb_scan + kb_scatter<2> + kb_accum<2>", "containers": C, "rows": n,
        "ms_per_launch": ms, "containers_per_s": C / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": alg,
                     "note": "bucketed: LDS histograms, staged scatter, LDS accumulation; "
                             "no global atomics"},
        "equals_csr_reduce": diff_rows == 0, "rows_differing": diff_rows,
    }


def pods_leg(eng, ptr, cpu, mem, n, dev, stream, steps, warmup):
    """SURVEY §8f row 4 (opt-in scheduler request model, NOT the reference's semantics),
    measured beside the step: the C4 containers cut into pods (a pod starts at every node
    start and with probability 1/2 at any other container: ~2 containers per pod), one
    init container on every third pod (30 % of them restartable sidecars), overhead on
    every fifth pod -> per-pod effective requests (pod_requests_kernel).  Algorithmic bytes
    per launch: P x 16 (app + init offsets) + C x 16 + I x 17 + P x 16 (overhead) in,
    P x 16 out.  Checked: with the init containers and overhead dropped, the per-node sums
    of the pod requests equal the step's CSR reduce."""
    import torch

    C = cpu.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(20261017)
    start = torch.rand(C, device=dev, generator=g) < 0.5
    start[ptr[:-1][torch.diff(ptr) > 0]] = True
    pod_ptr = torch.cat([torch.nonzero(start).flatten(),
                         torch.tensor([C], device=dev, dtype=torch.int64)])
    P = pod_ptr.numel() - 1
    node_pod_ptr = torch.cat([torch.zeros(1, device=dev, dtype=torch.int64),
                              torch.cumsum(start.to(torch.int64), 0)])[ptr]
    has_init = (torch.arange(P, device=dev) % 3) == 0
    init_ptr = torch.cat([torch.zeros(1, device=dev, dtype=torch.int64),
                          torch.cumsum(has_init.to(torch.int64), 0)])
    I = int(init_ptr[-1].item())
    init_cpu = torch.randint(0, 40, (I,), device=dev, generator=g, dtype=torch.int64) * 50
    init_mem = torch.randint(0, 256, (I,), device=dev, generator=g, dtype=torch.int64) << 26
    rst = (torch.rand(I, device=dev, generator=g) < 0.3).to(torch.uint8)
    sel = (torch.arange(P, device=dev) % 5) == 0
    ovh_cpu = torch.where(sel, 100, 0).to(torch.int64)
    ovh_mem = torch.where(sel, 1 << 27, 0).to(torch.int64)
    pc = torch.empty(P, dtype=torch.int64, device=dev)
    pm = torch.empty(P, dtype=torch.int64, device=dev)
    del start, has_init, sel
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        run = lambda: eng.pod_requests_async(pod_ptr, cpu, mem, pc, pm, init_ptr, init_cpu,
                                             init_mem, rst, ovh_cpu, ovh_mem, stream=stream)
        for _ in range(warmup):
            run()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(steps):
            run()
        ev1.record(stream)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / steps
        # default semantics (no init, no overhead): node sums == the step's reduce
        eng.pod_requests_async(pod_ptr, cpu, mem, pc, pm, stream=stream)
        uc = torch.empty(n, dtype=torch.int64, device=dev)
        um = torch.empty(n, dtype=torch.int64, device=dev)
        eng.reduce_requests_async(node_pod_ptr, pc, pm, uc, um, stream=stream)
        rc = torch.empty(n, dtype=torch.int64, device=dev)
        rm = torch.empty(n, dtype=torch.int64, device=dev)
        eng.reduce_requests_async(ptr, cpu, mem, rc, rm, stream=stream)
        torch.cuda.synchronize()
    diff_rows = int(((uc != rc) | (um != rm)).sum().item())
    alg = P * 16 + C * 16 + I * 17 + P * 16 + P * 16
    gbs = alg / (ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic("pod_requests_kernel")
    del pod_ptr, node_pod_ptr, init_ptr, init_cpu, init_mem, rst, ovh_cpu, ovh_mem, pc, pm
    return {
        "op": "opt-in scheduler pod requests: max(app sum, init max incl. sidecars) + overhead "
              "(NOT the reference's semantics)",
        "kernel": "pod_requests_kernel", "pods": P, "containers": C, "init_containers": I,
        "ms_per_launch": ms, "pods_per_s": P / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": alg, "traffic": traffic,
                     "traffic_source": tsrc},
        "default_semantics_equals_csr_reduce": diff_rows == 0, "rows_differing": diff_rows,
    }


def parse_leg(eng, cl, dev, stream, steps, warmup, with_cpu):
    """SURVEY §8f row 2, measured beside the step (not part of `value`): every container's
    canonical cpu request string (Quantity.String(), CC:280) -> convertCPUToMilis
    (CC:301-319) on the device, inputs resident in HBM.  Algorithmic bytes per launch:
    (n+1) x 8 offsets + the characters in, n x 8 values + n x 1 status out."""
    import torch

    from kubernetesclustercapacity_amd import quantity

    t0 = time.time()
    buf, off = quantity.cpu_quantity_strings(cl.cpu_req)
    fmt_s = time.time() - t0
    n = off.size - 1
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.empty(n, dtype=torch.int64, device=dev)
    d_st = torch.empty(n, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()  # the copies above ran on torch's current stream
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            eng.parse_cpu_millis_async(d_buf, d_off, d_out, d_st, stream=stream)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(steps):
            eng.parse_cpu_millis_async(d_buf, d_off, d_out, d_st, stream=stream)
        ev1.record(stream)
        torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    got = d_out.cpu().numpy().view(np.uint64)
    ok = bool((d_st.cpu().numpy() == 1).all() and np.array_equal(got, cl.cpu_req))
    nbytes = int(off[-1])
    alg = (n + 1) * 8 + nbytes + n * 9
    gbs = alg / (ms * 1e-3) / 1e9
    res = {
        "op": "convertCPUToMilis (CC:301-319) over every container's cpu request string",
        "kernel": "parse_cpu_kernel", "strings": n, "chars": nbytes,
        "ms_per_launch": ms, "strings_per_s": n / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": alg,
                     "traffic": pmc_traffic("parse_cpu_kernel")[0],
                     "traffic_source": pmc_traffic("parse_cpu_kernel")[1]},
        "round_trip_exact": ok, "format_seconds": fmt_s,
    }
    del d_buf, d_off, d_out, d_st
    res["quantity"] = quantity_leg(eng, cl, dev, stream, steps, warmup)
    if with_cpu:
        from oracle import coracle
        threads = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        ov, os_ = coracle.parse_cpu_millis(buf, off, 1)
        t1 = time.perf_counter()
        coracle.parse_cpu_millis(buf, off, threads)
        t2 = time.perf_counter()
        res["cpu_baseline"] = {
            "value": n / (t2 - t1), "unit": "strings/s", "cores": threads, "kind": "port",
            "value_1thread": n / (t1 - t0),
            "sample": f"C oracle (oracle/kcc_oracle.c) kcco_parse_cpu_millis over all {n} strings",
            "match": bool(np.array_equal(ov, got) and (os_ == 1).all()),
        }
    return res


def quantity_leg(eng, cl, dev, stream, steps, warmup):
    """SURVEY §8f row 2, the memory side: every container's canonical memory request
    string (Quantity.String()) -> Quantity.Value() (CC:285-286; apimachinery, parity
    unpinned) on the device.  Algorithmic bytes per launch: (n+1) x 8
    offsets + the characters in, n x 8 values + n x 1 status out."""
    import torch

    from kubernetesclustercapacity_amd import quantity

    buf, off = quantity.memory_quantity_strings(cl.mem_req)
    n = off.size - 1
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.empty(n, dtype=torch.int64, device=dev)
    d_st = torch.empty(n, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            eng.parse_quantity_async(d_buf, d_off, d_out, d_st, stream=stream)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(steps):
            eng.parse_quantity_async(d_buf, d_off, d_out, d_st, stream=stream)
        ev1.record(stream)
        torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    ok = bool((d_st.cpu().numpy() == 1).all() and np.array_equal(d_out.cpu().numpy(), cl.mem_req))
    nbytes = int(off[-1])
    alg = (n + 1) * 8 + nbytes + n * 9
    gbs = alg / (ms * 1e-3) / 1e9
    del d_buf, d_off, d_out, d_st
    return {
        "op": "Quantity.Value() (CC:285-286) over every container's memory request string",
        "kernel": "parse_quantity_kernel", "strings": n, "chars": nbytes,
        "ms_per_launch": ms, "strings_per_s": n / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": alg,
                     "traffic": pmc_traffic("parse_quantity_kernel")[0],
                     "traffic_source": pmc_traffic("parse_quantity_kernel")[1]},
        "round_trip_exact": ok,
    }


def cpu_baseline(cl, sc, sm, gpu_totals, gpu_err, target_s):
    """The C oracle (a restatement of the Go arithmetic, "port") on the host cores:
    full per-node reduce (1 thread, like the reference) + the fit over ALL nodes for a
    sample of the specs (pthreads over specs), extrapolated linearly in S.  Its
    totals for the sampled specs are also compared with the GPU's."""
    from oracle import coracle

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    t = time.perf_counter()
    uc, um, _, _ = coracle.reduce_requests(cl.node_ptr, cl.cpu_req, cl.mem_req)
    t_red = time.perf_counter() - t
    args = (cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, cl.pod_count, uc, um)
    k0 = min(32, sc.size)
    t = time.perf_counter()
    coracle.fit(*args, sc[:k0], sm[:k0], threads)
    per_spec = (time.perf_counter() - t) / k0
    k = int(min(sc.size, max(k0, target_s / max(per_spec, 1e-9))))
    k = max(threads, k - k % threads) if k >= threads else k
    t = time.perf_counter()
    ot, oe = coracle.fit(*args, sc[:k], sm[:k], threads)
    t_fit = time.perf_counter() - t
    step_s = t_red + t_fit * sc.size / k
    return {
        "value": cl.n_nodes * sc.size / step_s,
        "unit": "evals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"C oracle (oracle/kcc_oracle.c, -O3): full reduce over {cl.n_containers} "
                  f"containers (1 thread, {t_red:.3f}s) + fit of all {cl.n_nodes} nodes x first "
                  f"{k} of {sc.size} specs ({threads} threads, {t_fit:.2f}s), extrapolated "
                  f"linearly to {sc.size} specs",
        "match": bool(np.array_equal(ot, gpu_totals[:k]) and np.array_equal(oe, gpu_err[:k])),
    }


if __name__ == "__main__":
    main()
