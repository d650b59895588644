"""Benchmark: node x spec fit evaluations per second (BASELINE.json metric).

One step = one pass of the hot path over the resident synthetic cluster:
  segmented request reduce (CC:290-293) -> fit prepare (spec partition, per-node
  free capacity) -> nodes x specs fit kernel (CC:119-138) -> [RCCL all-reduce of the
  per-spec partials when N > 1] -> finalize (totals + div-by-zero flags).
Inputs are resident in HBM before the timed region; value = nodes x specs of the
whole job / step time (max over ranks).

Default workload = BASELINE config C4 (1M nodes, ~20M pods / ~40M containers, 4096
specs), which fits one MI355X.  --gpus N: one process per GPU; the SAME 1M-node
cluster is split into N contiguous node ranges (strong scaling, BASELINE configs[3]:
"1M nodes x 20M pods, 4096 specs, nodes sharded over 2/4/8 MI355X") and the only
exchange is the sum of the per-spec partials: by default one kernel on the kernels' own
stream that pushes each rank's partial into every peer's mailbox over xGMI peer memory,
waits for the peers' pushes and finalizes (kcc_exchange_finalize_async, --exchange p2p);
--exchange kcc: libkcc's RCCL all-reduce (kcc_allreduce_partial_async) + finalize.  Launched without torchrun
(`python bench.py --gpus N`), the script re-launches itself under
torch.distributed.run with N ranks before anything touches the GPU.  --scaling weak
(one C4-sized partition per rank, an N x 1M-node cluster) is a secondary mode.
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
# the same loop with the pod-slot clamp applied inside it (kcc_set_clamp_in_fit; small
# shards): min, compare, select, the clamp values by vector loads (tests/test_isa.py)
FIT_NC_VALU_PER_NODE_WAVE = 5.0
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 4  # wave-instructions / s
METRIC = "node×spec fit evals/sec at 1M nodes × 4K specs; % of HBM roofline"
# per-launch HBM traffic of each kernel from rocprofv3 PMC passes of this same bench
# command (scripts/profile.sh + scripts/summarize_prof.py); null when absent
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(kernel, shard=None):
    """HBM bytes per launch of `kernel` from profiles/pmc_traffic.json: the N = 1 C4 bench's
    PMC passes, or (shard = "<config>/w<W>") rank 0's shard of a W-way split."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
        # (the profiles name a kernel as rocprofv3 printed it in their round: `fit_kernel`
        # in round 3, `fit_kernel<false>` / `<true>` since; `reduce_kernel<2>` before round
        # 6, `reduce_kernel<2, false>` / `<2, true>` (node prep in the launch) since)
        names = {"fit_kernel": ("fit_kernel", "fit_kernel<false>", "fit_kernel<true>"),
                 "reduce_kernel<2>": ("reduce_kernel<2>", "reduce_kernel<2, false>",
                                      "reduce_kernel<2, true>")}.get(kernel, (kernel,))
        e = t["shards"][shard] if shard else t
        ks = e["kernels"]
        name = next(k for k in names if k in ks)
        src = f"{e['source']} (rank 0's shard {shard})" if shard else t["source"]
        return ks[name]["hbm_bytes_per_launch"], src
    except (OSError, KeyError, ValueError, TypeError, StopIteration):
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the config's cluster split over the ranks; "
                         "weak: a config-sized node partition per rank")
    ap.add_argument("--exchange", default="p2p", choices=["p2p", "kcc", "torch"],
                    help="N > 1: the partials' sum by one push-wait-finalize kernel over xGMI "
                         "peer memory (p2p, default), libkcc's own RCCL all-reduce on the "
                         "kernel stream (kcc), or torch.distributed.all_reduce (torch)")
    ap.add_argument("--chunks", type=int, default=1,
                    help="node chunks of the pipelined step (reduce of chunk k overlaps the fit "
                         "of chunk k-1); 1 = reduce, then fit")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--clamp-in-fit", type=int, default=-1, choices=[-1, 0, 1],
                    help="pod-slot clamp inside the fit: -1 by shard size (default), 0 never "
                         "(clamp correction launch), 1 whenever specs <= 4096")
    ap.add_argument("--no-dense", action="store_true",
                    help="skip the dense-layout comparison steps (every row through the fit)")
    ap.add_argument("--no-pods", action="store_true",
                    help="skip the opt-in scheduler pod-request leg (SURVEY §8f row 4)")
    ap.add_argument("--no-keyed", action="store_true",
                    help="skip the list-order (keyed) reduce leg (SURVEY §8f row 1)")
    ap.add_argument("--no-parse", action="store_true",
                    help="skip the quantity-string parse leg (SURVEY §8f row 2)")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip the cold-cache steps (a 1 GiB read between steps evicts the "
                         "256 MiB Infinity Cache and the L2s; roofline.frac_cold)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU time of the oracle's fit sample")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, production); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostic: run only rank 0's node shard of a world of this size "
                         "(no all-reduce) to estimate per-rank step time at N GPUs")
    ap.add_argument("--kernel-events", default="after", choices=["timed", "after"],
                    help="per-kernel HIP events inside the timed steps (timed) or in as many "
                         "extra steps after them (after)")
    ap.add_argument("--graph", type=int, default=0, choices=[0, 1],
                    help="1: the timed steps replay one step captured into a HIP graph "
                         "(torch.cuda.CUDAGraph on the bench stream; every kernel still runs "
                         "each step); not with --exchange torch")
    ap.add_argument("--lib", default=None,
                    help="diagnostic A/B: load this libkcc build (variants/libkcc_NAME.so) "
                         "instead of the release library; the line names it")
    ap.add_argument("--drill-exchange-fallback", action="store_true",
                    help="test drill (N > 1): treat the p2p exchange's pre-timing check as failed "
                         "on the last rank, so every rank takes the RCCL fallback path")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: start the ranks, exchange one gloo "
                         "all-reduce, print the rank count (no measurement)")
    return ap.parse_args()


def relaunch(args) -> int:
    """`python bench.py --gpus N` (N > 1) outside torchrun: run the N ranks under
    torch.distributed.run as a CHILD process and return its exit code.  This process
    never initialises the GPU (no exec from a GPU-initialised process)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


# per-rank timings every N > 1 line carries (rank_stats): the step, each rank's reduce and
# fit launches, its all-reduce of the partials, and its reduce's HBM roofline fraction
RANK_KEYS = ("step_ms", "reduce_ms", "fit_ms", "allreduce_ms", "reduce_frac")


def rank_stats(dist, world, local, device=None):
    """Gather every rank's RANK_KEYS values (one all_gather of a float64 vector; None ->
    NaN -> null) and summarise them: the slowest and fastest rank's step (value uses the
    slowest), the mean all-reduce time, and the per-rank lists."""
    import torch

    vec = torch.tensor([float("nan") if local.get(k) is None else float(local[k])
                        for k in RANK_KEYS], dtype=torch.float64, device=device)
    if world > 1:
        bufs = [torch.empty_like(vec) for _ in range(world)]
        dist.all_gather(bufs, vec)
        rows = [b.cpu().tolist() for b in bufs]
    else:
        rows = [vec.cpu().tolist()]
    per = {k: [None if r[i] != r[i] else r[i] for r in rows] for i, k in enumerate(RANK_KEYS)}
    steps = [v for v in per["step_ms"] if v is not None]
    ar = [v for v in per["allreduce_ms"] if v is not None]
    return {
        "step_ms_max": max(steps) if steps else None,
        "step_ms_min": min(steps) if steps else None,
        "allreduce_ms": sum(ar) / len(ar) if ar else None,
        "per_rank": per,
        "note": "step_ms: each rank's own timed steps (value uses the max); reduce_ms / fit_ms "
                "/ allreduce_ms: per launch, HIP events on the kernels' stream in the profiled "
                "steps; reduce_frac: that rank's reduce_kernel at algorithmic bytes / 8 TB/s",
    }


def dry_run(args, rank, world):
    """The launcher path without a GPU: every rank joins a gloo group and all-reduces
    its rank id; rank 0 reports how many ranks answered, and the per-rank table an N > 1
    line carries is gathered over the same group (placeholder values, no measurement)."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([1, rank], dtype=torch.int64)
        dist.all_reduce(t)
        seen, rank_sum = int(t[0]), int(t[1])
    else:
        seen, rank_sum = 1, 0
    ranks = rank_stats(dist, world, {"step_ms": 1.0 + rank, "reduce_ms": None, "fit_ms": None,
                                     "allreduce_ms": 0.5 if world > 1 else None,
                                     "reduce_frac": None})
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": seen, "gpus_requested": args.gpus,
                          "rank_sum": rank_sum, "scaling": args.scaling, "config": args.config,
                          "ranks": ranks}))
    return 0 if seen == args.gpus else 2


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but {world} rank(s) were launched (WORLD_SIZE): "
              "refusing to report a line for a different GPU count", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        sys.exit(dry_run(args, rank, world))

    import torch
    import torch.distributed as dist

    from kubernetesclustercapacity_amd import CapacityEngine, synth
    from kubernetesclustercapacity_amd.shard import node_range

    n_dev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if args.dist_backend == "nccl" and world > 1 and n_dev < int(os.environ.get(
            "LOCAL_WORLD_SIZE", world)):
        print(f"[bench] {world} ranks but {n_dev} visible GPU(s): RCCL needs one GPU per rank "
              "(use --dist-backend gloo only to rehearse ranks sharing a GPU)", file=sys.stderr)
        sys.exit(2)
    local = local % max(n_dev, 1)  # gloo rehearsal: several ranks, one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    exchange = args.exchange if args.dist_backend == "nccl" or args.exchange == "p2p" else "torch"
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
                            node_lo=lo, node_hi=hi, skew=cfg["skew"], limits=False)
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

    eng = CapacityEngine(local, 1, lib_path=args.lib)
    eng.reserve(n, C, S)
    eng.set_clamp_in_fit(args.clamp_in_fit)
    stream = torch.cuda.Stream(dev)
    exchange_note = None
    if world > 1 and exchange == "p2p":
        # every rank's mailbox handle to every rank over the process group; any failure
        # (on any rank) falls back to libkcc's RCCL all-reduce (gloo: torch's)
        try:
            handles = [None] * world
            dist.all_gather_object(handles, eng.p2p_export(world, S))
            eng.p2p_open(rank, handles)
        except Exception as e:  # noqa: BLE001 - every rank falls back the same way below
            exchange_note = f"p2p exchange setup failed ({e})"
        ok = torch.tensor([0 if exchange_note else 1], dtype=torch.int64,
                          device=dev if args.dist_backend == "nccl" else None)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            exchange = "kcc" if args.dist_backend == "nccl" else "torch"
            exchange_note = (exchange_note or "a peer's p2p setup failed") + f"; {exchange} used"
        dist.barrier()

    def setup_kcc():
        # libkcc's own RCCL communicator: rank 0's id travels over the process group;
        # returns the exchange every rank uses and a note when it is not kcc
        err_note = None
        try:
            obj = [CapacityEngine.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            eng.comm_init(obj[0], world, rank)
        except Exception as e:  # noqa: BLE001 - every rank falls back the same way below
            err_note = f"kcc communicator failed ({e}); torch.distributed all-reduce used"
        ok = torch.tensor([0 if err_note else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            return "torch", err_note or "a peer's kcc communicator failed; torch all-reduce used"
        return "kcc", None

    if world > 1 and exchange == "kcc":
        exchange, note = setup_kcc()
        exchange_note = note or exchange_note

    h_ptr = np.ascontiguousarray(cl.node_ptr, np.int64)

    ar_events = []  # profiled steps: HIP event pairs around the all-reduce (its stream)

    def step(prof=False):
        # reduce + spec ranks -> node prep + spec placement -> fit -> clamp correction,
        # one stream; one rank: the finalize rides in the clamp correction's launch
        if world == 1 and args.chunks <= 1:
            eng.capacity_async(h_ptr, ptr, cpu, mem, a_cpu, a_mem, a_pods, p_cnt, used_cpu,
                               used_mem, s_cpu, s_mem, totals, err, stream=stream)
            return
        eng.capacity_partial_async(h_ptr, ptr, cpu, mem, a_cpu, a_mem, a_pods, p_cnt, used_cpu,
                                   used_mem, s_cpu, s_mem, partial, n_chunks=args.chunks,
                                   stream=stream)
        if world > 1:
            if prof:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(stream)
            if exchange == "p2p":  # push, wait, sum and finalize: one kernel, same stream
                eng.exchange_finalize_async(S, partial, totals, err, stream=stream)
            elif exchange == "kcc":  # RCCL on the same stream: no cross-stream event
                eng.allreduce_partial_async(S, partial, stream=stream)
            else:
                dist.all_reduce(partial, op=dist.ReduceOp.SUM)
            if prof:
                ev[1].record(stream)
                ar_events.append(ev)
            if exchange == "p2p":
                return
        eng.fit_finalize_async(S, partial, totals, err, stream=stream)

    def exchange_verified(drill=False):
        """One step with the current exchange, checked on every rank before anything is
        timed: its totals / spec_err against the process group's all-reduce of the same
        partials + the library's finalize, and no device wait gave up (reduce look-back,
        exchange flag).  True only when every rank agrees (ClusterCapacity.go:138 summed
        over the node shards)."""
        with torch.cuda.stream(stream):
            eng.capacity_partial_async(h_ptr, ptr, cpu, mem, a_cpu, a_mem, a_pods, p_cnt,
                                       used_cpu, used_mem, s_cpu, s_mem, partial,
                                       n_chunks=args.chunks, stream=stream)
            own = partial.clone()
            totals.fill_(-1)
            if exchange == "p2p":
                eng.exchange_finalize_async(S, partial, totals, err, stream=stream)
            elif exchange == "kcc":
                eng.allreduce_partial_async(S, partial, stream=stream)
                eng.fit_finalize_async(S, partial, totals, err, stream=stream)
        torch.cuda.synchronize()
        if exchange == "torch":
            dist.all_reduce(partial, op=dist.ReduceOp.SUM)
            with torch.cuda.stream(stream):
                eng.fit_finalize_async(S, partial, totals, err, stream=stream)
            torch.cuda.synchronize()
        ref = own if args.dist_backend == "nccl" else own.cpu()
        dist.all_reduce(ref, op=dist.ReduceOp.SUM)
        ref_t, ref_e = torch.empty_like(totals), torch.empty_like(err)
        with torch.cuda.stream(stream):
            eng.fit_finalize_async(S, ref.to(dev), ref_t, ref_e, stream=stream)
        torch.cuda.synchronize()
        good = (torch.equal(ref_t, totals) and torch.equal(ref_e, err) and
                eng.p2p_faults() == 0 and eng.reduce_faults() == 0 and
                not (drill and rank == world - 1))
        flag = torch.tensor([1 if good else 0], dtype=torch.int64,
                            device=dev if args.dist_backend == "nccl" else None)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    verified = None
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            # the exchange proves itself before anything is timed: a p2p exchange that
            # disagrees falls back to libkcc's RCCL all-reduce (every rank), and a line is
            # only printed for totals the process group's own all-reduce reproduces
            tried = [exchange]
            ok = exchange_verified(drill=args.drill_exchange_fallback and exchange == "p2p")
            if not ok and exchange == "p2p":
                eng.clear_faults()  # (the failed exchange may have set the fault words)
                if args.dist_backend == "nccl":
                    exchange, note = setup_kcc()
                else:
                    exchange, note = "torch", None
                exchange_note = ("p2p exchange failed its pre-timing check (totals vs the process "
                                 f"group's all-reduce + finalize, fault words); {exchange} used"
                                 + (f"; {note}" if note else ""))
                tried.append(exchange)
                ok = exchange_verified()
            if not ok:
                print(f"[bench] rank {rank}: the exchange failed its pre-timing check "
                      f"({' then '.join(tried)}): no line is reported for unverified totals",
                      file=sys.stderr, flush=True)
                dist.destroy_process_group()
                sys.exit(3)
            verified = {"verified_before_timing": True, "exchanges_tried": tried,
                        "exchange": exchange,
                        "check": "one step's totals / spec_err == the process group's all-reduce "
                                 "of the same partials + kcc_fit_finalize_async, no device wait "
                                 "gave up, on every rank"}
            for _ in range(max(args.warmup, 1)):
                step()
            torch.cuda.synchronize()
        # --graph: one whole step (every launch, the exchange included) captured after the
        # warm-up and the exchange check (workspaces allocated; the library's epochs live
        # on the device, include/kcc.h), replayed for each timed step; its per-kernel
        # events come from eager steps after the timed region
        graph = None
        if args.graph and exchange != "torch":
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                step()
            graph.replay()
            torch.cuda.synchronize()
        run = graph.replay if graph is not None else step
        # per-launch kernel durations from HIP events the library records on the stream
        # each kernel runs on: over exactly the timed steps (--kernel-events timed), or
        # over as many extra steps right after them (after: the timed region has no events)
        eng.profile_enable(args.kernel_events == "timed" and graph is None)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t_end = time.perf_counter()
        if args.kernel_events == "after" or graph is not None:
            eng.profile_enable(True)
            for _ in range(args.steps):
                step(prof=True)
            torch.cuda.synchronize()
    red_ms_tot, red_launches, fit_ms_tot, fit_launches = eng.profile_read()
    eng.profile_enable(False)
    cold = None if args.no_cold else cold_leg(eng, step, stream, dev, args.steps, dist, world)
    ar_ms = (sum(a.elapsed_time(b) for a, b in ar_events) / len(ar_events)) if ar_events else None
    elapsed = t_end - t_start
    own_ms_step = elapsed / args.steps * 1e3  # this rank's own timed steps
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

    # the fit's node stream: the rows that can add to its fast sum (free CPU, free memory,
    # pods > 0; every other row adds exactly 0 there), compacted by node_prep
    streamed = eng.fit_stream_rows()
    clamp_in_fit = eng.clamp_in_fit_used()
    valu_pn = FIT_NC_VALU_PER_NODE_WAVE if clamp_in_fit else FIT_VALU_PER_NODE_WAVE

    # algorithmic bytes per launch (DESIGN.md "Roofline accounting"): a step runs
    # `chunks` reduce launches and `chunks` fit launches over node ranges of ~n/chunks
    fit_bytes = (streamed * (20 if clamp_in_fit else 16) + chunks * (S * 48 + S * 8)) / chunks  # FitGroupA (+ clamp values) + specs in, totals out
    red_bytes = (C * 16 + (n + 1) * 8 + n * 16) / chunks       # requests + CSR offsets in, sums out
    fit_gbs = fit_bytes / (fit_ms * 1e-3) / 1e9
    fit_instr = streamed * ((S + 63) // 64) * valu_pn
    fit_valu = fit_instr / chunks / (fit_ms * 1e-3)
    red_gbs = red_bytes / (red_ms * 1e-3) / 1e9
    # the clamp in the fit on one chunk: node prep's row work runs in the reduce launch
    # (kcc_abi.cpp np_fused), so its bytes are that launch's too
    np_fused = clamp_in_fit and chunks == 1
    np_bytes = n * (32 + 16) + streamed * 20  # alloc + pod_count and used_* in, stream out
    c4_alone = args.config == "C4" and world == 1 and args.emulate_world <= 1  # the profiled run
    w_eff = args.emulate_world if args.emulate_world > 1 else world
    shard_key = (f"{args.config}/w{w_eff}" if w_eff > 1 and args.scaling == "strong" and chunks == 1
                 else None)  # rank 0's shard, profiled alone
    if c4_alone or shard_key:
        fit_traffic, tsrc = pmc_traffic("fit_kernel", shard_key)
        red_traffic, _ = pmc_traffic("reduce_kernel<2>", shard_key)
        if clamp_in_fit:  # (the PMC passes profiled the clamp-correction layout)
            fit_traffic = None
    else:
        fit_traffic = red_traffic = tsrc = None

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
            "nodes": n_total, "pods": pods_total, "containers_rank0": C, "nodes_rank0": n,
            "pods_rank0": int(cl.pod_count.sum()),
            "pods_per_node": ("Zipf(s=1.2) capped at 2 x allocatable pods (SURVEY §8d); `pods` "
                              "is its expected total" if cl.meta["skew"] == "zipf" else
                              f"{cl.meta['skew']}, mean {pods_total / max(n_total, 1):g}"),
            "specs": S, "parallelism": f"node-sharded x{world}",
        },
        "world": {
            "ranks": world, "process_group_size": dist.get_world_size() if world > 1 else 1,
            "backend": args.dist_backend if world > 1 else None,
            "exchange": (("one-shot push over xGMI peer memory + finalize, one kernel "
                          "(kcc_exchange_finalize_async, kernel stream)" if exchange == "p2p" else
                          "libkcc RCCL (kcc_allreduce_partial_async, kernel stream)"
                          if exchange == "kcc" else f"torch.distributed.all_reduce ({args.dist_backend})")
                         if world > 1 else None),
            "exchange_note": exchange_note,
            "visible_gpus": n_dev,
        },
        # the dominant kernel of the step (longest per step): its HBM roofline
        "roofline": None,
        "roofline_fit": {
            "bound": "hbm", "kernel": "fit_kernel", "achieved": fit_gbs, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": fit_gbs / HBM_PEAK_GBS, "traffic": fit_traffic,
            "traffic_source": tsrc and f"profiles/pmc_traffic.json ({tsrc}); bytes per launch",
            "bytes_per_launch": fit_bytes, "ms_per_launch": fit_ms,
            "note": "the fit is VALU-bound (min(findMin(qc, qm), P) per node and spec, "
                    f"{valu_pn:g} VALU per node and 64-spec wave): see roofline_valu",
        },
        "roofline_valu": {
            "bound": "valu", "kernel": "fit_kernel", "achieved": fit_valu / 1e9,
            "peak": VALU_ISSUE_PEAK / 1e9, "unit": "G wave-instr/s",
            "frac": fit_valu / VALU_ISSUE_PEAK,
            "valu_per_node_wave": valu_pn,
            "fit_evals_per_s": n / chunks * S / (fit_ms * 1e-3),
            "fit_streamed_pairs_per_s": streamed / chunks * S / (fit_ms * 1e-3),
            "note": "counted over the streamed rows (the instructions the kernel issues): "
                    f"{valu_pn:g} per node x wave",
        },
        "clamp": {
            "in_fit": clamp_in_fit, "mode": args.clamp_in_fit,
            "note": ("the pod-slot clamp (CC:134-135) inside the fit: 5 VALU per node x wave, no "
                     "clamp_apply launch (small shards)" if clamp_in_fit else
                     "the pod-slot clamp by the clamp correction (clamp_apply launch), the fit "
                     "at 3 VALU per node x wave"),
        },
        "fit_stream": {
            "rows": n, "rows_streamed": streamed, "fraction": streamed / max(n, 1),
            "note": "node_prep streams into the fit only rows with free CPU, free memory and "
                    "allocatable pods > 0 (padded to groups of 8); the others add exactly 0 to "
                    "its sum of min(findMin(qc, qm), P) (their clamp terms are the clamp "
                    "correction's) — same totals bit for bit (tests/test_gpu_shards_configs.py); "
                    "value counts every node x spec pair; see dense_layout",
        },
        "roofline_reduce": {
            "bound": "hbm",
            "kernel": ("reduce_kernel<2, node prep> (the launch also runs spec_place and node "
                       "prep's row work behind the reduce's workgroups, DESIGN §4.2)" if np_fused else
                       "reduce_kernel<2>" + (" (+ the spec-rank workgroups in its launch)"
                                             if chunks == 1 else "")),
            "achieved": red_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": red_gbs / HBM_PEAK_GBS, "bytes_per_launch": red_bytes, "ms_per_launch": red_ms,
            "traffic": red_traffic,
            "traffic_source": tsrc and f"profiles/pmc_traffic.json ({tsrc}); bytes per launch",
        },
        "pipeline": {"chunks": chunks, "reduce_ms_per_step": red_ms_tot / args.steps,
                     "fit_ms_per_step": fit_ms_tot / args.steps,
                     "graph": graph is not None,
                     "note": "per-kernel HIP events, recorded in --kernel-events "
                             f"{'after' if graph is not None else args.kernel_events} steps"
                             + ("; the timed steps replay one captured HIP graph"
                                if graph is not None else "")},
        "fast_path_fraction": 1.0 - (slow_pairs / pairs if pairs else 0.0),
        "gen_seconds": gen_s,
    }
    if np_fused:
        lb = red_bytes + np_bytes
        out["roofline_reduce"].update(
            launch_bytes=lb, launch_frac=lb / (red_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            launch_note="launch_bytes adds node prep's algorithmic bytes (48 B per row in, 20 B "
                        "per streamed row out) to the reduce's: the bytes the whole launch moves")
    if cold is not None:  # the same kernels with the Infinity Cache and L2s flushed
        c_red = cold["reduce_ms_per_launch"]
        c_fit = cold["fit_ms_per_launch"]
        out["roofline_reduce"].update(
            ms_per_launch_cold=c_red, achieved_cold=red_bytes / (c_red * 1e-3) / 1e9,
            frac_cold=red_bytes / (c_red * 1e-3) / 1e9 / HBM_PEAK_GBS)
        if np_fused:
            out["roofline_reduce"]["launch_frac_cold"] = (
                (red_bytes + np_bytes) / (c_red * 1e-3) / 1e9 / HBM_PEAK_GBS)
        out["roofline_valu"].update(
            ms_per_launch_cold=c_fit, frac_cold=fit_instr / chunks / (c_fit * 1e-3) / VALU_ISSUE_PEAK)
        out["cold"] = cold
    if red_ms_tot >= fit_ms_tot:
        out["roofline"] = dict(out["roofline_reduce"], kernel="reduce_kernel<2>",
                               note="dominant kernel of the step (reduce vs fit time per step); "
                                    "the fit's: roofline_fit / roofline_valu")
    else:  # the fit dominates (C5's 16384 specs): its bound is VALU issue, not HBM
        out["roofline"] = dict(out["roofline_valu"], traffic=fit_traffic,
                               note="dominant kernel of the step; VALU issue-bound (no MFMA or HBM "
                                    "bound applies: 3 VALU per node and 64-spec wave); the HBM "
                                    "view: roofline_fit")
    if args.emulate_world > 1:
        out["emulated_world"] = args.emulate_world
    # every rank's own numbers (N > 1: who is slowest, and what the exchange costs)
    out["ranks"] = rank_stats(dist, world, {"step_ms": own_ms_step, "reduce_ms": red_ms,
                                            "fit_ms": fit_ms, "allreduce_ms": ar_ms,
                                            "reduce_frac": red_gbs / HBM_PEAK_GBS},
                              device=dev if args.dist_backend == "nccl" else None)
    out["allreduce_ms"] = out["ranks"]["allreduce_ms"]
    faults = eng.reduce_faults()
    out["reduce_lookback_faults"] = faults  # 0 on a healthy device (else sums are wrong)

    # order-independent fingerprint of the per-spec totals: identical for every N
    tot_np = totals.cpu().numpy().view(np.uint64)
    out["totals_checksum"] = int(((tot_np * np.uint64(0x9E3779B97F4A7C15)) ^ (tot_np >> np.uint64(29)))
                                 .sum(dtype=np.uint64))
    out["spec_errors"] = int(err.cpu().numpy().sum())
    if verified is not None:
        out["exchange_precheck"] = verified
    if args.lib:
        out["library"] = args.lib  # a diagnostic variant build, not the release library
    if world > 1 and exchange == "p2p":
        # again after the timed steps: the p2p exchange against the process group's
        # all-reduce of the same partials + the library's finalize (every rank), and the
        # flag waits that gave up (0)
        torch.cuda.synchronize()
        rp = partial.clone() if args.dist_backend == "nccl" else partial.cpu()
        dist.all_reduce(rp, op=dist.ReduceOp.SUM)
        ref_t = torch.empty_like(totals)
        ref_e = torch.empty_like(err)
        eng.fit_finalize_async(S, rp.to(dev), ref_t, ref_e, stream=stream)
        torch.cuda.synchronize()
        same = bool(torch.equal(ref_t, totals) and torch.equal(ref_e, err))
        p2p_faults = eng.p2p_faults()
        flag = torch.tensor([1 if same and p2p_faults == 0 else 0], dtype=torch.int64,
                            device=dev if args.dist_backend == "nccl" else None)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        out["exchange_check"] = {
            "equals_allreduce_finalize": bool(int(flag.item()) == 1), "p2p_faults_rank0": p2p_faults,
            "note": "allreduce_ms is the one-shot kernel's time: push + wait + sum + finalize"}
    if not args.no_dense:  # the same step with every node row streamed through the fit
        eng.set_fit_dense(True)
        with torch.cuda.stream(stream):
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
        eng.set_fit_dense(False)
        dt = t1 - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out["dense_layout"] = {"ms_per_step": dt / args.steps * 1e3,
                               "value": n_total * S / (dt / args.steps),
                               "note": "every node row streamed through the fit (round-1 layout)"}
    if rank == 0 and world == 1 and args.emulate_world <= 1:
        out["h2d"] = h2d_leg([cl.node_ptr, cl.cpu_req, cl.mem_req, cl.alloc_cpu, cl.alloc_mem,
                              cl.alloc_pods, cl.pod_count, sc, sm], dev, ms_step, n_total * S)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cl, sc, sm, totals.cpu().numpy(), err.cpu().numpy(),
                                           args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_keyed:
        out["keyed"] = keyed_leg(eng, ptr, cpu, mem, used_cpu, used_mem, n, dev, stream,
                                 args.steps, args.warmup, c4_alone)
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


COLD_FLUSH_BYTES = 1 << 30  # 4x the 256 MiB Infinity Cache (MI355X_MICROARCH.md)


def cold_leg(eng, step, stream, dev, steps, dist, world):
    """SURVEY §7 (HBM claims need a cold cache): `steps` more steps, each behind a streamed
    read of a COLD_FLUSH_BYTES scratch buffer on the step's own stream, which evicts the
    256 MiB Infinity Cache (MI355X_MICROARCH.md: a line stays resident only while
    everything loaded or stored between two uses fits in ~256 MiB) and every XCD's 4 MiB
    L2, so each step's inputs come from HBM.  A read, not a write: a written flush leaves
    up to 256 MiB of DIRTY lines that the step itself must then write back (measured: the
    C4 reduce 0.134 -> 0.181 ms, i.e. its 657 MB plus ~256 MB of the flush's write-back);
    the read leaves clean lines, and the previous step's own writes are written back during
    the flush, outside the timed pair.  Timed: each step alone, by HIP events on its stream
    after the flush, and its reduce / fit launches by the library's per-kernel events
    (kcc_profile_*).  Not part of `value` (the timed steps are warm, back to back)."""
    import torch

    scratch = torch.zeros(COLD_FLUSH_BYTES // 8, dtype=torch.int64, device=dev)
    sink = torch.empty((), dtype=torch.int64, device=dev)
    evs = []
    eng.profile_enable(True)
    with torch.cuda.stream(stream):
        for i in range(steps):
            torch.sum(scratch, dim=0, out=sink)  # the flush: a streamed read on the step's stream
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(stream)
            step()
            ev[1].record(stream)
            evs.append(ev)
        torch.cuda.synchronize()
    red_ms, red_n, fit_ms, fit_n = eng.profile_read()
    eng.profile_enable(False)
    del scratch, sink
    step_ms = sorted(a.elapsed_time(b) for a, b in evs)
    med = step_ms[len(step_ms) // 2]
    if world > 1:
        dist.barrier()
    return {
        "ms_per_step_median": med, "ms_per_step_min": step_ms[0],
        "reduce_ms_per_launch": red_ms / max(red_n, 1),
        "fit_ms_per_launch": fit_ms / max(fit_n, 1), "steps": steps,
        "flush": f"{COLD_FLUSH_BYTES >> 20} MiB streamed read (torch.sum) on the step's "
                 "stream before each step: evicts the 256 MiB Infinity Cache and the L2s, "
                 "leaving clean lines",
        "note": "each step timed alone by HIP events on its stream (the flush outside the "
                "pair); per-kernel times from the library's events around each launch",
    }


def side_warmup(run, warmup, min_s=0.1):
    """Untimed warm-up of a leg measured beside the step: `warmup` calls, and more until
    min_s seconds of them have run.  The legs start after seconds of host-only work (the
    cluster's generation, the CPU baseline, string formatting) with the GPU idle, and three
    calls of a few hundred microseconds do not bring its clocks back: the same builds timed
    back to back in scripts/ab_variants.py ran 8-15 % faster."""
    import torch
    t0, i = time.perf_counter(), 0
    while i < warmup or time.perf_counter() - t0 < min_s:
        run()
        i += 1
        torch.cuda.synchronize()


def keyed_leg(eng, ptr, cpu, mem, used_cpu, used_mem, n, dev, stream, steps, warmup,
              with_traffic=True):
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
        side_warmup(lambda: eng.reduce_requests_keyed_async(n, key, kc, km, oc, om, stream=stream),
                    warmup)
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
    kernels = ["kb_sweep<2>", "kb_gather<2>", "kb_escape"]  # the one-sweep path
    parts = [pmc_traffic(k) if with_traffic else (None, None) for k in kernels]
    traffic = sum(t for t, _ in parts) if all(t is not None for t, _ in parts) else None
    return {
        "op": "per-row request sums of CC:290-293 from containers in list order (random)",
        "kernel": " + ".join(kernels), "containers": C, "rows": n,
        "ms_per_launch": ms, "containers_per_s": C / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": alg,
                     "traffic": traffic,
                     "traffic_source": parts[0][1] and f"profiles/pmc_traffic.json ({parts[0][1]}); "
                                                       "sum of the kernels per call",
                     "note": "one sweep (one persistent workgroup per CU, the next tile's loads in "
                             "flight): each 8192-container tile counting-sorted by bucket in "
                             "LDS into 8-B records (row in bucket, low cpu bits, memory / 64; the "
                             "rest on an escape list) written as one contiguous run, then per "
                             "pair of buckets the tiles' segments summed in LDS; keys read once, no "
                             "histogram pass, no global atomics on the common path"},
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
        side_warmup(run, warmup)
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
        side_warmup(lambda: eng.parse_cpu_millis_async(d_buf, d_off, d_out, d_st, stream=stream),
                    warmup)
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
        threads = host_cpus()["threads"]
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
        side_warmup(lambda: eng.parse_quantity_async(d_buf, d_off, d_out, d_st, stream=stream),
                    warmup)
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

    host = host_cpus()
    threads = host["threads"]
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
    # one thread, like the reference's single goroutine (CC:105): a smaller spec sample
    k1 = int(min(sc.size, max(2, target_s / 3 / max(per_spec * threads, 1e-9))))
    t = time.perf_counter()
    o1, e1 = coracle.fit(*args, sc[:k1], sm[:k1], 1)
    t_fit1 = time.perf_counter() - t
    step1_s = t_red + t_fit1 * sc.size / k1
    return {
        "value": cl.n_nodes * sc.size / step_s,
        "unit": "evals/s",
        "cores": threads,
        "kind": "port",
        "value_1thread": cl.n_nodes * sc.size / step1_s,
        "host": host,
        "sample": f"C oracle (oracle/kcc_oracle.c, -O3): full reduce over {cl.n_containers} "
                  f"containers (1 thread, {t_red:.3f}s) + fit of all {cl.n_nodes} nodes x first "
                  f"{k} of {sc.size} specs ({threads} threads, {t_fit:.2f}s; 1 thread: first "
                  f"{k1} specs, {t_fit1:.2f}s), extrapolated linearly to {sc.size} specs",
        "match": bool(np.array_equal(ot, gpu_totals[:k]) and np.array_equal(oe, gpu_err[:k])
                      and np.array_equal(o1, gpu_totals[:k1]) and np.array_equal(e1, gpu_err[:k1])),
    }


def host_cpus():
    """The host cores the CPU baseline may use: this process's CPU share (affinity,
    capped by OMP_NUM_THREADS, which the GPU box sets to the slot's 16 CPUs — nproc
    there counts the whole machine), the CPU model, and what nproc reports."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = max(1, min(aff, int(omp))) if omp.isdigit() and int(omp) > 0 else aff
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    note = ("all of this process's CPUs" if threads == aff else
            f"the box's CPU share for this GPU job: OMP_NUM_THREADS={omp} (the GPU box sets it "
            f"to the slot's CPUs); the {aff} CPUs of the affinity mask / nproc belong to the "
            "whole host, shared with the other GPU slots, and the harness asks jobs to size "
            "their worker pools to the share — so every core this job owns is used")
    return {"threads": threads, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": omp or None, "cpu_model": model, "core_budget": note}


def h2d_leg(arrays, dev, step_ms, evals):
    """the host->device upload of the step's inputs, reported beside the
    device-resident rate (never `value`): pageable numpy arrays as a caller hands them
    over (torch .to(device)), and the same bytes from pinned buffers."""
    import torch

    host = [torch.from_numpy(np.ascontiguousarray(a).view(np.int64)) for a in arrays]
    nbytes = sum(h.numel() * 8 for h in host)
    torch.cuda.synchronize()
    t = time.perf_counter()
    outs = [h.to(dev) for h in host]
    torch.cuda.synchronize()
    t_page = time.perf_counter() - t
    del outs
    pinned = [h.pin_memory() for h in host]
    dst = [torch.empty_like(h, device=dev) for h in host]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for d, h in zip(dst, pinned):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t_pin = time.perf_counter() - t
    del pinned, dst
    return {
        "bytes": nbytes,
        "ms_pageable": t_page * 1e3, "gbs_pageable": nbytes / t_page / 1e9,
        "ms_pinned": t_pin * 1e3, "gbs_pinned": nbytes / t_pin / 1e9,
        "evals_per_s_incl_pinned_h2d": evals / (step_ms * 1e-3 + t_pin),
        "note": "inputs of one step (CSR offsets, container requests, node SoA, specs) "
                "host->device; not part of `value` (inputs resident in HBM)",
    }


if __name__ == "__main__":
    main()
