"""Node sharding over ranks, world_size 2 on CPU with gloo.

Each rank generates only its node range of the cluster (synth is shard-stable),
computes its per-spec partial vector [sums | div-by-zero counts] (the oracle stands
in for kcc_capacity_partial_async in the CPU tests; the -m gpu test runs libkcc in every
rank, the ranks sharing one GPU), all-reduces it with
shard.allreduce_partial and applies the finalize rule.  The result must equal the
unsharded computation bit for bit — the same exchange bench.py runs over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kubernetesclustercapacity_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partial(c, sc, sm):
    from oracle import coracle
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    return np.concatenate([t, e.astype(np.int64)])


def _finalize(partial, S):
    err = partial[S:] != 0
    return np.where(err, 0, partial[:S]), err.astype(np.int32)


def _worker(rank, world, port, n, pods, S, adversarial, out):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.node_range(n, rank, world)
    c = synth.make_cluster(n, pods, seed=77, node_lo=lo, node_hi=hi, adversarial=adversarial,
                           chunk=256)
    sc, sm = synth.make_specs(S, seed=77, adversarial=adversarial)
    p = torch.from_numpy(_partial(c, sc, sm))
    shard.allreduce_partial(p)
    if rank == 0:
        t, e = _finalize(p.numpy(), S)
        np.save(out, np.concatenate([t, e.astype(np.int64)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("adversarial", [False, True])
def test_two_rank_shards_equal_whole(tmp_path, adversarial):
    n, pods, S, world = 3_001, 50_000, 40, 2
    out = str(tmp_path / "r0.npy")
    mp.spawn(_worker, args=(world, _free_port(), n, pods, S, adversarial, out), nprocs=world,
             join=True)
    got = np.load(out)
    c = synth.make_cluster(n, pods, seed=77, adversarial=adversarial, chunk=256)
    sc, sm = synth.make_specs(S, seed=77, adversarial=adversarial)
    from oracle import coracle
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    np.testing.assert_array_equal(got[:S], t)
    np.testing.assert_array_equal(got[S:], e)


def test_node_range_partitions_exactly():
    for n in (0, 1, 7, 1_000_000, 5_000_003):
        for world in (1, 2, 3, 4, 8):
            b = shard.shard_bounds(n, world)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in b]
            assert max(sizes) - min(sizes) <= 1


def _worker_gpu(rank, world, port, n, pods, S, adversarial, out):
    """As _worker, but the rank's partial comes from libkcc on cuda:0
    (kcc_capacity_partial_async: reduce + spec setup + node prep + fit + clamp
    correction of the rank's own nodes), the ranks sharing the one GPU of the box."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.node_range(n, rank, world)
    c = synth.make_cluster(n, pods, seed=77, node_lo=lo, node_hi=hi, adversarial=adversarial,
                           chunk=256)
    sc, sm = synth.make_specs(S, seed=77, adversarial=adversarial)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    nl = c.alloc_cpu.size
    uc = torch.empty(nl, dtype=torch.int64, device=dev)
    um = torch.empty(nl, dtype=torch.int64, device=dev)
    part = torch.empty(2 * S, dtype=torch.int64, device=dev)
    with CapacityEngine(0, 1) as eng:
        eng.capacity_partial_async(c.node_ptr, T(c.node_ptr), T(c.cpu_req), T(c.mem_req),
                                   T(c.alloc_cpu), T(c.alloc_mem), T(c.alloc_pods),
                                   T(c.pod_count), uc, um, T(sc), T(sm), part)
        torch.cuda.synchronize()
        p = part.cpu()  # internal spec order (the same on every rank: same specs)
        shard.allreduce_partial(p)
        if rank == 0:  # the library's finalize maps it back to caller order
            totals = torch.empty(S, dtype=torch.int64, device=dev)
            err = torch.empty(S, dtype=torch.int32, device=dev)
            eng.fit_finalize_async(S, p.to(dev), totals, err)
            torch.cuda.synchronize()
            np.save(out, np.concatenate([totals.cpu().numpy(), err.cpu().numpy().astype(np.int64)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_rank_partials_equal_whole(tmp_path, world):
    """Rank-local libkcc partials (adversarial rows: slow rows, clamp cases, wraps)
    summed over a gloo all-reduce == the oracle over the whole cluster."""
    n, pods, S = 20_011, 300_000, 300
    out = str(tmp_path / "r0.npy")
    mp.spawn(_worker_gpu, args=(world, _free_port(), n, pods, S, True, out), nprocs=world,
             join=True)
    got = np.load(out)
    c = synth.make_cluster(n, pods, seed=77, adversarial=True, chunk=256)
    sc, sm = synth.make_specs(S, seed=77, adversarial=True)
    from oracle import coracle
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    np.testing.assert_array_equal(got[:S], t)
    np.testing.assert_array_equal(got[S:], e)


def _worker_p2p(rank, world, port, n, pods, S, adversarial, steps, out, graph=False):
    """Every rank: its node shard's partial from libkcc on cuda:0, then the one-shot
    exchange (kcc_exchange_finalize_async: push to every peer's mailbox, wait, sum,
    finalize) — the ranks sharing the box's one GPU, their mailboxes mapped through IPC
    handles gathered over gloo.  Several steps in a row (both mailbox parities)."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.node_range(n, rank, world)
    c = synth.make_cluster(n, pods, seed=78, node_lo=lo, node_hi=hi, adversarial=adversarial,
                           chunk=256)
    sc, sm = synth.make_specs(S, seed=78, adversarial=adversarial)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    nl = c.alloc_cpu.size
    uc = torch.empty(nl, dtype=torch.int64, device=dev)
    um = torch.empty(nl, dtype=torch.int64, device=dev)
    part = torch.empty(2 * S, dtype=torch.int64, device=dev)
    totals = torch.empty(S, dtype=torch.int64, device=dev)
    err = torch.empty(S, dtype=torch.int32, device=dev)
    args = (T(c.node_ptr), T(c.cpu_req), T(c.mem_req), T(c.alloc_cpu), T(c.alloc_mem),
            T(c.alloc_pods), T(c.pod_count), uc, um, T(sc), T(sm), part)
    with CapacityEngine(0, 1) as eng:
        handles = [None] * world
        dist.all_gather_object(handles, eng.p2p_export(world, S))
        eng.p2p_open(rank, handles)
        dist.barrier()
        got = []
        if not graph:
            for _ in range(steps):
                eng.capacity_partial_async(c.node_ptr, *args)
                eng.exchange_finalize_async(S, part, totals, err)
                got.append(np.concatenate([totals.cpu().numpy(), err.cpu().numpy().astype(np.int64)]))
        else:
            # one eager step, then the step captured into a hipGraph and replayed `steps`
            # times, the spec set alternating between two (copied into the captured
            # buffers): each replay must push a new epoch (the device word), or a rank
            # would read the previous replay's mailbox data
            specs = [synth.make_specs(S, seed=78 + k, adversarial=adversarial) for k in (0, 1)]
            dspecs = [(T(a), T(b)) for a, b in specs]
            stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(stream):
                eng.capacity_partial_async(c.node_ptr, *args, stream=stream)
                eng.exchange_finalize_async(S, part, totals, err, stream=stream)
            stream.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
                eng.capacity_partial_async(c.node_ptr, *args, stream=stream)
                eng.exchange_finalize_async(S, part, totals, err, stream=stream)
            for k in range(steps):
                with torch.cuda.stream(stream):
                    args[9].copy_(dspecs[k % 2][0])
                    args[10].copy_(dspecs[k % 2][1])
                    totals.fill_(-1)
                    g.replay()
                stream.synchronize()
                got.append(np.concatenate([totals.cpu().numpy(), err.cpu().numpy().astype(np.int64)]))
            del g
        faults = eng.p2p_faults()
        dist.barrier()  # no rank unmaps its mailbox while a peer may still push
    np.save(out + f".{rank}.npy", np.stack(got + [np.full(2 * S, faults, np.int64)]))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,S", [(2, 300), (3, 300), (4, 5000)])
def test_gpu_p2p_exchange_equals_whole(tmp_path, world, S):
    """The one-shot xGMI exchange (bench --exchange p2p): every rank's finalized totals
    after 3 steps == the oracle over the whole cluster, no flag wait gave up.  S = 5000:
    the spec ranks by sort (S > 4096) and an exchange grid of 20 workgroups."""
    n, pods, steps = 20_011, 300_000, 3
    out = str(tmp_path / "p2p")
    mp.spawn(_worker_p2p, args=(world, _free_port(), n, pods, S, True, steps, out), nprocs=world,
             join=True)
    c = synth.make_cluster(n, pods, seed=78, adversarial=True, chunk=256)
    sc, sm = synth.make_specs(S, seed=78, adversarial=True)
    from oracle import coracle
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    for r in range(world):
        got = np.load(out + f".{r}.npy")
        assert got[-1][0] == 0, f"rank {r}: {got[-1][0]} flag waits gave up"
        for k in range(steps):
            np.testing.assert_array_equal(got[k][:S], t, err_msg=f"rank {r} step {k}")
            np.testing.assert_array_equal(got[k][S:], e, err_msg=f"rank {r} step {k}")


@pytest.mark.gpu
def test_gpu_p2p_exchange_graph_replay(tmp_path):
    """kcc_capacity_partial_async + kcc_exchange_finalize_async captured into a hipGraph on
    each of 2 ranks (sharing the GPU, mailboxes mapped through IPC) and replayed 4 times
    with the spec set alternating between two: every replay == the oracle of its specs,
    no flag wait gave up."""
    n, pods, S, world, steps = 20_011, 300_000, 300, 2, 4
    out = str(tmp_path / "p2pg")
    mp.spawn(_worker_p2p, args=(world, _free_port(), n, pods, S, True, steps, out, True),
             nprocs=world, join=True)
    c = synth.make_cluster(n, pods, seed=78, adversarial=True, chunk=256)
    from oracle import coracle
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    ref = []
    for k in (0, 1):
        sc, sm = synth.make_specs(S, seed=78 + k, adversarial=True)
        ref.append(coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm))
    for r in range(world):
        got = np.load(out + f".{r}.npy")
        assert got[-1][0] == 0, f"rank {r}: {got[-1][0]} flag waits gave up"
        for k in range(steps):
            t, e = ref[k % 2]
            np.testing.assert_array_equal(got[k][:S], t, err_msg=f"rank {r} replay {k}")
            np.testing.assert_array_equal(got[k][S:], e, err_msg=f"rank {r} replay {k}")


def _worker_fault(rank, world, port, n, pods, S, exchange, faultdiag, out, clamp_mode=-1):
    """One rank's step with the library of `faultdiag` on rank `world - 1` only (every
    bounded wait there gives up, so its reduce's look-back faults its device), the others
    the release library; then the exchange: the one-shot p2p push (`p2p`) or a gloo
    all-reduce of the partials finalized on every rank (`allreduce`)."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.node_range(n, rank, world)
    c = synth.make_cluster(n, pods, seed=79, node_lo=lo, node_hi=hi, chunk=256)
    sc, sm = synth.make_specs(S, seed=79)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    nl = c.alloc_cpu.size
    uc = torch.empty(nl, dtype=torch.int64, device=dev)
    um = torch.empty(nl, dtype=torch.int64, device=dev)
    part = torch.empty(2 * S, dtype=torch.int64, device=dev)
    totals = torch.empty(S, dtype=torch.int64, device=dev)
    err = torch.empty(S, dtype=torch.int32, device=dev)
    lib = faultdiag if rank == world - 1 else None
    with CapacityEngine(0, 1, lib_path=lib) as eng:
        eng.set_clamp_in_fit(clamp_mode)  # -1: by size (here the fit's), 0: clamp_apply
        if exchange == "p2p":
            handles = [None] * world
            dist.all_gather_object(handles, eng.p2p_export(world, S))
            eng.p2p_open(rank, handles)
            dist.barrier()
        eng.capacity_partial_async(c.node_ptr, T(c.node_ptr), T(c.cpu_req), T(c.mem_req),
                                   T(c.alloc_cpu), T(c.alloc_mem), T(c.alloc_pods),
                                   T(c.pod_count), uc, um, T(sc), T(sm), part)
        if exchange == "p2p":
            eng.exchange_finalize_async(S, part, totals, err)
        else:
            torch.cuda.synchronize()
            p = part.cpu()
            shard.allreduce_partial(p)
            eng.fit_finalize_async(S, p.to(dev), totals, err)
        torch.cuda.synchronize()
        got = np.concatenate([totals.cpu().numpy(), err.cpu().numpy().astype(np.int64),
                              [eng.reduce_faults()]])
        dist.barrier()  # no rank unmaps its mailbox while a peer may still push
    np.save(out + f".{rank}.npy", got)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("exchange,clamp_mode", [("p2p", -1), ("allreduce", -1), ("p2p", 0)])
def test_gpu_fault_reaches_every_rank(tmp_path, exchange, clamp_mode):
    """A device fault on ONE rank (its reduce's look-back gave up: the fault-path build on
    the last rank) reaches every rank's totals: the faulted rank's partial carries
    SPEC_FAULT_MARK in its div-by-zero counts, so the healthy rank's finalize — after the
    p2p exchange or after an all-reduce — marks every spec KCC_SPEC_FAULT with total 0,
    never a wrong total with spec_err 0."""
    faultdiag = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "kubernetesclustercapacity_amd", "libkcc_faultdiag.so")
    if not os.path.exists(faultdiag):
        pytest.fail("libkcc_faultdiag.so missing: __graft_entry__.build() builds it")
    n, pods, S, world = 20_011, 300_000, 300, 2
    out = str(tmp_path / "flt")
    mp.spawn(_worker_fault, args=(world, _free_port(), n, pods, S, exchange, faultdiag, out,
                                  clamp_mode), nprocs=world, join=True)
    for r in range(world):
        got = np.load(out + f".{r}.npy")
        assert (got[S:2 * S] == 2).all(), f"rank {r}: spec_err {np.unique(got[S:2 * S])}"
        assert (got[:S] == 0).all(), f"rank {r}"
        assert (got[-1] > 0) == (r == world - 1), f"rank {r} reduce faults {got[-1]}"
