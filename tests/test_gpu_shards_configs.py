"""GPU: node sharding and the BASELINE configs at their own sizes.

Sharding — the per-spec totals of CC:105-140 are wrapping int64 sums over node rows,
so any split of the rows into contiguous shards must give the same totals bit for bit:
  - the library's own split (kcc_set_node_shards: k shards on one device, the
    shard/rebase logic of the host-array path, partials folded on the device);
  - the split bench.py runs per rank (kcc_capacity_partial_async on a node range of the
    resident arrays, partials summed as the RCCL all-reduce would, then finalize);
  - the library's RCCL communicator with a single rank (the all-reduce entry point);
  - bench.py itself with 2 ranks sharing GPU 0 over gloo (the launcher + exchange path)
    against its own 1-rank run.
Configs (BASELINE.json `configs`) against the C oracle, every spec, at full size:
C2 (10k x 200k pods x 1 spec), C3 (100k x 2M x 256), C4 (1M x 20M x 4096), C5 (5M nodes with
Zipf(1.2) pods per node, capped at 2 x allocatable pods — SURVEY §8d — x 16384 specs: the
whole cluster, as 8 rank shards and on one device, plus the rank-0 and rank-7 shards alone).
C1 (100 nodes x 1k pods x 1 spec) runs end to end through the host CLI in test_host.py.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from kubernetesclustercapacity_amd.shard import node_range
from oracle import coracle

pytestmark = pytest.mark.gpu
NT = min(16, len(os.sched_getaffinity(0)))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def seg_sums(node_ptr, vals):
    v = np.asarray(vals).view(np.uint64)
    cs = np.zeros(v.size + 1, np.uint64)
    np.cumsum(v, out=cs[1:])
    return cs[node_ptr[1:]] - cs[node_ptr[:-1]]


def oracle_totals(c, sc, sm):
    uc = seg_sums(c.node_ptr, c.cpu_req)
    um = seg_sums(c.node_ptr, c.mem_req).view(np.int64)
    return coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)


def capacity(engine, c, sc, sm):
    return engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                           c.alloc_pods, c.pod_count, sc, sm)


def device_shards(c, sc, sm, k):
    """bench.py's per-rank step for each of k node ranges of the resident arrays."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    torch.cuda.init()  # torch's HIP runtime before libkcc's (tests/conftest.py)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    S = sc.size
    acc = torch.zeros(2 * S, dtype=torch.int64, device=dev)
    with CapacityEngine(0, 1) as eng:
        stream = torch.cuda.Stream(dev)
        s_cpu, s_mem = T(sc), T(sm)
        for r in range(k):
            lo, hi = node_range(c.n_nodes, r, k)
            c0, c1 = int(c.node_ptr[lo]), int(c.node_ptr[hi])
            hp = c.node_ptr[lo:hi + 1] - c0           # the rank's own CSR, rebased
            n = hi - lo
            used = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]
            partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
            with torch.cuda.stream(stream):
                eng.capacity_partial_async(hp, T(hp), T(c.cpu_req[c0:c1]), T(c.mem_req[c0:c1]),
                                           T(c.alloc_cpu[lo:hi]), T(c.alloc_mem[lo:hi]),
                                           T(c.alloc_pods[lo:hi]), T(c.pod_count[lo:hi]),
                                           used[0], used[1], s_cpu, s_mem, partial, stream=stream)
            stream.synchronize()
            acc += partial                            # the all-reduce (int64 adds wrap)
        totals = torch.empty(S, dtype=torch.int64, device=dev)
        err = torch.empty(S, dtype=torch.int32, device=dev)
        with torch.cuda.stream(stream):
            eng.fit_finalize_async(S, acc, totals, err, stream=stream)
        stream.synchronize()
    return totals.cpu().numpy(), err.cpu().numpy()


# ---- BASELINE C4 at full size: every spec vs the oracle, and its shards --------------------
@pytest.fixture(scope="module")
def c4():
    return synth.config_cluster("C4"), synth.config_specs("C4")


@pytest.fixture(scope="module")
def c4_oracle(c4):
    c, (sc, sm) = c4
    return oracle_totals(c, sc, sm)


def test_c4_every_spec_vs_oracle(engine, c4, c4_oracle):
    c, (sc, sm) = c4
    t, e = capacity(engine, c, sc, sm)
    np.testing.assert_array_equal(e, c4_oracle[1])
    np.testing.assert_array_equal(t, c4_oracle[0])


@pytest.mark.parametrize("k", [2, 3, 8])
def test_c4_library_node_shards(engine, c4, c4_oracle, k):
    c, (sc, sm) = c4
    engine.set_node_shards(k)
    try:
        t, e = capacity(engine, c, sc, sm)
    finally:
        engine.set_node_shards(0)
    np.testing.assert_array_equal(e, c4_oracle[1])
    np.testing.assert_array_equal(t, c4_oracle[0])


@pytest.mark.parametrize("k", [2, 8])
def test_c4_rank_shards_like_bench(c4, c4_oracle, k):
    c, (sc, sm) = c4
    t, e = device_shards(c, sc, sm, k)
    np.testing.assert_array_equal(e, c4_oracle[1])
    np.testing.assert_array_equal(t, c4_oracle[0])


# ---- skewed (Zipf(1.2) pods per node) cluster with the adversarial slice, sharded ----------
@pytest.fixture(scope="module")
def zipf_adv():
    c = synth.make_cluster(80_003, 0, seed=55, skew="zipf", adversarial=True, chunk=4096)
    sc, sm = synth.make_specs(1000, seed=55, adversarial=True)
    return c, sc, sm, oracle_totals(c, sc, sm)


@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_zipf_adversarial_shards(engine, zipf_adv, k):
    c, sc, sm, (ot, oe) = zipf_adv
    engine.set_node_shards(k)
    try:
        t, e = capacity(engine, c, sc, sm)
    finally:
        engine.set_node_shards(0)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)
    t2, e2 = device_shards(c, sc, sm, k)
    np.testing.assert_array_equal(e2, oe)
    np.testing.assert_array_equal(t2, ot)


def test_single_rank_communicator():
    """kcc_comm_unique_id / kcc_comm_init / kcc_allreduce_partial_async with one rank:
    the all-reduce of one partial is the identity, on the kernel stream."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    torch.cuda.init()
    c = synth.make_cluster(20_000, 400_000, seed=9, chunk=4096)
    sc, sm = synth.make_specs(300, seed=9, adversarial=True)
    ot, oe = oracle_totals(c, sc, sm)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    S, n = sc.size, c.n_nodes
    with CapacityEngine(0, 1) as eng:
        eng.comm_init(CapacityEngine.comm_unique_id(), 1, 0)
        used = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]
        partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
        totals = torch.empty(S, dtype=torch.int64, device=dev)
        err = torch.empty(S, dtype=torch.int32, device=dev)
        stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(stream):
            eng.capacity_partial_async(c.node_ptr, T(c.node_ptr), T(c.cpu_req), T(c.mem_req),
                                       T(c.alloc_cpu), T(c.alloc_mem), T(c.alloc_pods),
                                       T(c.pod_count), used[0], used[1], T(sc), T(sm), partial,
                                       stream=stream)
            eng.allreduce_partial_async(S, partial, stream=stream)
            eng.fit_finalize_async(S, partial, totals, err, stream=stream)
        stream.synchronize()
    np.testing.assert_array_equal(err.cpu().numpy(), oe)
    np.testing.assert_array_equal(totals.cpu().numpy(), ot)


# ---- the other BASELINE configs at their own sizes -----------------------------------------
@pytest.mark.parametrize("name", ["C2", "C3"])
def test_config_every_spec_vs_oracle(engine, name):
    c, (sc, sm) = synth.config_cluster(name), synth.config_specs(name)
    assert c.n_nodes == synth.CONFIGS[name]["n_nodes"] and sc.size == synth.CONFIGS[name]["n_specs"]
    r = engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req)
    np.testing.assert_array_equal(r.cpu_requests, seg_sums(c.node_ptr, c.cpu_req))
    np.testing.assert_array_equal(r.memory_requests.view(np.uint64), seg_sums(c.node_ptr, c.mem_req))
    ot, oe = oracle_totals(c, sc, sm)
    t, e = capacity(engine, c, sc, sm)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize("rank", [0, 7])
def test_c5_rank_shard_every_spec_vs_oracle(engine, rank):
    """C5 = 5M nodes (Zipf(1.2) pods per node, capped at 2 x allocatable pods) x 16384 specs
    over 8 GPUs: rank 0's and rank 7's node ranges (~150M containers each)."""
    lo, hi = node_range(synth.CONFIGS["C5"]["n_nodes"], rank, 8)
    c = synth.config_cluster("C5", node_lo=lo, node_hi=hi, limits=False)
    sc, sm = synth.config_specs("C5")
    assert c.n_nodes == 625_000 and sc.size == 16384
    assert c.meta["skew"] == "zipf" and c.pod_count.mean() > 100  # the survey's heavy tail
    r = engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req)
    np.testing.assert_array_equal(r.cpu_requests, seg_sums(c.node_ptr, c.cpu_req))
    np.testing.assert_array_equal(r.memory_requests.view(np.uint64), seg_sums(c.node_ptr, c.mem_req))
    ot, oe = oracle_totals(c, sc, sm)
    t, e = capacity(engine, c, sc, sm)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


def test_c5_whole_cluster_every_spec_vs_oracle():
    """C5 at full size: 5M nodes (Zipf(1.2) pods per node, capped at 2 x allocatable pods;
    ~1.21e9 containers) x 16384 specs, every spec against the C oracle over the whole
    cluster.  Generated one 8-way rank shard at a time (host memory stays at one shard);
    the oracle's whole-cluster totals are assembled from its shard results (a spec's total
    is the wrapping sum of the shards' totals; it is flagged when any shard flags it —
    CC:138, CC:119-130).  Two device paths, both vs those totals:
      (a) the 8-GPU decomposition: each shard's kcc_capacity_partial_async on its own
          arrays, the partials summed (the all-reduce), one finalize;
      (b) one GPU: the whole cluster resident (the shards copied into one CSR), one
          kcc_capacity_async over all 5M nodes."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    N, W = synth.CONFIGS["C5"]["n_nodes"], 8
    sc, sm = synth.config_specs("C5")
    S = sc.size
    assert S == 16384
    # the whole cluster's device arrays, filled shard by shard
    n_cont, shards = 0, []
    for r in range(W):
        lo, hi = node_range(N, r, W)
        c = synth.config_cluster("C5", node_lo=lo, node_hi=hi, limits=False)
        shards.append(c)
        n_cont += c.n_containers
    assert n_cont > 1_100_000_000
    whole = {k: torch.empty(N, dtype=torch.int64, device=dev)
             for k in ("ac", "am", "ap", "pc", "uc", "um")}
    wptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
    wcpu = torch.empty(n_cont, dtype=torch.int64, device=dev)
    wmem = torch.empty(n_cont, dtype=torch.int64, device=dev)
    acc = torch.zeros(2 * S, dtype=torch.int64, device=dev)
    ot = np.zeros(S, np.uint64)
    oe = np.zeros(S, np.int32)
    s_cpu, s_mem = T(sc), T(sm)
    c_off = 0
    with CapacityEngine(0, 1) as eng:
        stream = torch.cuda.Stream(dev)
        for r, c in enumerate(shards):
            lo, hi = node_range(N, r, W)
            n, nc = c.n_nodes, c.n_containers
            # (a) this shard as one rank
            used = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]
            partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
            arrs = [T(x) for x in (c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                                   c.alloc_pods, c.pod_count)]
            with torch.cuda.stream(stream):
                eng.capacity_partial_async(c.node_ptr, *arrs, used[0], used[1], s_cpu, s_mem,
                                           partial, stream=stream)
            stream.synchronize()
            acc += partial
            # the per-node sums of the shard's reduce vs numpy
            np.testing.assert_array_equal(used[0].cpu().numpy().view(np.uint64),
                                          seg_sums(c.node_ptr, c.cpu_req))
            np.testing.assert_array_equal(used[1].cpu().numpy().view(np.uint64),
                                          seg_sums(c.node_ptr, c.mem_req))
            # (b) into the whole cluster's arrays
            wptr[lo:hi + 1] = arrs[0] + c_off
            wcpu[c_off:c_off + nc] = arrs[1]
            wmem[c_off:c_off + nc] = arrs[2]
            for k, a in zip(("ac", "am", "ap", "pc"), arrs[3:]):
                whole[k][lo:hi] = a
            c_off += nc
            # the oracle on this shard
            st, se = oracle_totals(c, sc, sm)
            ot += st.view(np.uint64)
            oe |= se
            del arrs, used, partial
            shards[r] = None
        ot = np.where(oe != 0, np.uint64(0), ot).view(np.int64)
        totals = torch.empty(S, dtype=torch.int64, device=dev)
        err = torch.empty(S, dtype=torch.int32, device=dev)
        with torch.cuda.stream(stream):
            eng.fit_finalize_async(S, acc, totals, err, stream=stream)
        stream.synchronize()
        np.testing.assert_array_equal(err.cpu().numpy(), oe)
        np.testing.assert_array_equal(totals.cpu().numpy(), ot)
        # (b) the whole cluster on one device, one call
        totals.fill_(-1)
        err.fill_(-1)
        with torch.cuda.stream(stream):
            eng.capacity_async(None, wptr, wcpu, wmem, whole["ac"], whole["am"], whole["ap"],
                               whole["pc"], whole["uc"], whole["um"], s_cpu, s_mem, totals, err,
                               stream=stream)
        stream.synchronize()
        np.testing.assert_array_equal(err.cpu().numpy(), oe)
        np.testing.assert_array_equal(totals.cpu().numpy(), ot)
        assert eng.reduce_faults() == 0


# ---- bench.py: 2 ranks (gloo, sharing GPU 0) == 1 rank -------------------------------------
def _bench(*extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C3",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-keyed",
                        "--no-pods", "--no-parse", *extra], capture_output=True, text=True,
                       timeout=100, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_two_ranks_equal_one():
    one = _bench("--gpus", "1")
    two = _bench("--gpus", "2", "--dist-backend", "gloo")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["world"]["process_group_size"] == 2 and two["scaling"] == "strong"
    assert two["config"]["nodes"] == one["config"]["nodes"] == 100_000
    assert two["config"]["nodes_rank0"] == 50_000
    assert two["totals_checksum"] == one["totals_checksum"]
    assert two["spec_errors"] == one["spec_errors"]
    # the exchange proved itself before the timed steps (p2p, no fallback needed)
    pre = two["exchange_precheck"]
    assert pre["verified_before_timing"] and pre["exchanges_tried"] == ["p2p"]
    assert two["exchange_check"]["equals_allreduce_finalize"]
    assert "exchange_precheck" not in one


def test_bench_exchange_fallback_drill():
    """--drill-exchange-fallback: the p2p pre-timing check reads as failed on the last
    rank, every rank switches to the fallback exchange (gloo: torch's all-reduce; RCCL
    under nccl), re-verifies it, and the totals are still the single-rank ones."""
    one = _bench("--gpus", "1")
    two = _bench("--gpus", "2", "--dist-backend", "gloo", "--drill-exchange-fallback")
    pre = two["exchange_precheck"]
    assert pre["verified_before_timing"] and pre["exchanges_tried"] == ["p2p", "torch"]
    assert "failed its pre-timing check" in two["world"]["exchange_note"]
    assert two["totals_checksum"] == one["totals_checksum"]


# ---- the fit's node stream: compacted (default) == every row (dense) -----------------------
def test_fit_stream_compacted_equals_dense(engine, c4, c4_oracle):
    c, (sc, sm) = c4
    t, e = capacity(engine, c, sc, sm)
    streamed = engine.fit_stream_rows()
    engine.set_fit_dense(True)
    try:
        td, ed = capacity(engine, c, sc, sm)
        dense = engine.fit_stream_rows()
    finally:
        engine.set_fit_dense(False)
    np.testing.assert_array_equal(t, c4_oracle[0])
    np.testing.assert_array_equal(td, c4_oracle[0])
    np.testing.assert_array_equal(ed, e)
    assert dense >= c.n_nodes and 0 < streamed < dense
    # streamed = the rows with free CPU, free memory and allocatable pods (whole groups)
    uc = seg_sums(c.node_ptr, c.cpu_req)
    um = seg_sums(c.node_ptr, c.mem_req).view(np.int64)
    free = (c.alloc_cpu > uc) & (c.alloc_mem > um) & (c.alloc_pods > 0)
    assert int(free.sum()) <= streamed <= int(free.sum()) + 7 * (c.n_nodes // 1024 + 1)


def test_reduce_lookback_never_timed_out_configs(engine):
    assert engine.reduce_faults() == 0
