"""Device faults and graph capture (include/kcc.h conventions).

  - The fault-path build (libkcc_faultdiag.so, csrc/Makefile `faultdiag`: every bounded
    device wait — the reduce's look-back, the exchange's flag wait — gives up at once, as a
    timed-out wait would): the synchronous entry points return KCC_EFAULT instead of
    wrong sums as success; the async finalizes (fused clamp finalize, clamp-in-fit finalize,
    fit_finalize, the exchange kernel) mark every spec KCC_SPEC_FAULT with total 0;
    kcc_clear_faults resets the fault words.
  - The release build: the fault words stay 0 and clearing them is harmless.
  - hipGraph capture: kcc_capacity_async (reduce + fit + clamp + fused finalize) and
    kcc_capacity_partial_async + kcc_exchange_finalize_async captured once and replayed
    with NEW inputs each time == the oracle for each input (no launch depends on host
    state a replay would freeze: the look-back records are left free by every launch,
    the exchange epoch is a device word).  ClusterCapacity.go:101-140, 290-293.
"""
import os

import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from kubernetesclustercapacity_amd._lib import KCC_EFAULT, KCC_SPEC_FAULT
from oracle import coracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAULTDIAG = os.path.join(ROOT, "kubernetesclustercapacity_amd", "libkcc_faultdiag.so")
NT = min(16, os.cpu_count() or 1)


def _cluster(n=20_000, s=300, seed=51, adv=False):
    # ~40 containers per node and one 512-container tile per wave range at this size: most
    # wave ranges end inside a node, so the reduce assembles those nodes by look-back
    c = synth.make_cluster(n, 20 * n, seed=seed, chunk=1024, adversarial=adv)
    sc, sm = synth.make_specs(s, seed=seed, adversarial=adv)
    return c, sc, sm


def _oracle(c, sc, sm):
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    return uc, um, t, e


def _dev_args(c, sc, sm, dev):
    import torch
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    n = c.n_nodes
    return [T(c.node_ptr), T(c.cpu_req), T(c.mem_req), T(c.alloc_cpu), T(c.alloc_mem),
            T(c.alloc_pods), T(c.pod_count), torch.empty(n, dtype=torch.int64, device=dev),
            torch.empty(n, dtype=torch.int64, device=dev), T(sc), T(sm)]


@pytest.fixture(scope="module")
def diag_engine():
    from conftest import init_torch_first
    init_torch_first()
    if not os.path.exists(FAULTDIAG):
        pytest.fail("libkcc_faultdiag.so missing: __graft_entry__.build() builds it")
    from kubernetesclustercapacity_amd import CapacityEngine
    eng = CapacityEngine(0, 1, lib_path=FAULTDIAG)
    assert "faultdiag" in eng._lib.kcc_build_info().decode()
    yield eng
    eng.close()


def test_release_build_fault_words_clear(engine):
    c, sc, sm = _cluster()
    _, _, t, e = _oracle(c, sc, sm)
    assert engine._lib.kcc_build_info().decode() == "release"
    got_t, got_e = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                                   c.alloc_pods, c.pod_count, sc, sm)
    np.testing.assert_array_equal(got_t, t)
    np.testing.assert_array_equal(got_e, e)
    assert engine.reduce_faults() == 0 and engine.p2p_faults() == 0
    engine.clear_faults()  # re-zeroes the look-back records: the next call is unaffected
    got_t, _ = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                               c.alloc_pods, c.pod_count, sc, sm)
    np.testing.assert_array_equal(got_t, t)


def test_sync_entry_points_return_efault(diag_engine):
    from kubernetesclustercapacity_amd import KccError
    c, sc, sm = _cluster()
    for call in (lambda: diag_engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req,
                                                                         c.mem_req),
                 lambda: diag_engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu,
                                              c.alloc_mem, c.alloc_pods, c.pod_count, sc, sm)):
        with pytest.raises(KccError) as ei:
            call()
        assert ei.value.code == KCC_EFAULT, ei.value
        assert "gave up" in str(ei.value)
        assert diag_engine.reduce_faults() > 0
        diag_engine.clear_faults()
        assert diag_engine.reduce_faults() == 0
    # the fault word is sticky: a fit without a reduce after a faulted reduce fails too
    with pytest.raises(KccError):
        diag_engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    with pytest.raises(KccError) as ei:
        diag_engine.total_possible_max_replicas(c.alloc_cpu, c.alloc_mem, c.alloc_pods,
                                                c.pod_count, uc, um, sc, sm)
    assert ei.value.code == KCC_EFAULT
    diag_engine.clear_faults()
    # ... and without any fault the same build's fit (no reduce, no wait) succeeds
    t, e = diag_engine.total_possible_max_replicas(c.alloc_cpu, c.alloc_mem, c.alloc_pods,
                                                   c.pod_count, uc, um, sc, sm)
    _, _, ot, oe = _oracle(c, sc, sm)
    np.testing.assert_array_equal(t, ot)
    np.testing.assert_array_equal(e, oe)


def test_keyed_entry_points_return_efault(diag_engine, engine):
    """The keyed one-sweep path (requests, count_by_key): the gather's part wait gives up at
    once in the fault-path build (several parts per bucket group at this key count), so the
    synchronous entry points return KCC_EFAULT; the bucketed path (calls with limits) has no
    wait and is exact once the faults are cleared.  The release build's next calls after
    kcc_clear_faults are exact (it re-zeroes the gather's arrival and ready counts)."""
    from kubernetesclustercapacity_amd import KccError
    rng = np.random.default_rng(5)
    nk, nc = 3_000, 200_000
    key = rng.integers(0, nk, nc).astype(np.int32)
    cpu = rng.integers(0, 1 << 20, nc).astype(np.uint64)
    mem = rng.integers(0, 1 << 40, nc).astype(np.int64)
    ok = np.argsort(key, kind="stable")
    ptr = np.searchsorted(key[ok], np.arange(nk + 1)).astype(np.int64)
    uc, um, _, _ = coracle.reduce_requests(ptr, cpu[ok], mem[ok])
    diag_engine.clear_faults()
    for call in (lambda: diag_engine.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem),
                 lambda: diag_engine.count_by_key(nk, key)):
        with pytest.raises(KccError) as ei:
            call()
        assert ei.value.code == KCC_EFAULT, ei.value
        assert "gave up" in str(ei.value)
        diag_engine.clear_faults()
    r = diag_engine.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem, cpu, mem)
    np.testing.assert_array_equal(r.cpu_requests, uc)
    np.testing.assert_array_equal(r.memory_requests, um)
    engine.clear_faults()
    for _ in range(2):
        r = engine.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem)
        np.testing.assert_array_equal(r.cpu_requests, uc)
        np.testing.assert_array_equal(r.memory_requests, um)
        np.testing.assert_array_equal(engine.count_by_key(nk, key), np.diff(ptr))


@pytest.mark.parametrize("mode", [0, 1])
def test_async_finalizes_mark_every_spec(diag_engine, mode):
    """kcc_capacity_async (mode 0: fused clamp finalize; 1: clamp in the fit + finalize)
    and capacity_partial_async + fit_finalize_async after a look-back give-up."""
    import torch
    dev = torch.device("cuda", 0)
    c, sc, sm = _cluster(s=700)
    a = _dev_args(c, sc, sm, dev)
    S = sc.size
    totals = torch.full((S,), 123, dtype=torch.int64, device=dev)
    err = torch.zeros(S, dtype=torch.int32, device=dev)
    partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
    diag_engine.set_clamp_in_fit(mode)
    try:
        for k in range(2):
            diag_engine.clear_faults()
            if k == 0:
                diag_engine.capacity_async(c.node_ptr, *a, totals, err)
            else:
                diag_engine.capacity_partial_async(c.node_ptr, *a, partial)
                diag_engine.fit_finalize_async(S, partial, totals, err)
            torch.cuda.synchronize()
            assert diag_engine.reduce_faults() > 0
            assert (err.cpu().numpy() == KCC_SPEC_FAULT).all(), f"call {k}"
            assert (totals.cpu().numpy() == 0).all(), f"call {k}"
    finally:
        diag_engine.set_clamp_in_fit(-1)
        diag_engine.clear_faults()


def test_exchange_give_up_marks_specs(diag_engine):
    """A one-rank mailbox (own memory, no IPC peer): the exchange kernel's flag wait gives
    up, counts FAULT_P2P and marks every spec."""
    import torch
    dev = torch.device("cuda", 0)
    c, sc, sm = _cluster(n=5_000, s=300)
    a = _dev_args(c, sc, sm, dev)
    S = sc.size
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1, lib_path=FAULTDIAG) as eng:
        h = eng.p2p_export(1, S)
        eng.p2p_open(0, [h])
        partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
        totals = torch.full((S,), 5, dtype=torch.int64, device=dev)
        err = torch.zeros(S, dtype=torch.int32, device=dev)
        eng.capacity_partial_async(c.node_ptr, *a, partial)
        eng.exchange_finalize_async(S, partial, totals, err)
        torch.cuda.synchronize()
        assert eng.p2p_faults() >= 1
        assert (err.cpu().numpy() == KCC_SPEC_FAULT).all()
        assert (totals.cpu().numpy() == 0).all()


def test_release_one_rank_exchange_equals_finalize(engine):
    """The release build's exchange with one rank (its own mailbox): == the oracle, several
    launches in a row (the device epoch advances; both parities)."""
    import torch
    dev = torch.device("cuda", 0)
    c, sc, sm = _cluster(n=5_000, s=300, adv=True)
    _, _, t, e = _oracle(c, sc, sm)
    a = _dev_args(c, sc, sm, dev)
    S = sc.size
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1) as eng:
        eng.p2p_open(0, [eng.p2p_export(1, S)])
        partial = torch.empty(2 * S, dtype=torch.int64, device=dev)
        totals = torch.empty(S, dtype=torch.int64, device=dev)
        err = torch.empty(S, dtype=torch.int32, device=dev)
        for k in range(3):
            totals.fill_(-1)
            eng.capacity_partial_async(c.node_ptr, *a, partial)
            eng.exchange_finalize_async(S, partial, totals, err)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(totals.cpu().numpy(), t, err_msg=f"launch {k}")
            np.testing.assert_array_equal(err.cpu().numpy(), e, err_msg=f"launch {k}")
        assert eng.p2p_faults() == 0


def _variants(n, s, seeds, adv):
    """Clusters of one shape (same node count, container count and spec count) with
    different CSR offsets, requests, allocatables and specs."""
    out = []
    base = synth.make_cluster(n, 20 * n, seed=seeds[0], chunk=1024, adversarial=adv)
    per = np.diff(base.node_ptr)
    for i, sd in enumerate(seeds):
        c = synth.make_cluster(n, 20 * n, seed=sd, chunk=1024, adversarial=adv)
        rng = np.random.default_rng(sd)
        cnt = rng.permutation(per) if i else per  # same total, another segmentation
        ptr = np.zeros(n + 1, np.int64)
        np.cumsum(cnt, out=ptr[1:])
        C = int(ptr[-1])
        cpu = rng.integers(0, 41, C).astype(np.uint64) * np.uint64(50)
        mem = rng.integers(0, 8192, C).astype(np.int64) << 20
        if adv:
            cpu[rng.random(C) < 0.01] = np.uint64(2**64 - 100)
        c.node_ptr, c.cpu_req, c.mem_req = ptr, cpu, mem
        c.cpu_lim, c.mem_lim = cpu * np.uint64(2), mem * 2
        sc, sm = synth.make_specs(s, seed=sd, adversarial=adv)
        out.append((c, sc, sm))
    return out


@pytest.mark.parametrize("mode", [0, 1])
def test_graph_replay_capacity_async(mode):
    """kcc_capacity_async captured into a hipGraph (torch.cuda.graph) after kcc_reserve,
    replayed over three different clusters and spec sets of one shape (copied into the
    captured buffers before each replay), twice each: per-node sums and totals == the
    oracle every time.  mode: 0 = the clamp correction (4 launches), 1 = the clamp in the
    fit."""
    import torch

    from kubernetesclustercapacity_amd import CapacityEngine
    from conftest import init_torch_first
    init_torch_first()
    dev = torch.device("cuda", 0)
    n, s = 30_000, 600
    vs = _variants(n, s, (61, 62, 63), adv=True)
    refs = [_oracle(*v) for v in vs]
    bufs = _dev_args(*vs[0], dev)
    totals = torch.empty(s, dtype=torch.int64, device=dev)
    err = torch.empty(s, dtype=torch.int32, device=dev)
    with CapacityEngine(0, 1) as eng:
        eng.set_clamp_in_fit(mode)
        eng.reserve(n, vs[0][0].n_containers, s)
        stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(stream):  # warm-up: every workspace allocated, first-use state set
            eng.capacity_async(None, *bufs, totals, err, stream=stream)
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            eng.capacity_async(None, *bufs, totals, err, stream=stream)
        new = [_dev_args(*v, dev) for v in vs]
        for rep in range(2):
            for k, (v, ref) in enumerate(zip(vs, refs)):
                with torch.cuda.stream(stream):
                    for i in (0, 1, 2, 3, 4, 5, 6, 9, 10):  # all but the used_* outputs
                        bufs[i].copy_(new[k][i])
                    bufs[7].fill_(-1)
                    bufs[8].fill_(-1)
                    totals.fill_(-9)
                    g.replay()
                stream.synchronize()
                uc, um, t, e = ref
                msg = f"replay {rep} cluster {k}"
                np.testing.assert_array_equal(bufs[7].cpu().numpy().view(np.uint64), uc, err_msg=msg)
                np.testing.assert_array_equal(bufs[8].cpu().numpy(), um, err_msg=msg)
                np.testing.assert_array_equal(totals.cpu().numpy(), t, err_msg=msg)
                np.testing.assert_array_equal(err.cpu().numpy(), e, err_msg=msg)
        assert eng.reduce_faults() == 0
        del g
