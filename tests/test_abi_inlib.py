"""GPU: the in-library multi-device path (kcc_create(first, n_gpus > 1) -> ncclCommInitAll,
ncclAllReduce of the devices' partials inside kcc_capacity / kcc_fit) verifies its first
all-reduce per context against a host-side sum of the devices' partials (CC:138 summed over
devices) and returns KCC_ERCCL on a mismatch, never wrong totals.

The box has one GPU, so the diagnostic build libkcc_inlibcomm.so (csrc/Makefile `diag`:
KCC_DIAG_INLIB_COMM) sends a one-device context through the same RCCL all-reduce and check;
KCC_DRILL_CORRUPT_ALLREDUCE=1 corrupts the all-reduced partial after the collective.
"""
import os

import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from oracle import coracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INLIB = os.path.join(ROOT, "kubernetesclustercapacity_amd", "libkcc_inlibcomm.so")


def _engine():
    from conftest import init_torch_first
    init_torch_first()
    if not os.path.exists(INLIB):
        pytest.fail("libkcc_inlibcomm.so missing: __graft_entry__.build() builds it")
    from kubernetesclustercapacity_amd import CapacityEngine
    eng = CapacityEngine(0, 1, lib_path=INLIB)
    assert "inlibcomm" in eng._lib.kcc_build_info().decode()
    return eng


def _cluster():
    c = synth.make_cluster(30_011, 500_000, seed=31, adversarial=True, chunk=1024)
    sc, sm = synth.make_specs(700, seed=31, adversarial=True)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm)
    return c, sc, sm, t, e


def test_inlib_allreduce_verified(monkeypatch):
    monkeypatch.delenv("KCC_DRILL_CORRUPT_ALLREDUCE", raising=False)
    c, sc, sm, t, e = _cluster()
    eng = _engine()
    try:
        for shards in (0, 3):  # one shard per device; three folded on the device first
            eng.set_node_shards(shards)
            got_t, got_e = eng.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu,
                                        c.alloc_mem, c.alloc_pods, c.pod_count, sc, sm)
            np.testing.assert_array_equal(got_t, t)
            np.testing.assert_array_equal(got_e, e)
    finally:
        eng.close()


def test_inlib_allreduce_mismatch_returns_ercc(monkeypatch):
    from kubernetesclustercapacity_amd import KccError
    from kubernetesclustercapacity_amd._lib import KCC_ERCCL
    c, sc, sm, t, e = _cluster()
    eng = _engine()
    try:
        monkeypatch.setenv("KCC_DRILL_CORRUPT_ALLREDUCE", "1")
        with pytest.raises(KccError) as ei:
            eng.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                         c.alloc_pods, c.pod_count, sc, sm)
        assert ei.value.code == KCC_ERCCL
        assert "verification failed" in str(ei.value)
        # the check belongs to the context's first all-reduce: a clean retry verifies and passes
        monkeypatch.delenv("KCC_DRILL_CORRUPT_ALLREDUCE")
        got_t, got_e = eng.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                                    c.alloc_pods, c.pod_count, sc, sm)
        np.testing.assert_array_equal(got_t, t)
        np.testing.assert_array_equal(got_e, e)
    finally:
        eng.close()


def test_inlib_allreduce_verify_every_call(monkeypatch):
    """After a verified first all-reduce, a later corrupted one goes unchecked by default
    and is caught with kcc_set_allreduce_verify(ctx, 1)."""
    from kubernetesclustercapacity_amd import KccError
    from kubernetesclustercapacity_amd._lib import KCC_ERCCL
    monkeypatch.delenv("KCC_DRILL_CORRUPT_ALLREDUCE", raising=False)
    c, sc, sm, t, e = _cluster()
    eng = _engine()
    args = (c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem, c.alloc_pods,
            c.pod_count, sc, sm)
    try:
        got_t, _ = eng.capacity(*args)  # the first call verifies
        np.testing.assert_array_equal(got_t, t)
        monkeypatch.setenv("KCC_DRILL_CORRUPT_ALLREDUCE", "1")
        got_t, _ = eng.capacity(*args)  # unchecked (the documented default): wrong word 0
        assert not np.array_equal(got_t, t)
        assert eng._lib.kcc_set_allreduce_verify(eng._h, 1) == 0
        with pytest.raises(KccError) as ei:
            eng.capacity(*args)
        assert ei.value.code == KCC_ERCCL
    finally:
        eng.close()
