"""Property-based parity: random clusters and spec sets, drawn from value mixtures that hit
every branch of the path at once — empty and giant nodes, wrapped (negative) requests,
free CPU around the class-A bound 2^23, free memory around 2^50 and negative, memory
requests below 2^18 (class B) and above 2^50, zero requests (divide-by-zero flags),
alloc_pods <= 0 and |clamp| > 2^20 (the exact path) — through the C-ABI against the C
oracle (CC:101-140, CC:276-294), bit for bit, in every fit layout: the clamp correction,
the clamp in the fit, and the dense stream.  The keyed reduce gets the
same treatment: random list-order keys (off-row keys included), key counts across the
one-sweep / bucketed / atomic paths.  hypothesis draws the shapes and seeds (derandomized:
the same examples every run); numpy draws the values from the seed.
"""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import coracle

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)
U64 = np.uint64


def _mix(rng, n, parts, dtype):
    """n values, each from one of `parts` ((weight, draw(k)) pairs) chosen per value."""
    w = np.array([p[0] for p in parts], float)
    pick = rng.choice(len(parts), n, p=w / w.sum())
    out = np.zeros(n, dtype)
    for j, (_, draw) in enumerate(parts):
        k = int((pick == j).sum())
        if k:
            out[pick == j] = draw(k)
    return out


def _near(rng, v, k, dtype, span=4):
    return (np.array(v, dtype) + rng.integers(-span, span + 1, k).astype(dtype)).astype(dtype)


def make_case(seed, n, s):
    rng = np.random.default_rng(seed)
    i64, u64 = np.int64, np.uint64
    full_u = lambda k: rng.integers(0, 2**64, k, dtype=np.uint64)  # noqa: E731
    full_i = lambda k: rng.integers(-2**63, 2**63, k, dtype=np.int64)  # noqa: E731
    per = _mix(rng, n, [(40, lambda k: rng.integers(0, 9, k)), (30, lambda k: rng.integers(0, 81, k)),
                        (20, lambda k: np.zeros(k, i64)), (10, lambda k: rng.integers(500, 3000, k))],
               i64)
    ptr = np.zeros(n + 1, i64)
    np.cumsum(per, out=ptr[1:])
    c = int(ptr[-1])
    cpu = _mix(rng, c, [(70, lambda k: rng.integers(0, 4000, k).astype(u64)),
                        (10, lambda k: np.zeros(k, u64)), (10, full_u),
                        (10, lambda k: _near(rng, 2**64 - 100, k, u64))], u64)
    mem = _mix(rng, c, [(70, lambda k: rng.integers(0, 2**34, k)), (10, lambda k: -rng.integers(1, 2**30, k)),
                        (10, full_i), (10, lambda k: np.zeros(k, i64))], i64)
    acpu = _mix(rng, n, [(70, lambda k: rng.integers(0, 2**17, k).astype(u64)),
                         (10, lambda k: np.zeros(k, u64)), (10, full_u),
                         (10, lambda k: _near(rng, 2**23, k, u64))], u64)
    amem = _mix(rng, n, [(70, lambda k: rng.integers(0, 2**40, k)), (10, lambda k: -rng.integers(1, 2**40, k)),
                         (10, full_i), (10, lambda k: _near(rng, 2**50, k, i64))], i64)
    apods = _mix(rng, n, [(70, lambda k: rng.integers(0, 256, k)), (10, lambda k: -rng.integers(1, 50, k)),
                          (10, lambda k: np.zeros(k, i64)), (10, lambda k: _near(rng, 2**20, k, i64, 300))],
                 i64)
    pcount = _mix(rng, n, [(70, lambda k: rng.integers(0, 300, k)), (20, lambda k: np.zeros(k, i64)),
                           (10, lambda k: rng.integers(2**20, 2**21, k))], i64)
    sc = _mix(rng, s, [(60, lambda k: rng.integers(1, 8001, k).astype(u64)), (10, lambda k: np.zeros(k, u64)),
                       (10, lambda k: rng.integers(2**23, 2**40, k).astype(u64)),
                       (10, lambda k: _near(rng, 2**51, k, u64, 2)), (10, full_u)], u64)
    sm = _mix(rng, s, [(60, lambda k: rng.integers(2**20, 2**35, k)), (8, lambda k: np.zeros(k, i64)),
                       (8, lambda k: -rng.integers(1, 2**40, k)), (8, lambda k: rng.integers(1, 2**18, k)),
                       (8, lambda k: _near(rng, 2**50, k, i64, 2)), (8, full_i)], i64)
    return ptr, cpu, mem, acpu, amem, apods, pcount, sc, sm


# (hypothesis favours small integers: the sizes around the kernels' 64-lane, 512-container and
# 1024-row granules are drawn as often as free ones)
SIZES_N = st.one_of(st.sampled_from([0, 1, 2, 63, 64, 65, 511, 512, 1023, 1024, 1025, 2048, 2500]),
                    st.integers(0, 2500))
SIZES_S = st.one_of(st.sampled_from([1, 63, 64, 65, 127, 128, 255, 256, 257, 700]),
                    st.integers(1, 700))


@settings(max_examples=200, derandomize=True, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), n=SIZES_N, s=SIZES_S,
       layout=st.sampled_from(["correction", "in_fit", "dense"]),
       shards=st.sampled_from([0, 0, 2, 3]))
def test_capacity_fuzz(engine, seed, n, s, layout, shards):
    """shards > 0: the host-array calls cut the nodes into that many shards on the one
    device (partials summed on the device, kcc_set_node_shards)."""
    ptr, cpu, mem, acpu, amem, apods, pcount, sc, sm = make_case(seed, n, s)
    uc, um, _, _ = coracle.reduce_requests(ptr, cpu, mem)
    ot, oe = coracle.fit(acpu, amem, apods, pcount, uc, um, sc, sm, NT)
    engine.set_clamp_in_fit({"correction": 0, "in_fit": 1, "dense": -1}[layout])
    engine.set_fit_dense(layout == "dense")
    engine.set_node_shards(shards)
    try:
        r = engine.get_pod_cpu_memory_requests_limits(ptr, cpu, mem)
        np.testing.assert_array_equal(r.cpu_requests, uc)
        np.testing.assert_array_equal(r.memory_requests, um)
        t, e = engine.capacity(ptr, cpu, mem, acpu, amem, apods, pcount, sc, sm)
        np.testing.assert_array_equal(e, oe)
        np.testing.assert_array_equal(t, ot)
        t2, e2 = engine.total_possible_max_replicas(acpu, amem, apods, pcount, uc, um, sc, sm)
        np.testing.assert_array_equal(e2, oe)
        np.testing.assert_array_equal(t2, ot)
    finally:
        engine.set_clamp_in_fit(-1)
        engine.set_fit_dense(False)
        engine.set_node_shards(0)


@settings(max_examples=60, derandomize=True, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), nk=st.sampled_from([1, 7, 64, 1000, 8191, 8192, 40_000, 300_000]),
       nc=st.one_of(st.sampled_from([0, 1, 511, 512, 4096, 100_000, 300_000]),
                     st.integers(0, 300_000)), off=st.sampled_from([0.0, 0.02, 0.5]), lim=st.booleans())
def test_keyed_fuzz(engine, seed, nk, nc, off, lim):
    rng = np.random.default_rng(seed)
    key = rng.integers(0, nk, nc).astype(np.int32)
    bad = rng.random(nc) < off
    key[bad] = rng.choice(np.array([-1, nk, nk + 5, -(2**31), 2**31 - 1], np.int32), int(bad.sum()))
    cpu = _mix(rng, nc, [(80, lambda k: rng.integers(0, 4000, k).astype(U64)),
                         (20, lambda k: rng.integers(0, 2**64, k, dtype=np.uint64))], U64)
    mem = _mix(rng, nc, [(80, lambda k: rng.integers(0, 2**34, k)),
                         (20, lambda k: rng.integers(-2**63, 2**63, k, dtype=np.int64))], np.int64)
    ok = (key >= 0) & (key < nk)
    srt = np.argsort(key[ok], kind="stable")
    ptr = np.searchsorted(key[ok][srt], np.arange(nk + 1)).astype(np.int64)
    sel = lambda a: a[ok][srt]  # noqa: E731
    if lim:
        cl, ml = cpu ^ U64(0x5555), mem // 3
        o = coracle.reduce_requests(ptr, sel(cpu), sel(mem), sel(cl), sel(ml))
        r = engine.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem, cl, ml)
        np.testing.assert_array_equal(r.cpu_limits, o[2])
        np.testing.assert_array_equal(r.memory_limits, o[3])
    else:
        o = coracle.reduce_requests(ptr, sel(cpu), sel(mem))
        r = engine.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem)
    np.testing.assert_array_equal(r.cpu_requests, o[0])
    np.testing.assert_array_equal(r.memory_requests, o[1])
    np.testing.assert_array_equal(engine.count_by_key(nk, key), np.diff(ptr))
