"""GPU parity: libkcc.so (gfx950 kernels) vs the CPU oracles, bit for bit.

Every call goes through the C-ABI.  Integer work: the bar is exact equality
(uint64/int64 two's-complement), no tolerance.
  - golden fixtures (tests/golden/*.npz, from the Python big-int restatement);
  - seeded clusters (normal / adversarial / skewed / sparse) vs the C oracle;
  - CSR edge cases of the segmented reduce (empty nodes, runs crossing the
    4096-container wave ranges, giant nodes, odd sizes);
  - BASELINE config C4 at full size (1M nodes, ~40M containers, 4096 specs)
    through size-independent properties: exact numpy segment sums, a spec sample
    vs the C oracle over all nodes, node-shard linearity, run-to-run identity.
"""
import glob
import os

import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from oracle import coracle

pytestmark = pytest.mark.gpu
GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if os.path.basename(p) != "parse.npz")  # parse.npz: tests/test_parse.py
NT = min(16, os.cpu_count() or 1)


def seg_sums(node_ptr, vals):
    """Exact wrapping per-node sums with numpy (uint64 arithmetic wraps)."""
    v = np.asarray(vals).view(np.uint64)
    cs = np.zeros(v.size + 1, np.uint64)
    np.cumsum(v, out=cs[1:])
    return cs[node_ptr[1:]] - cs[node_ptr[:-1]]


# ---- golden fixtures --------------------------------------------------------------
@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_reduce_golden(engine, path):
    d = np.load(path)
    r = engine.get_pod_cpu_memory_requests_limits(d["node_ptr"], d["cpu_req"], d["mem_req"],
                                                  d["cpu_lim"], d["mem_lim"])
    np.testing.assert_array_equal(r.cpu_requests, d["exp_used_cpu"])
    np.testing.assert_array_equal(r.memory_requests, d["exp_used_mem"])
    np.testing.assert_array_equal(r.cpu_limits, d["exp_lim_cpu"])
    np.testing.assert_array_equal(r.memory_limits, d["exp_lim_mem"])
    r2 = engine.get_pod_cpu_memory_requests_limits(d["node_ptr"], d["cpu_req"], d["mem_req"])
    np.testing.assert_array_equal(r2.cpu_requests, d["exp_used_cpu"])
    assert r2.cpu_limits is None


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_fit_golden(engine, path):
    d = np.load(path)
    t, e = engine.total_possible_max_replicas(d["alloc_cpu"], d["alloc_mem"], d["alloc_pods"],
                                              d["pod_count"], d["exp_used_cpu"],
                                              d["exp_used_mem"], d["spec_cpu"], d["spec_mem"])
    np.testing.assert_array_equal(e, d["exp_err"])
    np.testing.assert_array_equal(t, d["exp_totals"])


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p))
def test_capacity_golden(engine, path):
    d = np.load(path)
    t, e = engine.capacity(d["node_ptr"], d["cpu_req"], d["mem_req"], d["alloc_cpu"],
                           d["alloc_mem"], d["alloc_pods"], d["pod_count"], d["spec_cpu"],
                           d["spec_mem"])
    np.testing.assert_array_equal(e, d["exp_err"])
    np.testing.assert_array_equal(t, d["exp_totals"])


# ---- seeded clusters vs the C oracle --------------------------------------------------
CASES = [
    dict(n=20_000, pods=400_000, s=300, seed=1),
    dict(n=20_000, pods=400_000, s=300, seed=2, adversarial=True),
    dict(n=8_000, pods=200_000, s=129, seed=3, skew=True),
    dict(n=30_000, pods=3_000, s=65, seed=4, unhealthy=0.3),
    dict(n=5_000, pods=100_000, s=1, seed=5),
    dict(n=1, pods=50, s=7, seed=6),
]


@pytest.mark.parametrize("cfg", CASES, ids=lambda c: f"n{c['n']}_s{c['s']}_seed{c['seed']}")
def test_capacity_vs_oracle(engine, cfg):
    c = synth.make_cluster(cfg["n"], cfg["pods"], seed=cfg["seed"], skew=cfg.get("skew", False),
                           adversarial=cfg.get("adversarial", False),
                           unhealthy=cfg.get("unhealthy", 0.01), chunk=1024)
    sc, sm = synth.make_specs(cfg["s"], seed=cfg["seed"], adversarial=cfg.get("adversarial", False))
    r = engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim,
                                                  c.mem_lim)
    uc, um, lc, lm = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim,
                                             c.mem_lim)
    np.testing.assert_array_equal(r.cpu_requests, uc)
    np.testing.assert_array_equal(r.memory_requests, um)
    np.testing.assert_array_equal(r.cpu_limits, lc)
    np.testing.assert_array_equal(r.memory_limits, lm)
    t, e = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                           c.alloc_pods, c.pod_count, sc, sm)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize("s,adv", [(64, False), (4095, False), (4096, False), (4097, False),
                                   (6000, False), (4100, True), (6000, True), (8193, False),
                                   (16384, False), (9000, True)])
def test_spec_count_clamp_paths(engine, s, adv):
    """Spec counts around the LDS search tables (<= 4096 specs: LDS tables in node_prep;
    more: global searches) and the rank kernel's staging (<= 8192: candidates staged in
    LDS; more, e.g. C5's 16384: straight from memory), with heavy ties."""
    c = synth.make_cluster(2_500, 50_000, seed=11, chunk=1024)
    sc, sm = synth.make_specs(s, seed=11, adversarial=adv)
    sc[::3] = sc[0]
    sm[::5] = sm[1]
    sc[1::7] = sc[2]
    t, e = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                           c.alloc_pods, c.pod_count, sc, sm)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize("s", [1025, 3000, 9000])
def test_spec_rank_top_requests(engine, s):
    """The spec ranks' slices (1024 candidates each, sorted and searched): requests at the
    top of the normal range (2^51 - 1, whose 'count v_j <= v_i' threshold does not fit the
    64-bit key) in several slices, ties across slices, non-normal specs between them."""
    rng = np.random.default_rng(31 + s)
    c = synth.make_cluster(2_000, 40_000, seed=13, chunk=1024)
    sc, sm = synth.make_specs(s, seed=13)
    top = (1 << 51) - 1
    sc[[0, 1024 % s, s - 1, s // 2]] = top
    sm[[1, 1025 % s, s - 2, s // 3]] = top
    sc[::11] = sc[5]
    sm[::13] = sm[6]
    sc[rng.integers(0, s, s // 50)] = 0                   # exact path: div-by-zero flags
    sm[rng.integers(0, s, s // 50)] = (1 << 51) + 3       # exact path
    t, e = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                           c.alloc_pods, c.pod_count, sc, sm)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


def test_fit_random_raw_rows(engine):
    """Arbitrary 64-bit rows (not derived from a cluster) against the oracle."""
    rng = np.random.default_rng(99)
    n, s = 4_000, 200
    pick = lambda a, b: rng.choice(np.array(a + b, dtype=object), n)  # noqa: E731
    alloc_cpu = rng.integers(0, 2**64, n, dtype=np.uint64)
    alloc_cpu[: n // 2] = rng.integers(0, 200_000, n // 2)
    used_cpu = rng.integers(0, 2**64, n, dtype=np.uint64)
    used_cpu[: n // 2] = rng.integers(0, 100_000, n // 2)
    alloc_mem = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    alloc_mem[: n // 2] = rng.integers(0, 2**40, n // 2)
    used_mem = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    used_mem[: n // 2] = rng.integers(0, 2**39, n // 2)
    alloc_pods = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    alloc_pods[: 3 * n // 4] = rng.integers(-3, 300, 3 * n // 4)
    pod_count = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    pod_count[: 3 * n // 4] = rng.integers(0, 400, 3 * n // 4)
    del pick
    sc = rng.integers(1, 10_000, s).astype(np.uint64)
    sm = rng.integers(1, 2**36, s, dtype=np.int64)
    sc[::17] = rng.integers(0, 2**64, len(sc[::17]), dtype=np.uint64)
    sm[::13] = rng.integers(-2**63, 2**63, len(sm[::13]), dtype=np.int64)
    sm[5], sc[7], sm[9] = -1, 0, 0
    t, e = engine.total_possible_max_replicas(alloc_cpu, alloc_mem, alloc_pods, pod_count,
                                              used_cpu, used_mem, sc, sm)
    ot, oe = coracle.fit(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, sc, sm,
                         NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


def test_fast_path_boundaries(engine):
    """Quotients landing exactly on / next to integers and on the pod clamp."""
    rng = np.random.default_rng(5)
    n = 6_000
    sc = np.array([1, 2, 3, 7, 50, 100, 200, 250, 333, 1000, 4096, 8000, 8388607, 4194303,
                   1048573, 2**21], np.uint64)
    sm = np.array([1, 3, 1 << 20, 104_857_600, 262_144_000, 1 << 30, 3 << 30, 2**37 - 1,
                   999_999_937, 5, 64 << 20, 1_000_000, 7, 2**51 - 1, 2**44 + 7, 2**47 - 5],
                  np.int64)
    k = rng.integers(0, 300, n)
    j = rng.integers(0, len(sc), n)
    alloc_cpu = (k * sc[j].astype(np.int64) + rng.integers(-1, 2, n)).clip(0).astype(np.uint64)
    alloc_mem = (k * sm[j] + rng.integers(-1, 2, n)).clip(0)
    alloc_pods = k + rng.integers(-1, 2, n)
    pod_count = rng.integers(0, 300, n)
    used_cpu = np.zeros(n, np.uint64)
    used_mem = np.zeros(n, np.int64)
    t, e = engine.total_possible_max_replicas(alloc_cpu, alloc_mem, alloc_pods, pod_count,
                                              used_cpu, used_mem, sc, sm)
    ot, oe = coracle.fit(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, sc, sm)
    np.testing.assert_array_equal(t, ot)
    np.testing.assert_array_equal(e, oe)


def _rows_near_bounds(rng, n, sc, sm):
    """Rows whose quotients sit on / next to integers for the given specs, free CPU on
    both sides of 2^23 (class-A node bound) and free memory up to 2^50."""
    k = rng.integers(0, 300, n)
    j = rng.integers(0, len(sc), n)
    fc = (k * sc[j].astype(np.int64) + rng.integers(-1, 2, n)).clip(0)
    fc[: n // 8] = (1 << 23) + rng.integers(-3, 3, n // 8)           # around the f32 bound
    fm = (k * sm[j] + rng.integers(-1, 2, n)).clip(0)
    fm[n // 8: n // 4] = (1 << 50) - rng.integers(1, 1 << 20, n // 8)  # top of the fm range
    alloc_pods = k + rng.integers(-1, 2, n)
    alloc_pods[-50:] = rng.integers(-3, 1, 50)                        # P <= 0: always clamped
    pod_count = rng.integers(0, 300, n)
    return (fc.astype(np.uint64), fm, alloc_pods, pod_count, np.zeros(n, np.uint64),
            np.zeros(n, np.int64))


def test_class_a_wave_boundaries(engine):
    """Whole class-A waves (memory requests >= 2^18): quotients on/next to integers,
    free CPU around 2^23, free memory near 2^50, P <= 0, memory requests at 2^18."""
    rng = np.random.default_rng(23)
    sc = np.concatenate([[1, 2, 3, 7, 100, 250, 8000, (1 << 23) - 1, 1 << 23, 2**51 - 1],
                         rng.integers(1, 9000, 118)]).astype(np.uint64)
    sm = np.concatenate([[1 << 18, (1 << 18) + 1, 104_857_600, 2**51 - 1, 1 << 30, 3 << 30,
                          999_999_937, 2**37 - 1, (1 << 18) + 3, 1 << 32],
                         rng.integers(1 << 18, 1 << 36, 118)]).astype(np.int64)
    args = _rows_near_bounds(rng, 8_000, sc, sm)
    t, e = engine.total_possible_max_replicas(*args, sc, sm)
    ot, oe = coracle.fit(*args, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize("mode", [0, 1])
def test_fit_fast_path_bounds_near_2_32_and_2_50(engine, mode):
    """The class-A fast path at its bounds, against the oracle: free memory just below 2^50
    (the f64 quotient's exactness bound) with P = 1..3, free memory exactly on
    a spec's request times P (fm = m x P and m x P - 1, the quotient on / next to an integer
    at the pod clamp), and class-A waves whose largest memory request is 3 x 2^30,
    2^32 - 2, 2^32 - 1, 2^32 or 2^40 (the 32-bit quotient's low dword); both
    clamp modes."""
    rng = np.random.default_rng(77)
    tops = [3 << 30, (1 << 32) - 2, (1 << 32) - 1, 1 << 32, 1 << 40]
    waves, lo = [], 1 << 18  # wave w (memory order): 63 requests in (top[w-1], top[w]] + top[w]
    for top in tops:
        waves.append(np.append(rng.integers(lo, top + 1, 63), top))
        lo = top + 1
    sm = rng.permutation(np.concatenate(waves)).astype(np.int64)
    sc = rng.integers(1, 4000, sm.size).astype(np.uint64)
    n = 16_000
    P = rng.integers(1, 4, n)
    fm = (1 << 50) - rng.integers(1, 1 << 30, n)                  # V saturates
    on = np.arange(n) % 4 == 1
    mm = np.asarray(tops, np.int64)[rng.integers(0, len(tops), n)]
    fm[on] = mm[on] * P[on] - (np.arange(n)[on] % 8 == 1)          # V = m or m - 1 (rounded)
    fm[np.arange(n) % 4 == 2] = rng.integers(1 << 20, 1 << 34, (np.arange(n) % 4 == 2).sum())
    fc = rng.integers(1, 1 << 22, n)
    args = (fc.astype(np.uint64), fm.astype(np.int64), P.astype(np.int64),
            rng.integers(0, 3, n).astype(np.int64), np.zeros(n, np.uint64), np.zeros(n, np.int64))
    engine.set_clamp_in_fit(mode)
    try:
        t, e = engine.total_possible_max_replicas(*args, sc, sm)
    finally:
        engine.set_clamp_in_fit(-1)
    ot, oe = coracle.fit(*args, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


def test_mixed_class_waves(engine):
    """64 class-A, 64 class-B (memory < 2^18) and 64 exact-path specs, shuffled: the
    partition regroups them and every class matches the oracle."""
    rng = np.random.default_rng(29)
    sc = rng.integers(1, 9000, 192).astype(np.uint64)
    sm = np.concatenate([rng.integers(1 << 18, 1 << 36, 64), rng.integers(1, 1 << 18, 64),
                         rng.integers(1, 1 << 36, 64)]).astype(np.int64)
    sm[128:160] = 0                                      # exact path: div-by-zero flags
    sc[160:] = (1 << 51) + rng.integers(0, 1 << 40, 32).astype(np.uint64)  # exact path
    perm = rng.permutation(192)
    sc, sm = sc[perm], sm[perm]
    args = _rows_near_bounds(rng, 5_000, sc, sm)
    t, e = engine.total_possible_max_replicas(*args, sc, sm)
    ot, oe = coracle.fit(*args, sc, sm, NT)
    np.testing.assert_array_equal(e, oe)
    np.testing.assert_array_equal(t, ot)


# ---- CSR edge cases of the segmented reduce ----------------------------------------
def _reduce_check(engine, sizes, seed=0):
    sizes = np.asarray(sizes, np.int64)
    ptr = np.zeros(sizes.size + 1, np.int64)
    np.cumsum(sizes, out=ptr[1:])
    rng = np.random.default_rng(seed)
    c = int(ptr[-1])
    cpu = rng.integers(0, 2**64, c, dtype=np.uint64)
    mem = rng.integers(-2**63, 2**63, c, dtype=np.int64)
    r = engine.get_pod_cpu_memory_requests_limits(ptr, cpu, mem, cpu ^ np.uint64(7), mem // 3)
    np.testing.assert_array_equal(r.cpu_requests, seg_sums(ptr, cpu))
    np.testing.assert_array_equal(r.memory_requests.view(np.uint64), seg_sums(ptr, mem))
    np.testing.assert_array_equal(r.cpu_limits, seg_sums(ptr, cpu ^ np.uint64(7)))
    np.testing.assert_array_equal(r.memory_limits.view(np.uint64), seg_sums(ptr, mem // 3))
    r2 = engine.get_pod_cpu_memory_requests_limits(ptr, cpu, mem)  # the 2-array kernel
    np.testing.assert_array_equal(r2.cpu_requests, r.cpu_requests)
    np.testing.assert_array_equal(r2.memory_requests, r.memory_requests)


@pytest.mark.parametrize("name,sizes", [
    ("all_empty", [0] * 1000),
    ("one_container", [1]),
    ("one_giant_node", [300_001]),
    ("giant_in_middle", [3, 250_000, 5]),
    ("exact_wave_ranges", [4096, 4096, 8192, 1, 4095]),
    ("tile_multiples", [128] * 200 + [64] * 100 + [2] * 50),
    ("empty_runs_longer_than_64", [3] + [0] * 500 + [7] + [0] * 64 + [1] + [0] * 63 + [2]),
    ("singletons", [1] * 20_001),
    ("odd_total", [1, 0, 2, 0, 0, 3] * 1000 + [1]),
    ("trailing_empty", [5, 9] + [0] * 300),
    ("leading_empty", [0] * 300 + [5, 9]),
    ("leading_empty_then_long", [0, 0, 0, 1763, 5, 0, 700]),  # wave 0: empties end at 0
])
def test_reduce_csr_edges(engine, name, sizes):
    _reduce_check(engine, sizes, seed=hash(name) & 0xFFFF)


def test_reduce_random_shapes(engine):
    rng = np.random.default_rng(17)
    for _ in range(8):
        n = int(rng.integers(1, 20_000))
        kind = rng.integers(0, 3)
        if kind == 0:
            sizes = rng.poisson(rng.uniform(0, 60), n)
        elif kind == 1:
            sizes = np.minimum(rng.zipf(1.3, n) - 1, 20_000)
        else:
            sizes = rng.integers(0, 2, n) * rng.integers(0, 9000, n)
        _reduce_check(engine, sizes, seed=int(rng.integers(1 << 30)))


def test_empty_inputs(engine):
    r = engine.get_pod_cpu_memory_requests_limits(np.zeros(1, np.int64), [], [])
    assert r.cpu_requests.size == 0
    t, e = engine.total_possible_max_replicas([], [], [], [], [], [], [100], [1 << 20])
    assert list(t) == [0] and list(e) == [0]
    t, e = engine.total_possible_max_replicas([4000], [1 << 30], [110], [3], [0], [0], [], [])
    assert t.size == 0


def test_invalid_csr_rejected(engine):
    from kubernetesclustercapacity_amd import KccError
    with pytest.raises(KccError):
        engine.get_pod_cpu_memory_requests_limits(np.array([0, 3, 2], np.int64), [1, 2, 3],
                                                  [1, 2, 3])
    with pytest.raises(KccError):
        engine.get_pod_cpu_memory_requests_limits(np.array([1, 3], np.int64), [1, 2, 3],
                                                  [1, 2, 3])


# ---- device API on a torch stream == host API ----------------------------------------------
def test_device_api_matches_host(engine):
    import torch
    c = synth.make_cluster(50_000, 1_000_000, seed=21, chunk=4096)
    sc, sm = synth.make_specs(700, seed=21, adversarial=True)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    n, s = c.n_nodes, sc.size
    ptr, cpu, mem = T(c.node_ptr), T(c.cpu_req), T(c.mem_req)
    used_cpu = torch.empty(n, dtype=torch.int64, device=dev)
    used_mem = torch.empty(n, dtype=torch.int64, device=dev)
    partial = torch.empty(2 * s, dtype=torch.int64, device=dev)
    totals = torch.empty(s, dtype=torch.int64, device=dev)
    err = torch.empty(s, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        engine.reduce_requests_async(ptr, cpu, mem, used_cpu, used_mem, stream=stream)
        engine.fit_prepare_async(T(c.alloc_cpu), T(c.alloc_mem), T(c.alloc_pods),
                                 T(c.pod_count), used_cpu, used_mem, T(sc), T(sm), partial,
                                 stream=stream)
        engine.fit_run_async(n, s, partial, stream=stream)
        engine.fit_finalize_async(s, partial, totals, err, stream=stream)
    stream.synchronize()
    ht, he = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                             c.alloc_pods, c.pod_count, sc, sm)
    np.testing.assert_array_equal(totals.cpu().numpy(), ht)
    np.testing.assert_array_equal(err.cpu().numpy(), he)
    slow, pairs = engine.fit_slow_pairs()
    assert pairs == n * s and 0 < slow < pairs


@pytest.mark.parametrize("n,s,adv", [(20_000, 700, True), (9_000, 4097, False),
                                     (6_000, 300, True), (0, 50, False)])
def test_capacity_async_fused_finalize(engine, n, s, adv):
    """kcc_capacity_async (the clamp correction's last workgroup finalizes) == the oracle,
    three calls in a row (its arrival counter returns to zero), incl. > 4096 specs (C's row
    suffixes), exact-path specs (adversarial) and no nodes (a finalize launch instead)."""
    import torch
    pods = 20 * n
    c = synth.make_cluster(n, pods, seed=41, chunk=1024, adversarial=adv)
    sc, sm = synth.make_specs(s, seed=41, adversarial=adv)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    used_cpu = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    used_mem = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    totals = torch.empty(s, dtype=torch.int64, device=dev)
    err = torch.empty(s, dtype=torch.int32, device=dev)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    stream = torch.cuda.Stream(dev)
    for _ in range(3):
        totals.fill_(-7)
        with torch.cuda.stream(stream):
            engine.capacity_async(c.node_ptr, T(c.node_ptr), T(c.cpu_req), T(c.mem_req),
                                  T(c.alloc_cpu), T(c.alloc_mem), T(c.alloc_pods), T(c.pod_count),
                                  used_cpu, used_mem, T(sc), T(sm), totals, err, stream=stream)
        stream.synchronize()
        np.testing.assert_array_equal(totals.cpu().numpy(), ot)
        np.testing.assert_array_equal(err.cpu().numpy(), oe)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n,s,adv,zipf", [(20_000, 700, True, False), (30_011, 4096, False, False),
                                          (12_345, 1000, False, True), (5_000, 64, True, False)])
def test_clamp_in_fit_modes(engine, mode, n, s, adv, zipf):
    """The pod-slot clamp (CC:134-135) applied by the clamp correction launch (mode 0) or
    inside the fit (mode 1: node_prep's clamp values, x >= P ? clamp : x in the fit's
    loops, the always-clamped rows' sum subtracted once per spec): both == the oracle, two
    calls in a row, through kcc_capacity_async and kcc_capacity_partial_async + finalize."""
    import torch
    pods = 20 * n
    c = synth.make_cluster(n, pods, seed=43, chunk=1024, adversarial=adv, skew=zipf)
    sc, sm = synth.make_specs(s, seed=43, adversarial=adv)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    used_cpu = torch.empty(n, dtype=torch.int64, device=dev)
    used_mem = torch.empty(n, dtype=torch.int64, device=dev)
    partial = torch.empty(2 * s, dtype=torch.int64, device=dev)
    totals = torch.empty(s, dtype=torch.int64, device=dev)
    err = torch.empty(s, dtype=torch.int32, device=dev)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    args = (T(c.node_ptr), T(c.cpu_req), T(c.mem_req), T(c.alloc_cpu), T(c.alloc_mem),
            T(c.alloc_pods), T(c.pod_count), used_cpu, used_mem, T(sc), T(sm))
    stream = torch.cuda.Stream(dev)
    engine.set_clamp_in_fit(mode)
    try:
        for k in range(2):
            totals.fill_(-7)
            with torch.cuda.stream(stream):
                if k == 0:
                    engine.capacity_async(c.node_ptr, *args, totals, err, stream=stream)
                else:
                    engine.capacity_partial_async(c.node_ptr, *args, partial, n_chunks=1, stream=stream)
                    engine.fit_finalize_async(s, partial, totals, err, stream=stream)
            stream.synchronize()
            np.testing.assert_array_equal(totals.cpu().numpy(), ot, err_msg=f"call {k}")
            np.testing.assert_array_equal(err.cpu().numpy(), oe, err_msg=f"call {k}")
    finally:
        engine.set_clamp_in_fit(-1)


# ---- pipelined reduce + fit (node chunks, side stream) == host API ------------------------
@pytest.mark.parametrize("n_chunks", [1, 2, 3, 4, 16])
def test_pipelined_capacity_matches_host(engine, n_chunks):
    import torch
    c = synth.make_cluster(300_001, 6_000_000, seed=31, chunk=4096, adversarial=True)
    sc, sm = synth.make_specs(333, seed=31, adversarial=True)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    n, s = c.n_nodes, sc.size
    used_cpu = torch.full((n,), 7, dtype=torch.int64, device=dev)   # garbage: must be overwritten
    used_mem = torch.full((n,), 7, dtype=torch.int64, device=dev)
    partial = torch.empty(2 * s, dtype=torch.int64, device=dev)
    totals = torch.empty(s, dtype=torch.int64, device=dev)
    err = torch.empty(s, dtype=torch.int32, device=dev)
    args = [T(c.node_ptr), T(c.cpu_req), T(c.mem_req), T(c.alloc_cpu), T(c.alloc_mem),
            T(c.alloc_pods), T(c.pod_count), used_cpu, used_mem, T(sc), T(sm), partial]
    stream = torch.cuda.Stream(dev)
    engine.profile_enable(True)
    with torch.cuda.stream(stream):
        for _ in range(2):  # back to back: the second call must wait for the first's fits
            engine.capacity_partial_async(c.node_ptr, *args, n_chunks=n_chunks, stream=stream)
            engine.fit_finalize_async(s, partial, totals, err, stream=stream)
    stream.synchronize()
    rms, rn, fms, fn = engine.profile_read()
    engine.profile_enable(False)
    assert rn == fn and rn >= 2 and rms > 0 and fms > 0
    np.testing.assert_array_equal(used_cpu.cpu().numpy().view(np.uint64), seg_sums(c.node_ptr, c.cpu_req))
    np.testing.assert_array_equal(used_mem.cpu().numpy().view(np.uint64), seg_sums(c.node_ptr, c.mem_req))
    ht, he = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                             c.alloc_pods, c.pod_count, sc, sm)
    np.testing.assert_array_equal(err.cpu().numpy(), he)
    np.testing.assert_array_equal(totals.cpu().numpy(), ht)


def test_pipelined_rejects_bad_host_csr(engine):
    import torch
    from kubernetesclustercapacity_amd import KccError
    dev = torch.device("cuda", 0)
    n = 100_000
    ptr = np.arange(n + 1, dtype=np.int64)
    bad = ptr.copy()
    bad[n // 2:] = 10 * n  # the chunk boundaries past the middle point beyond n_containers
    z = lambda k: torch.zeros(k, dtype=torch.int64, device=dev)  # noqa: E731
    with pytest.raises(KccError):
        engine.capacity_partial_async(bad, z(n + 1), z(n), z(n), z(n), z(n), z(n), z(n), z(n),
                                      z(n), z(4), z(4), z(8), n_chunks=4)


# ---- BASELINE config C4 at full size: size-independent properties ------------------------
@pytest.fixture(scope="module")
def c4():
    return synth.config_cluster("C4"), synth.config_specs("C4")


def test_c4_reduce_exact(engine, c4):
    c, _ = c4
    r = engine.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req)
    np.testing.assert_array_equal(r.cpu_requests, seg_sums(c.node_ptr, c.cpu_req))
    np.testing.assert_array_equal(r.memory_requests.view(np.uint64),
                                  seg_sums(c.node_ptr, c.mem_req))
    # checksum of checksums
    assert int(r.cpu_requests.sum(dtype=np.uint64)) == int(c.cpu_req.sum(dtype=np.uint64))


def test_c4_fit_sample_linearity_determinism(engine, c4):
    c, (sc, sm) = c4
    uc = seg_sums(c.node_ptr, c.cpu_req)
    um = seg_sums(c.node_ptr, c.mem_req).view(np.int64)
    t, e = engine.capacity(c.node_ptr, c.cpu_req, c.mem_req, c.alloc_cpu, c.alloc_mem,
                           c.alloc_pods, c.pod_count, sc, sm)
    assert not e.any()
    frac = engine.last_slow_fraction()
    assert 0.0 <= frac < 0.05, frac       # synthetic C4 stays on the fast path
    # a spec sample against the oracle over all 1M nodes
    idx = np.random.default_rng(4).choice(sc.size, 24, replace=False)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc[idx],
                         sm[idx], NT)
    np.testing.assert_array_equal(t[idx], ot)
    # node-shard linearity: halves sum to the whole (mod 2^64)
    h = c.n_nodes // 2
    args = (c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um)
    ta, _ = engine.total_possible_max_replicas(*[x[:h] for x in args], sc, sm)
    tb, _ = engine.total_possible_max_replicas(*[x[h:] for x in args], sc, sm)
    np.testing.assert_array_equal((ta.view(np.uint64) + tb.view(np.uint64)).view(np.int64), t)
    # run-to-run identity
    t2, _ = engine.total_possible_max_replicas(*args, sc, sm)
    np.testing.assert_array_equal(t2, t)


def test_reduce_lookback_never_timed_out(engine):
    """Every reduce launch of this session assembled its range-cut nodes from the pieces
    the other waves published (decoupled look-back): no wait gave up."""
    assert engine.reduce_faults() == 0


@pytest.mark.parametrize("seed", [5, 6])
def test_node_prep_in_reduce_range_boundaries(engine, seed):
    """Node prep inside the reduce launch (clamp in the fit, one node chunk: kcc::NpArgs)
    waits for the flags of the reduce waves storing its rows.  CSR offsets built against
    that window: empty nodes at every multiple of 512 containers (every possible range
    boundary), leading and trailing empty nodes, one node spanning ~300k containers (many
    ranges), the rest cut at random.  Three calls in a row (the epoch advances): node sums
    and totals == the oracle."""
    import torch
    n = 20_000
    c = synth.make_cluster(n, 2_000_000, seed=seed, chunk=1024)
    total = int(c.node_ptr[-1])
    rng = np.random.default_rng(seed)
    mult = np.arange(512, total, 512)
    giant0 = total // 3
    mult = mult[(mult < giant0) | (mult > giant0 + 300_000)]
    fixed = np.concatenate([np.zeros(3, np.int64), np.repeat(mult, 2), np.full(3, total, np.int64)])
    assert fixed.size < n - 100
    free = rng.integers(0, total, n - 1 - fixed.size)
    free = free[(free < giant0) | (free > giant0 + 300_000)]
    free = np.concatenate([free, rng.integers(0, giant0, n - 1 - fixed.size - free.size)])
    ptr = np.concatenate([[0], np.sort(np.concatenate([fixed, free]))[: n - 1], [total]]).astype(np.int64)
    assert ptr.size == n + 1 and np.all(np.diff(ptr) >= 0)
    sc, sm = synth.make_specs(700, seed=seed)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    uc, um, _, _ = coracle.reduce_requests(ptr, c.cpu_req, c.mem_req, c.cpu_lim, c.mem_lim)
    ot, oe = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um, sc, sm, NT)
    used_cpu = torch.empty(n, dtype=torch.int64, device=dev)
    used_mem = torch.empty(n, dtype=torch.int64, device=dev)
    totals = torch.empty(sc.size, dtype=torch.int64, device=dev)
    err = torch.empty(sc.size, dtype=torch.int32, device=dev)
    args = (T(ptr), T(c.cpu_req), T(c.mem_req), T(c.alloc_cpu), T(c.alloc_mem),
            T(c.alloc_pods), T(c.pod_count), used_cpu, used_mem, T(sc), T(sm))
    stream = torch.cuda.Stream(dev)
    engine.set_clamp_in_fit(1)
    try:
        for k in range(3):
            totals.fill_(-7)
            used_cpu.fill_(-7)
            with torch.cuda.stream(stream):
                engine.capacity_async(ptr, *args, totals, err, stream=stream)
            stream.synchronize()
            np.testing.assert_array_equal(used_cpu.cpu().numpy().view(np.uint64), uc, err_msg=f"call {k}")
            np.testing.assert_array_equal(used_mem.cpu().numpy(), um, err_msg=f"call {k}")
            np.testing.assert_array_equal(totals.cpu().numpy(), ot, err_msg=f"call {k}")
            np.testing.assert_array_equal(err.cpu().numpy(), oe, err_msg=f"call {k}")
    finally:
        engine.set_clamp_in_fit(-1)
    assert engine.reduce_faults() == 0  # no wait gave up
