"""List-order (keyed) request sums: containers of a cluster-wide
Pods("").List in namespace/name order, each tagged with its node's row, must give the
sums of getPodCPUMemoryRequestsLimits (CC:255-299) per row bit for bit — checked
against the C oracle on the same containers grouped into CSR (stable by key)."""
import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from oracle import coracle


def list_order(c, seed, skip_frac=0.0):
    """Shuffle a CSR cluster into pod-list order: pods permuted, a pod's containers kept
    together (as the API returns them); some pods keyed off the rows (skipped)."""
    rng = np.random.default_rng(seed)
    n = c.n_nodes
    node_of = np.repeat(np.arange(n, dtype=np.int32), np.diff(c.node_ptr))
    # pods: runs of 1-3 containers within a node
    starts = np.flatnonzero(np.r_[True, (rng.random(node_of.size - 1) < 0.5) |
                                  (node_of[1:] != node_of[:-1])])
    mark = np.zeros(node_of.size, bool)
    mark[starts] = True
    pod_of = np.cumsum(mark) - 1
    perm_pods = rng.permutation(starts.size)
    order = np.argsort(perm_pods[pod_of], kind="stable")
    key = node_of[order].copy()
    if skip_frac:
        bad = rng.random(key.size) < skip_frac
        key[bad] = rng.choice(np.array([-1, n, n + 7, -(2 ** 31)], np.int32), bad.sum())
    return key, c.cpu_req[order], c.mem_req[order], order, pod_of[order], key


def oracle_keyed(n, key, cpu, mem, cl=None, ml=None):
    ok = (key >= 0) & (key < n)
    srt = np.argsort(key[ok], kind="stable")
    k = key[ok][srt]
    ptr = np.searchsorted(k, np.arange(n + 1)).astype(np.int64)
    sel = lambda a: None if a is None else a[ok][srt]  # noqa: E731
    return coracle.reduce_requests(ptr, sel(cpu), sel(mem), sel(cl), sel(ml))


def test_list_order_model_matches_csr():
    """The host-side model (oracle over the regrouped list) equals the CSR sums."""
    c = synth.make_cluster(2_000, 30_000, seed=3, chunk=512)
    key, cpu, mem, *_ = list_order(c, 1)
    a = oracle_keyed(c.n_nodes, key, cpu, mem)
    b = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.fixture(scope="module")
def eng():
    from tests.conftest import init_torch_first
    init_torch_first()
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1) as e:
        yield e


@pytest.mark.gpu
@pytest.mark.parametrize("n,pods,skip,adv", [(1, 10, 0.0, False), (3_000, 60_000, 0.0, True),
                                             (20_000, 400_000, 0.05, True),
                                             (50_000, 200_000, 0.3, False)])
def test_gpu_keyed_matches_oracle(eng, n, pods, skip, adv):
    c = synth.make_cluster(n, pods, seed=n, chunk=1024, adversarial=adv)
    key, cpu, mem, *_ = list_order(c, n + 1, skip)
    rng = np.random.default_rng(n)
    cl = rng.integers(0, 1 << 63, key.size, dtype=np.int64).view(np.uint64) * np.uint64(3)
    ml = rng.integers(-(1 << 62), 1 << 62, key.size, dtype=np.int64)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(n, key, cpu, mem, cl, ml)
    o = oracle_keyed(n, key, cpu, mem, cl, ml)
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    assert np.array_equal(r.cpu_limits, o[2]) and np.array_equal(r.memory_limits, o[3])
    r2 = eng.get_pod_cpu_memory_requests_limits_keyed(n, key, cpu, mem)
    assert np.array_equal(r2.cpu_requests, o[0]) and np.array_equal(r2.memory_requests, o[1])


@pytest.mark.gpu
def test_gpu_keyed_edges(eng):
    r = eng.get_pod_cpu_memory_requests_limits_keyed(5, np.zeros(0, np.int32), [], [])
    assert (r.cpu_requests == 0).all() and r.cpu_requests.size == 5
    # tails (n % 4 != 0), one key everywhere, runs crossing lane quads
    for nc in (1, 2, 3, 5, 7, 1025):
        key = np.zeros(nc, np.int32)
        v = np.arange(1, nc + 1, dtype=np.uint64)
        r = eng.get_pod_cpu_memory_requests_limits_keyed(1, key, v, v.astype(np.int64))
        assert int(r.cpu_requests[0]) == nc * (nc + 1) // 2
    # wrapping: 2^63 + 2^63 == 0 mod 2^64
    r = eng.get_pod_cpu_memory_requests_limits_keyed(
        2, np.array([1, 1, 0], np.int32), np.array([1 << 63, 1 << 63, 5], np.uint64),
        np.array([-(1 << 63), -(1 << 63), 7], np.int64))
    assert r.cpu_requests.tolist() == [5, 0] and r.memory_requests.tolist() == [7, 0]
    # staged records: row 4095 of a bucket with the low cpu bits all ones, and cpu requests
    # past the record's field (their high parts on the escape list)
    key = np.array([4095, 4095, 4095, 8191, 1], np.int32)
    cpu = np.array([(1 << 20) - 1, (1 << 20) + 3, (1 << 64) - 1, (1 << 40) + 5, 1 << 20],
                   np.uint64)
    mem = np.array([1, 2, 3, 4, 5], np.int64)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(8192, key, cpu, mem)
    o = oracle_keyed(8192, key, cpu, mem)
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    assert int(r.cpu_requests[4095]) == ((1 << 21) + 1) % (1 << 64)
    # memory requests the record holds and the ones it does not (odd, negative, large):
    # the latter on the escape list
    mem = np.array([64, 100, -64, 1 << 38, (1 << 38) - 64], np.int64)
    cpu = np.array([1, 2, 3, 4, 5], np.uint64)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(8192, key, cpu, mem)
    o = oracle_keyed(8192, key, cpu, mem)
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])


@pytest.mark.gpu
def test_gpu_keyed_record_fields(eng):
    """The sweep's staged record (kcc_keyed.hip kb_record: 20 cpu bits, memory / 64 below
    2^38) and round 5's measured-and-dropped 6-byte one (16 cpu bits, memory as 19-bit MiB
    or 10^6-B counts): values at and around every field edge of both, and the escapes past
    them — each container alone on its row, and all of them on one row."""
    MI, M = 1 << 20, 1_000_000
    cpu_edges = [0, 1, (1 << 16) - 1, 1 << 16, (1 << 16) + 1, (1 << 20) - 1, 1 << 20,
                 (1 << 64) - 1, (1 << 63) + 7]
    mem_edges = [0, MI, ((1 << 19) - 1) * MI, (1 << 19) * MI, ((1 << 19) + 1) * MI,
                 M, ((1 << 19) - 1) * M, (1 << 19) * M, ((1 << 19) - 1) * M + 1,
                 15625 * MI, 64, 100, -MI, -M, 1 << 62, -(1 << 63), (1 << 63) - 1,
                 250 * M, 128 * MI, 3 * MI + M, (1 << 38) - 64, 1 << 38, (1 << 38) + 64]
    cpu = np.array([c for c in cpu_edges for _ in mem_edges], np.uint64)
    mem = np.array([m for _ in cpu_edges for m in mem_edges], np.int64)
    nk = cpu.size
    for key in (np.arange(nk, dtype=np.int32), np.full(nk, 4097, np.int32)):
        r = eng.get_pod_cpu_memory_requests_limits_keyed(8192, key, cpu, mem)
        o = oracle_keyed(8192, key, cpu, mem)
        assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])


@pytest.mark.gpu
@pytest.mark.parametrize("nk", [1, 4096, 4097, 2 * 4096 + 7, 5 * 4096, 97 * 4096 + 11])
def test_gpu_keyed_bucket_groups(eng, nk):
    """The gather's bucket pairs and parts: one bucket, a key space ending exactly on a
    bucket, an odd bucket count (the last group a single bucket), few groups gathered by up
    to 4 parts each, and a mid-size key space; a 300k-container list with a hot row on each
    side of every pair's split and rows at both ends."""
    rng = np.random.default_rng(nk)
    key = rng.integers(-1, nk + 1, 300_001).astype(np.int32)
    hot = [0, nk - 1, min(nk - 1, 4095), min(nk - 1, 4096)]
    key[rng.random(key.size) < 0.2] = hot[0]
    key[:len(hot)] = hot
    cpu = (rng.integers(0, 41, key.size) * 50).astype(np.uint64)
    mem = rng.integers(0, 8192, key.size).astype(np.int64) << 20
    r = eng.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem)
    o = oracle_keyed(nk, key, cpu, mem)
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    ok = key[(key >= 0) & (key < nk)]
    assert np.array_equal(eng.count_by_key(nk, key), np.bincount(ok, minlength=nk).astype(np.int64))


@pytest.mark.gpu
def test_gpu_keyed_atomic_fallback(eng):
    """More rows than the bucketed path holds (4096 buckets x 4096 rows): the device-atomic
    kernels."""
    nk = 4096 * 4096 + 5
    rng = np.random.default_rng(6)
    key = rng.integers(-2, nk + 2, 50_001).astype(np.int32)
    key[:7] = [nk - 1, nk - 1, 0, 0, 5, nk, -1]
    v = rng.integers(0, 1 << 62, key.size).astype(np.uint64)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(nk, key, v, v.astype(np.int64))
    o = oracle_keyed(nk, key, v, v.astype(np.int64))
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    got = eng.count_by_key(nk, key)
    ok = key[(key >= 0) & (key < nk)]
    assert np.array_equal(got, np.bincount(ok, minlength=nk).astype(np.int64))


@pytest.mark.gpu
def test_gpu_keyed_max_buckets_with_limits(eng):
    """The largest bucketed key space (4096 buckets x 4096 rows) with limits: the scatter's
    LDS (cursors for 4096 buckets + the 4-value stage) at its maximum."""
    nk = 4096 * 4096
    rng = np.random.default_rng(8)
    key = rng.integers(0, nk, 300_000).astype(np.int32)
    key[:4] = [nk - 1, nk - 1, 0, 4095]
    v = rng.integers(0, 1 << 62, (4, key.size)).astype(np.uint64)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(nk, key, v[0], v[1].astype(np.int64),
                                                      v[2], v[3].astype(np.int64))
    o = oracle_keyed(nk, key, v[0], v[1].astype(np.int64), v[2], v[3].astype(np.int64))
    for got, want in zip((r.cpu_requests, r.memory_requests, r.cpu_limits, r.memory_limits), o):
        assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_count_by_key(eng):
    rng = np.random.default_rng(4)
    key = rng.integers(-3, 1003, 100_003).astype(np.int32)
    got = eng.count_by_key(1000, key)
    ok = key[(key >= 0) & (key < 1000)]
    assert np.array_equal(got, np.bincount(ok, minlength=1000).astype(np.int64))


@pytest.mark.gpu
def test_gpu_keyed_c4_equals_csr(eng):
    """C4 scale: 1M rows, 39.6M containers in list order == the CSR reduce, bit for bit."""
    c = synth.config_cluster("C4")
    key, cpu, mem, *_ = list_order(c, 9)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(c.n_nodes, key, cpu, mem)
    s = eng.get_pod_cpu_memory_requests_limits(c.node_ptr, c.cpu_req, c.mem_req)
    assert np.array_equal(r.cpu_requests, s.cpu_requests)
    assert np.array_equal(r.memory_requests, s.memory_requests)


@pytest.mark.gpu
@pytest.mark.parametrize("nc", [8191, 8192, 8193, 16385, 3 * 8192 + 3, 200_001, 2_200_001])
def test_gpu_keyed_sweep_tiles(eng, nc):
    """The one-sweep path's tiles (8192 containers each; past one per CU, cut into whole
    rounds, and several per persistent workgroup): sizes around and across tile
    boundaries, a skewed key mix (half of the containers on one row: segments far longer
    than a wave's 64-record step), skipped keys, the largest key space (4096 buckets: the
    packed 16-bit LDS counters of all of them), and two calls in a row (the escape list and
    the gather's arrival counters are left empty / zero)."""
    nk = 4096 * 4096
    rng = np.random.default_rng(nc)
    key = rng.integers(-1, nk + 1, nc).astype(np.int32)
    key[rng.random(nc) < 0.5] = 12345
    key[:3] = [nk - 1, 0, 4096]
    cpu = (rng.integers(0, 41, nc) * 50).astype(np.uint64)
    cpu[rng.random(nc) < 0.01] = np.uint64(1 << 40)   # escapes
    mem = rng.integers(0, 8192, nc).astype(np.int64) << 20
    mem[rng.random(nc) < 0.01] = 12345                # escapes
    o = oracle_keyed(nk, key, cpu, mem)
    for _ in range(2):
        r = eng.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem)
        assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    ok = key[(key >= 0) & (key < nk)]
    assert np.array_equal(eng.count_by_key(nk, key), np.bincount(ok, minlength=nk).astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 3, 4, 31, 32, 33, 127, 128, 129, 1023, 4095])
def test_gpu_keyed_bucket_counts_table_blocks(eng, nb):
    """The sweep's table (u16 bucket starts in blocks of 32 buckets, [b / 32][tile][b % 32],
    kcc_keyed.hip kb_tab_at): key spaces whose bucket count sits at and around the block
    edges and the 4-entry groups a sweep thread stores, the last entry (nb) in a block of
    its own or shared, over several tiles per workgroup (more than 256 tiles), vs the
    oracle; the pod counts through the same kernels."""
    nk = (nb - 1) * 4096 + 1 + (nb * 37) % 4096  # nb buckets, the last one partial
    rng = np.random.default_rng(nb)
    nc = 2_300_000
    key = rng.integers(0, nk, nc).astype(np.int32)
    key[rng.random(nc) < 0.02] = -1
    cpu = (rng.integers(0, 41, nc) * 25).astype(np.uint64)
    mem = rng.integers(0, 4096, nc).astype(np.int64) << 20
    o = oracle_keyed(nk, key, cpu, mem)
    r = eng.get_pod_cpu_memory_requests_limits_keyed(nk, key, cpu, mem)
    assert np.array_equal(r.cpu_requests, o[0]) and np.array_equal(r.memory_requests, o[1])
    ok = key[(key >= 0) & (key < nk)]
    assert np.array_equal(eng.count_by_key(nk, key), np.bincount(ok, minlength=nk).astype(np.int64))
