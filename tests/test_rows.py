"""Per-row "Max replicas" of one spec (CC:119-137): kcc_fit_rows
against the C oracle's per-(node, spec) restatement (kcco_fit_one), including the
adversarial slice (wrapping differences, negative clamps, MinInt64 / -1, zero
requests -> per-row panic flags), and the rows summing to the fit's total."""
import numpy as np
import pytest

from kubernetesclustercapacity_amd import synth
from oracle import coracle

U64 = 1 << 64


@pytest.fixture(scope="module")
def eng():
    from tests.conftest import init_torch_first
    init_torch_first()
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1) as e:
        yield e


def rows_case(seed, n=5000):
    c = synth.make_cluster(n, n * 20, seed=seed, chunk=1024, adversarial=True)
    uc, um, _, _ = coracle.reduce_requests(c.node_ptr, c.cpu_req, c.mem_req)
    rng = np.random.default_rng(seed)
    # raw extremes on a few rows (the fit's fast-path bounds do not apply here)
    k = rng.choice(n, 40, replace=False)
    c.alloc_mem[k[:10]] = np.iinfo(np.int64).max
    um[k[:10]] = np.iinfo(np.int64).min + 5         # am - um wraps negative
    c.alloc_cpu[k[10:20]] = np.uint64(U64 - 1)
    c.pod_count[k[20:30]] = np.iinfo(np.int64).min  # P - pc wraps
    c.alloc_pods[k[30:40]] = -3
    return c, uc, um


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [(200, 262_144_000), (1, 1), (0, 1 << 20), (100, 0),
                                  (U64 - 1, -1), (7, -(1 << 63)), (4000, 5 << 30)])
def test_gpu_rows_match_oracle(eng, spec):
    c, uc, um = rows_case(3)
    sc, sm = spec
    q, err = eng.max_replicas_per_row(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count,
                                      uc, um, sc, sm)
    for i in range(c.n_nodes):
        oq, oz = coracle.fit_one(int(c.alloc_cpu[i]), int(c.alloc_mem[i]), int(c.alloc_pods[i]),
                                 int(c.pod_count[i]), int(uc[i]), int(um[i]), sc, sm)
        assert int(err[i]) == oz, i
        if not oz:
            assert int(q[i]) == oq, i
    if not err.any():  # the rows sum (wrapping) to the fit's total
        t, e = coracle.fit(c.alloc_cpu, c.alloc_mem, c.alloc_pods, c.pod_count, uc, um,
                           np.array([sc], np.uint64), np.array([sm], np.int64))
        assert int(q.astype(np.uint64).sum(dtype=np.uint64)) == int(t[0]) % U64


@pytest.mark.gpu
def test_gpu_rows_empty(eng):
    q, err = eng.max_replicas_per_row([], [], [], [], [], [], 1, 1)
    assert q.size == 0 and err.size == 0
