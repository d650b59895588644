"""OPT-IN scheduler request model — explicitly NOT the reference's
semantics (the reference sums app containers only, CC:276-294; that stays the default).

Per pod, per resource: max(app sum, init max incl. sidecars) + overhead, as the
kube-scheduler's PodRequests (pkg/api/v1/resource, sidecar-aware form) computes it.
That dependency is absent here, so parity is unpinned beyond the hand-derived cases
below; the C oracle (kcco_pod_requests) and the independent Python restatement
(pyoracle.pod_requests) check each other, and the GPU path is checked bit for bit
against the C oracle.
"""
import numpy as np
import pytest

from oracle import coracle, pyoracle

U64 = 1 << 64
I64_MIN = -(1 << 63)


def pods_case(seed, n_nodes=300, mean_pods=6, extremes=False):
    """Seeded pods grouped by node: 1-3 app containers, 0-3 init containers (some
    restartable), overhead on some pods."""
    rng = np.random.default_rng(seed)
    ppn = rng.poisson(mean_pods, n_nodes)
    node_pod_ptr = np.zeros(n_nodes + 1, np.int64)
    node_pod_ptr[1:] = np.cumsum(ppn)
    P = int(node_pod_ptr[-1])
    nc = rng.integers(1, 4, P)
    ni = rng.choice([0, 0, 1, 2, 3], P)
    pod_ptr = np.zeros(P + 1, np.int64)
    pod_ptr[1:] = np.cumsum(nc)
    init_ptr = np.zeros(P + 1, np.int64)
    init_ptr[1:] = np.cumsum(ni)
    C, I = int(pod_ptr[-1]), int(init_ptr[-1])
    cpu = rng.integers(0, 40, C).astype(np.uint64) * np.uint64(50)
    mem = rng.integers(0, 128, C).astype(np.int64) << 26
    icpu = rng.integers(0, 80, I).astype(np.uint64) * np.uint64(50)
    imem = rng.integers(0, 256, I).astype(np.int64) << 26
    rst = (rng.random(I) < 0.3).astype(np.uint8)
    ocpu = np.where(rng.random(P) < 0.2, rng.integers(0, 500, P), 0).astype(np.uint64)
    omem = np.where(rng.random(P) < 0.2, rng.integers(0, 1 << 28, P), 0).astype(np.int64)
    if extremes:  # wrapping sums, sign flips of the memory max, huge cpu
        k = rng.choice(C, 20, replace=False)
        cpu[k[:10]] = np.uint64(U64 - 7)
        mem[k[10:]] = np.int64(-(1 << 62))
        if I:
            j = rng.choice(I, min(I, 20), replace=False)
            icpu[j[:10]] = np.uint64(U64 - 1000)
            imem[j[10:]] = np.iinfo(np.int64).max - 3
    return dict(node_pod_ptr=node_pod_ptr, pod_ptr=pod_ptr, cpu_req=cpu, mem_req=mem,
                init_ptr=init_ptr, init_cpu=icpu, init_mem=imem, restartable=rst,
                ovh_cpu=ocpu, ovh_mem=omem)


def _pod_kw(case):
    return {k: v for k, v in case.items() if k != "node_pod_ptr"}


# ---- hand-derived cases (oracle, CPU) -----------------------------------------------

# (app cpu, app mem), [(init cpu, init mem, restartable)], overhead -> (cpu, mem)
HAND = [
    ([(100, 10), (200, 20)], [], None, (300, 30)),                       # app sum only
    ([(100, 10), (200, 20)], [(500, 5, 0)], None, (500, 30)),            # init cpu dominates
    ([(100, 10), (200, 20)], [(50, 50, 0)], None, (300, 50)),            # init mem dominates
    # sidecar 100 then a regular init 400: app = 300 + 100; init = max(100, 400 + 100)
    ([(300, 30)], [(100, 1, 1), (400, 40, 0)], None, (500, 41)),
    # regular init before the sidecar does not see it: max(400, 100) vs app 300 + 100
    ([(300, 30)], [(400, 40, 0), (100, 1, 1)], None, (400, 40)),
    ([(300, 30)], [(100, 1, 1), (200, 2, 1)], None, (600, 33)),          # sidecars add up
    ([(100, 10)], [(50, 5, 0)], (7, 3), (107, 13)),                      # overhead
    ([(0, -5)], [], None, (0, -5)),        # no init: max identity keeps a negative sum
    ([(0, -5)], [(0, -9, 0)], None, (0, -5)),                            # signed max
    ([(U64 - 1, 0)], [(5, 0, 0)], None, (U64 - 1, 0)),                   # unsigned max
    ([(U64 - 1, 0), (3, 0)], [], None, (2, 0)),                          # wrapping sum
    ([], [(70, 7, 0)], None, (70, 7)),                                   # no app containers
]


def _hand_arrays(app, init, ovh):
    return dict(pod_ptr=[0, len(app)], cpu_req=np.array([a[0] for a in app], np.uint64),
                mem_req=np.array([a[1] for a in app], np.int64), init_ptr=[0, len(init)],
                init_cpu=np.array([i[0] for i in init], np.uint64),
                init_mem=np.array([i[1] for i in init], np.int64),
                restartable=np.array([i[2] for i in init], np.uint8),
                ovh_cpu=None if ovh is None else np.array([ovh[0]], np.uint64),
                ovh_mem=None if ovh is None else np.array([ovh[1]], np.int64))


@pytest.mark.parametrize("app,init,ovh,want", HAND)
def test_oracles_hand_cases(app, init, ovh, want):
    a = _hand_arrays(app, init, ovh)
    pc, pm = coracle.pod_requests(**a)
    assert (int(pc[0]), int(pm[0])) == want
    assert pyoracle.pod_requests(**a)[0] == want


@pytest.mark.parametrize("seed,extremes", [(1, False), (2, True), (3, True)])
def test_c_oracle_matches_python_oracle(seed, extremes):
    c = pods_case(seed, n_nodes=60, extremes=extremes)
    pc, pm = coracle.pod_requests(**_pod_kw(c))
    py = pyoracle.pod_requests(**_pod_kw(c))
    assert [(int(a), int(b)) for a, b in zip(pc, pm)] == py


def test_default_semantics_is_the_reference_sum():
    """No init containers, no overhead: the per-node sums of the pod requests are the
    reference's container sums (CC:290-293) over the same containers."""
    c = pods_case(4)
    pc, pm = coracle.pod_requests(c["pod_ptr"], c["cpu_req"], c["mem_req"])
    nuc, num, _, _ = coracle.reduce_requests(c["node_pod_ptr"], pc, pm)
    node_ptr = c["pod_ptr"][c["node_pod_ptr"]]  # containers grouped by node
    ruc, rum, _, _ = coracle.reduce_requests(node_ptr, c["cpu_req"], c["mem_req"])
    assert np.array_equal(nuc, ruc) and np.array_equal(num, rum)


# ---- GPU parity (through the C-ABI) ---------------------------------------------------

@pytest.fixture(scope="module")
def eng():
    from tests.conftest import init_torch_first
    init_torch_first()
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1) as e:
        yield e


@pytest.mark.gpu
@pytest.mark.parametrize("app,init,ovh,want", HAND)
def test_gpu_hand_cases(eng, app, init, ovh, want):
    pc, pm = eng.pod_requests(**_hand_arrays(app, init, ovh))
    assert (int(pc[0]), int(pm[0])) == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_nodes,extremes", [(5, 2000, False), (6, 3000, True),
                                                   (7, 50000, False)])
def test_gpu_pod_requests_match_oracle(eng, seed, n_nodes, extremes):
    c = pods_case(seed, n_nodes=n_nodes, extremes=extremes)
    pc, pm = eng.pod_requests(**_pod_kw(c))
    oc, om = coracle.pod_requests(**_pod_kw(c))
    assert np.array_equal(pc, oc) and np.array_equal(pm, om)
    uc, um = eng.reduce_requests_pods(**c)
    nuc, num, _, _ = coracle.reduce_requests(c["node_pod_ptr"], oc, om)
    assert np.array_equal(uc, nuc) and np.array_equal(um, num)


@pytest.mark.gpu
def test_gpu_optional_inputs_absent(eng):
    c = pods_case(8, n_nodes=500)
    for drop in (("init_ptr", "init_cpu", "init_mem", "restartable"), ("restartable",),
                 ("ovh_cpu",), ("ovh_mem", "ovh_cpu")):
        kw = {k: v for k, v in _pod_kw(c).items() if k not in drop}
        pc, pm = eng.pod_requests(**kw)
        oc, om = coracle.pod_requests(**kw)
        assert np.array_equal(pc, oc) and np.array_equal(pm, om), drop


@pytest.mark.gpu
def test_gpu_default_semantics_equals_reduce_requests(eng):
    c = pods_case(9, n_nodes=4000)
    uc, um = eng.reduce_requests_pods(c["node_pod_ptr"], c["pod_ptr"], c["cpu_req"],
                                      c["mem_req"])
    node_ptr = c["pod_ptr"][c["node_pod_ptr"]]
    ruc, rum, _, _ = coracle.reduce_requests(node_ptr, c["cpu_req"], c["mem_req"])
    assert np.array_equal(uc, ruc) and np.array_equal(um, rum)


@pytest.mark.gpu
def test_gpu_empty_nodes_and_pods(eng):
    uc, um = eng.reduce_requests_pods([0, 0, 0], [0], [], [])
    assert uc.tolist() == [0, 0] and um.tolist() == [0, 0]
    pc, pm = eng.pod_requests([0, 0, 0], [], [], init_ptr=[0, 0, 0], init_cpu=[], init_mem=[])
    assert pc.tolist() == [0, 0] and pm.tolist() == [0, 0]
    pc, pm = eng.pod_requests([0], [], [])
    assert pc.size == 0 and pm.size == 0


@pytest.mark.gpu
def test_gpu_rejects_malformed_input(eng):
    from kubernetesclustercapacity_amd import KccError
    with pytest.raises(KccError):  # pod_ptr not ending at n_containers
        eng.pod_requests([0, 2], [1], [1])
    with pytest.raises(KccError):  # decreasing init offsets
        eng.pod_requests([0, 1, 2], [1, 1], [1, 1], init_ptr=[0, 2, 1], init_cpu=[1, 1],
                         init_mem=[1, 1])
    with pytest.raises(ValueError):
        eng.pod_requests([0, 1], [1], [1], restartable=[1])


@pytest.mark.gpu
def test_gpu_device_api_matches_host_api(eng):
    """kcc_pod_requests_async on device tensors (the bench's path) == the host entry."""
    import torch
    c = pods_case(10, n_nodes=3000, extremes=True)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
         for k, v in c.items()}
    P = c["pod_ptr"].size - 1
    pc = torch.empty(P, dtype=torch.int64, device=dev)
    pm = torch.empty(P, dtype=torch.int64, device=dev)
    eng.pod_requests_async(t["pod_ptr"], t["cpu_req"], t["mem_req"], pc, pm, t["init_ptr"],
                           t["init_cpu"], t["init_mem"], t["restartable"], t["ovh_cpu"],
                           t["ovh_mem"])
    torch.cuda.synchronize()
    oc, om = coracle.pod_requests(**_pod_kw(c))
    assert np.array_equal(pc.cpu().numpy().view(np.uint64), oc)
    assert np.array_equal(pm.cpu().numpy(), om)
