"""Seeded synthetic clusters for parity tests and benchmarks.

A cluster is generated in node chunks of CHUNK nodes, each from its own
PCG64(seed, chunk) stream, so any contiguous node range (a rank's shard) can be
generated alone and is identical to the same rows of the whole cluster.

Arrays (SoA, the engine's input layout):
  alloc_cpu u64[N] (millicores), alloc_mem i64[N] (bytes), alloc_pods i64[N],
  pod_count i64[N] (= len(pods), CC:106/135), node_ptr i64[N+1] (CSR over containers),
  cpu_req u64[C], mem_req i64[C], cpu_lim u64[C], mem_lim i64[C],
  spec_cpu u64[S], spec_mem i64[S].
Unhealthy nodes are zero rows (CC:221-226): alloc 0/0/0, and their "pods" are the
pods listed for node name "" (none by default).

Pods per node: C2-C4 Poisson with the config's mean; C5 (skew="zipf", also
skew=True) Zipf with s = 1.2 (numpy's Generator.zipf: P(k) ∝ k^-1.2, k >= 1) capped at
2 x allocatable pods — the survey's distribution, so its pod total follows from it
(~122 pods per node: ~611M pods on 5M nodes; ~32 % of the nodes hold more pods than
allocatable: negative clamps, CC:135).  skew="lognormal" is round 3's mean-matched
lognormal (sigma 1, capped the same way), kept only as a named alternative.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

CHUNK = 1 << 14
KIB, MIB, GIB = 1 << 10, 1 << 20, 1 << 30
ZIPF_S = 1.2  # C5 pods per node ~ Zipf(s ≈ 1.2), capped at 2 x alloc_pods

CONFIGS = {
    # BASELINE.json configs (C1 is the reference's CPU-only fake-clientset case)
    "C1": dict(n_nodes=100, pods=1_000, n_specs=1, skew=False),
    "C2": dict(n_nodes=10_000, pods=200_000, n_specs=1, skew=False),
    "C3": dict(n_nodes=100_000, pods=2_000_000, n_specs=256, skew=False),
    "C4": dict(n_nodes=1_000_000, pods=20_000_000, n_specs=4096, skew=False),
    # C5: pods from the Zipf draw (the total is the distribution's, ~611M; `pods` is
    # the expected value, used only for labels)
    "C5": dict(n_nodes=5_000_000, pods=611_000_000, n_specs=16384, skew="zipf"),
}


@dataclass
class Cluster:
    node_lo: int
    alloc_cpu: np.ndarray
    alloc_mem: np.ndarray
    alloc_pods: np.ndarray
    pod_count: np.ndarray
    node_ptr: np.ndarray
    cpu_req: np.ndarray
    mem_req: np.ndarray
    cpu_lim: np.ndarray
    mem_lim: np.ndarray
    meta: dict = field(default_factory=dict)

    @property
    def n_nodes(self) -> int:
        return self.alloc_cpu.size

    @property
    def n_containers(self) -> int:
        return self.cpu_req.size


def _skew_kind(skew) -> str:
    if skew is True or skew == "zipf":
        return "zipf"
    if skew in (False, None, "poisson"):
        return "poisson"
    if skew == "lognormal":
        return "lognormal"
    raise ValueError(f"skew: False / 'poisson', True / 'zipf' or 'lognormal', not {skew!r}")


def _chunk(seed: int, ci: int, n: int, mean_pods: float, skew, unhealthy: float,
           adversarial: bool, limits: bool = True):
    rng = np.random.Generator(np.random.PCG64([seed, ci]))
    alloc_cpu = rng.choice(np.array([4000, 8000, 16000, 32000, 64000, 96000], np.uint64), n)
    alloc_mem = rng.integers(8 * GIB // KIB, 512 * GIB // KIB, n, dtype=np.int64) * KIB
    alloc_pods = rng.choice(np.array([110, 250], np.int64), n)
    kind = _skew_kind(skew)
    if kind == "zipf":
        # Zipf(s = 1.2) pods per node, capped at 2x allocatable pods (the cap
        # makes negative clamps, CC:135); the mean is the distribution's, not mean_pods
        pods = np.minimum(rng.zipf(ZIPF_S, n), 2 * alloc_pods)
    elif kind == "lognormal":
        # round 3's mean-matched lognormal (sigma 1), capped the same way
        raw = rng.lognormal(np.log(max(mean_pods, 1e-9)) - 0.5, 1.0, n)
        pods = np.minimum(np.floor(raw).astype(np.int64), 2 * alloc_pods)
    else:
        pods = rng.poisson(mean_pods, n)
    pods = pods.astype(np.int64)
    zero = rng.random(n) < unhealthy
    alloc_cpu[zero] = 0
    alloc_mem[zero] = 0
    alloc_pods[zero] = 0
    pods[zero] = 0
    if adversarial:
        # overcommit, podCount > allocPods, huge values, negative (wrapped) requests
        k = max(1, n // 16)
        idx = rng.choice(n, k, replace=False)
        pods[idx[: k // 4]] = alloc_pods[idx[: k // 4]] + rng.integers(1, 50, k // 4)
        alloc_cpu[idx[k // 4: k // 2]] = rng.integers(0, 1 << 63, k // 2 - k // 4,
                                                      dtype=np.uint64) * np.uint64(2)
        alloc_mem[idx[k // 2: 3 * k // 4]] = rng.integers(1 << 40, 1 << 62, 3 * k // 4 - k // 2,
                                                          dtype=np.int64)
        alloc_pods[idx[3 * k // 4:]] = rng.integers(-5, 1 << 20, k - 3 * k // 4)
    # containers: 1-3 per pod
    npods = int(pods.sum())
    cpp = rng.integers(1, 4, npods)
    per_node = np.zeros(n, np.int64)
    pod_node = np.repeat(np.arange(n), pods)
    np.add.at(per_node, pod_node, cpp)
    c = int(per_node.sum())
    cpu_req = (rng.integers(1, 41, c) * 50).astype(np.uint64)
    cpu_req[rng.random(c) < 0.15] = 0
    mem_bin = rng.integers(64, 8 * 1024, c, dtype=np.int64) * MIB       # "Mi" quantities
    mem_dec = rng.integers(64, 8 * 1024, c, dtype=np.int64) * 1_000_000  # "M" quantities
    mem_req = np.where(rng.random(c) < 0.5, mem_bin, mem_dec)
    mem_req[rng.random(c) < 0.10] = 0
    cpu_lim = cpu_req * np.uint64(2) if limits else np.zeros(0, np.uint64)
    mem_lim = mem_req * 2 if limits else np.zeros(0, np.int64)
    if adversarial and c:
        k = max(1, c // 64)
        idx = rng.choice(c, k, replace=False)
        cpu_req[idx[: k // 2]] = np.uint64(2**64 - 100)  # "-100m" wraps (CC:318, K8)
        mem_req[idx[k // 2:]] = rng.integers(-(1 << 62), 1 << 62, k - k // 2, dtype=np.int64)
    return alloc_cpu, alloc_mem, alloc_pods, pods, per_node, cpu_req, mem_req, cpu_lim, mem_lim


def make_cluster(n_nodes: int, pods: int, seed: int = 20261015, node_lo: int = 0,
                 node_hi: int | None = None, skew=False, unhealthy: float = 0.01,
                 adversarial: bool = False, chunk: int = CHUNK, limits: bool = True) -> Cluster:
    """Nodes [node_lo, node_hi) of the cluster (seed, n_nodes, pods).  skew: False (Poisson
    with mean pods / n_nodes), True / "zipf" (SURVEY §8d's Zipf(1.2) capped at 2 x alloc
    pods; `pods` is then not used) or "lognormal".  limits=False: no limit arrays (empty),
    for workloads that never read them (the bench at C5 scale)."""
    node_hi = n_nodes if node_hi is None else node_hi
    mean = pods / max(n_nodes, 1)
    parts = []
    for ci in range(node_lo // chunk, (node_hi + chunk - 1) // chunk if node_hi > node_lo else 0):
        c0 = ci * chunk
        cn = min(chunk, n_nodes - c0)
        g = _chunk(seed, ci, cn, mean, skew, unhealthy, adversarial, limits)
        a, b = max(node_lo, c0) - c0, min(node_hi, c0 + cn) - c0
        per_node = g[4]
        cptr = np.concatenate([[0], np.cumsum(per_node)])
        parts.append((g[0][a:b], g[1][a:b], g[2][a:b], g[3][a:b], per_node[a:b],
                      *(x[cptr[a]:cptr[b]] if x.size else x for x in g[5:])))
    if parts:
        cols = [np.concatenate([p[k] for p in parts]) for k in range(9)]
    else:
        cols = [np.zeros(0, t) for t in (np.uint64, np.int64, np.int64, np.int64, np.int64,
                                          np.uint64, np.int64, np.uint64, np.int64)]
    node_ptr = np.zeros(cols[0].size + 1, np.int64)
    np.cumsum(cols[4], out=node_ptr[1:])
    return Cluster(node_lo, cols[0], cols[1], cols[2], cols[3].astype(np.int64), node_ptr,
                   cols[5], cols[6], cols[7], cols[8],
                   meta=dict(n_nodes_total=n_nodes, pods=pods, seed=seed, skew=_skew_kind(skew)))


def make_specs(n_specs: int, seed: int = 20261015, adversarial: bool = False):
    """What-if pod specs: cpu log-uniform 1-8000 m, memory log-uniform 1 MiB-32 GiB."""
    rng = np.random.Generator(np.random.PCG64([seed, 0x5BEC]))
    cpu = np.exp(rng.uniform(np.log(1), np.log(8000), n_specs)).astype(np.uint64)
    cpu = np.maximum(cpu, np.uint64(1))
    mem = np.exp(rng.uniform(np.log(MIB), np.log(32 * GIB), n_specs)).astype(np.int64)
    if adversarial and n_specs:
        k = max(1, n_specs // 8)
        idx = rng.choice(n_specs, min(n_specs, 6 * k), replace=False)
        cpu[idx[:k]] = 0                                   # div-by-zero flag (K7)
        mem[idx[k:2 * k]] = 0
        mem[idx[2 * k:3 * k]] = -rng.integers(1, 1 << 40, len(idx[2 * k:3 * k]))
        cpu[idx[3 * k:4 * k]] = rng.integers(1 << 23, 1 << 63, len(idx[3 * k:4 * k]),
                                             dtype=np.uint64)
        mem[idx[4 * k:5 * k]] = rng.integers(1 << 37, 1 << 62, len(idx[4 * k:5 * k]),
                                             dtype=np.int64)
        mem[idx[5 * k:6 * k]] = -1
    return cpu, mem


def config_cluster(name: str, node_lo: int = 0, node_hi: int | None = None, seed: int = 20261015,
                   limits: bool = True):
    cfg = CONFIGS[name]
    s = seed + int(name[1:])
    return make_cluster(cfg["n_nodes"], cfg["pods"], seed=s, node_lo=node_lo, node_hi=node_hi,
                        skew=cfg["skew"], limits=limits)


def config_specs(name: str, seed: int = 20261015):
    return make_specs(CONFIGS[name]["n_specs"], seed=seed + int(name[1:]))
