"""kubernetesclustercapacity_amd — MI355X-native engine for the hot path of
AshutoshNirkhe/KubernetesClusterCapacity (per-node request sums + nodes x specs fit).

The compute lives in libkcc.so (hand-written gfx950 HIP kernels behind the C-ABI of
include/kcc.h).  Importing this package does not touch the GPU; constructing a
CapacityEngine loads libkcc.so and fails loudly if it is missing.
"""
from .engine import CapacityEngine, KccError, RequestSums, verdict  # noqa: F401
from .shard import node_range, shard_bounds  # noqa: F401

__all__ = ["CapacityEngine", "KccError", "RequestSums", "verdict", "node_range",
           "shard_bounds"]
