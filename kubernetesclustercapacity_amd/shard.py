"""Node sharding for one-process-per-GPU runs.

Nodes are independent and the per-spec total is an exact int64 (mod 2^64) sum, so
nodes are split into contiguous ranges balanced by node count and the only exchange
is one all-reduce(sum, int64) of the 2*S partial vector (sums + div-by-zero counts)
before kcc_fit_finalize_async.  Mirrors the in-library split of kcc_abi.cpp
(shard_nodes) so the two agree.
"""
from __future__ import annotations


def node_range(n_nodes: int, rank: int, world: int) -> tuple[int, int]:
    return n_nodes * rank // world, n_nodes * (rank + 1) // world


def shard_bounds(n_nodes: int, world: int) -> list[tuple[int, int]]:
    return [node_range(n_nodes, r, world) for r in range(world)]


def allreduce_partial(partial, group=None):
    """Sum the int64 [2*S] partial vector over ranks (RCCL on GPU, gloo on CPU)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    return partial
