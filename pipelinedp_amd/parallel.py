"""Multi-GPU execution: rows sharded by privacy id, one accumulator exchange.

All contribution bounding is a function of one privacy id's rows
(contribution_bounders.py:62-111), so each rank bounds and reduces its own
shard with no communication.  The only exchange is the per-partition merge
(LocalBackend.combine_accumulators_per_key, pipeline_backend.py:555-565):
the dense per-partition accumulator arrays are summed across ranks with one
reduce-scatter (RCCL over xGMI on MI355X; gloo in the CPU tests), after which
rank r owns partitions [r * slice, (r + 1) * slice) and runs selection and
noise on them locally (noise counters are global partition indices, so the
result does not depend on the number of ranks).
"""
from typing import Dict, Optional, Tuple


def world_info(group=None) -> Tuple[int, int]:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def partition_slices(n_partitions: int, world: int) -> Tuple[int, int]:
    """(padded partition count, partitions per rank)."""
    padded = ((n_partitions + world - 1) // world) * world
    return padded, padded // world


def exchange_accumulators(acc: Dict[str, Optional["torch.Tensor"]], group=None):
    """Sums the dense accumulators of all ranks and returns (this rank's
    slice of every accumulator, global index of the slice's first partition).
    Accumulator tensors must have the padded length partition_slices(...)[0]."""
    import torch
    import torch.distributed as dist
    world, rank = world_info(group)
    if world == 1:
        return acc, 0
    sizes = {t.shape[0] for t in acc.values() if t is not None}
    if len(sizes) != 1:
        raise ValueError("accumulators must have equal lengths")
    padded = sizes.pop()
    if padded % world:
        raise ValueError(f"accumulator length {padded} is not a multiple of world size {world}")
    slice_len = padded // world
    backend = dist.get_backend(group)
    out = {}
    for name, t in acc.items():
        if t is None:
            out[name] = None
            continue
        if backend == "nccl":
            part = torch.empty(slice_len, dtype=t.dtype, device=t.device)
            dist.reduce_scatter_tensor(part, t.contiguous(), op=dist.ReduceOp.SUM, group=group)
        else:  # gloo (CPU tests): all-reduce then keep the owned slice
            full = t.clone()
            dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
            part = full[rank * slice_len:(rank + 1) * slice_len].clone()
        out[name] = part
    return out, rank * slice_len


def shard_by_privacy_id(privacy_ids, world: int, rank: int):
    """Boolean mask of the rows rank `rank` owns (privacy id hashed mod world),
    for callers that shard their own input before building a ColumnTable."""
    import numpy as np
    pid = np.asarray(privacy_ids)
    if pid.dtype.kind in "iu":
        h = (pid.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(32)
        return (h % np.uint64(world)) == np.uint64(rank)
    import hashlib
    return np.fromiter((int(hashlib.blake2b(repr(p).encode(), digest_size=8).hexdigest(), 16) % world == rank
                        for p in pid), dtype=bool, count=len(pid))
