"""Multi-GPU sharding of value batches.

Every LZ4 block is self-contained -- a fresh zeroed table per call
(algorithm/lz4.cc:669) and no cross-value dictionary (compressor.cc:30) -- so a
batch splits into contiguous value ranges, one per GPU, with NO exchange step:
each rank compresses/decompresses its own range on its own HIP stream and the
host stitches the per-device outputs together with a prefix sum of per-device
frame-byte totals.  No RCCL collective touches the data path; torch.distributed
carries only the benchmark's barrier and max-over-ranks of the elapsed time.

Parts of one multipart value (database.cc:143-248, 64 KiB parts) stay on one
device, so the host can apply the sequential disable rule per value without
gathering: pass ``groups`` (a value id per part) and cuts snap to group
boundaries.
"""
from __future__ import annotations

import numpy as np


def byte_balanced_ranges(sizes, world: int, groups=None) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) index ranges, one per rank, balanced by Σ bytes.

    Cut k is placed at the first unit boundary whose prefix sum reaches
    k·total/world (ties to the nearer side); with ``groups`` only boundaries
    where the group id changes are eligible.  Ranges may be empty when there
    are fewer units than ranks."""
    if world < 1:
        raise ValueError("world must be >= 1")
    s = np.asarray(sizes, dtype=np.int64)
    n = len(s)
    if n == 0:
        return [(0, 0)] * world
    csum = np.concatenate([[0], np.cumsum(s)])  # csum[i] = bytes before unit i
    if groups is None:
        eligible = np.arange(n + 1)
    else:
        g = np.asarray(groups)
        if len(g) != n:
            raise ValueError("groups must have one id per unit")
        if n > 1 and np.any(g[1:] < g[:-1]):
            raise ValueError("groups must be non-decreasing (parts of a value are contiguous)")
        eligible = np.concatenate([[0], np.nonzero(g[1:] != g[:-1])[0] + 1, [n]])
    ecs = csum[eligible]
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        j = int(np.searchsorted(ecs, target))
        if j >= len(eligible):
            j = len(eligible) - 1
        if j > 0 and abs(ecs[j - 1] - target) <= abs(ecs[j] - target):
            j -= 1
        cuts.append(max(int(eligible[j]), cuts[-1]))
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def stitch_offsets(per_rank_bytes) -> np.ndarray:
    """Host prefix sum: where each rank's frame bytes start in the combined
    output (the only cross-device step, done on the host after the fact)."""
    b = np.asarray(per_rank_bytes, dtype=np.int64)
    return np.concatenate([[0], np.cumsum(b)[:-1]]) if len(b) else b


def g1_first_piece(rank: int, values_per_rank: int, value_bytes: int) -> int:
    """First G1-long piece of rank's shard when every rank holds the same
    number of equal-size values: the shards are consecutive slices of one
    G1-long stream (100-byte pieces, db_bench_kingdb.cc:113-142)."""
    return rank * ((values_per_rank * value_bytes + 99) // 100)


def max_over_ranks(seconds: float, op: str = "max") -> float:
    """Max (or, with op="sum", the sum) of a scalar over all ranks -- the
    bench's job time and its total bytes; identity when torch.distributed is
    not initialised."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return float(t.item())


def gather_ranks(x: float) -> list[float]:
    """A scalar from every rank, in rank order (the bench's per-GPU rates);
    [x] when torch.distributed is not initialised."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(x)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, float(x))
    return [float(v) for v in out]
