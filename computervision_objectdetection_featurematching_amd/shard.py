"""Scene-batch data parallelism across the GPUs of one node.

Problems are independent (TestsDetector.cpp:58-95 keeps no cross-problem state), so a batch of
scenes is split across ranks with no data-path collective; the only exchange is an all-gather of the
fixed-size per-problem result records (mim_result, 96 B each) once per batch — RCCL over xGMI on the
GPU box ("nccl" backend), gloo in the CPU tests.  Model (query) descriptor sets are replicated.
"""
from __future__ import annotations

import numpy as np

from ._lib import RESULT_DTYPE


def shard_range(n_items: int, world: int, rank: int) -> range:
    """Contiguous block of items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def shard_round_robin(n_items: int, world: int, rank: int) -> range:
    """Round-robin assignment (balances adaptive-termination cost on real data)."""
    return range(rank, n_items, world)


def gather_results(local_bytes, world: int, group=None):
    """All-gather equal-sized uint8 tensors of packed mim_result records -> (world, n) structured array.

    `local_bytes` is a torch uint8 tensor (device tensor with the nccl backend, CPU with gloo).  With a
    process group the collective runs at every world size, world 1 included (bench.py creates an RCCL
    group at N = 1 too, so the N = 1 line runs the same all_gather_into_tensor as N = 8); without
    one (a lone process) the gather is the identity copy."""
    import torch
    import torch.distributed as dist

    n = local_bytes.numel()
    flat = torch.empty(world * n, dtype=torch.uint8, device=local_bytes.device)
    if dist.is_available() and dist.is_initialized():
        if dist.get_world_size(group) != world:
            raise ValueError(f"gather_results: world {world}, process group of {dist.get_world_size(group)}")
        dist.all_gather_into_tensor(flat, local_bytes, group=group)
    elif world == 1:
        flat.copy_(local_bytes)
    else:
        raise RuntimeError("gather_results: world > 1 without a process group")
    return flat.view(world, n)


def gather_objects(obj, world: int, group=None) -> list:
    """All-gather one picklable object per rank (the per-scene detections of the real-data run, whose
    scenes are split round-robin: Output.cpp:19-57 loops over every test image, one after another)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        out = [None] * world
        dist.all_gather_object(out, obj, group=group)
        return out
    if world != 1:
        raise RuntimeError("gather_objects: world > 1 without a process group")
    return [obj]


def merge_scene_results(parts: list, n_items: int) -> list:
    """Per-rank lists of (scene index, result) from shard_round_robin shards -> results in scene order;
    every scene exactly once."""
    out = [None] * n_items
    seen = np.zeros(n_items, bool)
    for part in parts:
        for i, r in part:
            if seen[i]:
                raise ValueError(f"scene {i} processed by two ranks")
            seen[i] = True
            out[i] = r
    if not seen.all():
        raise ValueError(f"scenes {np.nonzero(~seen)[0].tolist()} processed by no rank")
    return out


def decode(gathered) -> np.ndarray:
    arr = gathered.cpu().numpy()
    return arr.reshape(arr.shape[0], -1).view(RESULT_DTYPE)


def best_per_rank(records: np.ndarray):
    """Global 'best inlier' pick over all ranks: (rank, problem) with the most inliers among accepted."""
    n_inl = np.where(records["status"] == 0, records["n_inl"], -1)
    flat = int(np.argmax(n_inl))
    return divmod(flat, records.shape[1])
