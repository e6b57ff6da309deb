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

    `local_bytes` is a torch uint8 tensor (device tensor with the nccl backend, CPU with gloo)."""
    import torch
    import torch.distributed as dist

    n = local_bytes.numel()
    flat = torch.empty(world * n, dtype=torch.uint8, device=local_bytes.device)
    if world == 1:
        flat.copy_(local_bytes)
    else:
        dist.all_gather_into_tensor(flat, local_bytes, group=group)
    return flat.view(world, n)


def decode(gathered) -> np.ndarray:
    arr = gathered.cpu().numpy()
    return arr.reshape(arr.shape[0], -1).view(RESULT_DTYPE)


def best_per_rank(records: np.ndarray):
    """Global 'best inlier' pick over all ranks: (rank, problem) with the most inliers among accepted."""
    n_inl = np.where(records["status"] == 0, records["n_inl"], -1)
    flat = int(np.argmax(n_inl))
    return divmod(flat, records.shape[1])
