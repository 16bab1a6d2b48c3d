"""Multi-GPU: one process per GPU, independent replicas.

The path does not exchange data per token: images are sharded across ranks and every rank
runs its own full replica.  The only collective is the load-time broadcast of the packed
bf16 weight slab from rank 0 (RCCL over xGMI with the "nccl" backend on ROCm; gloo on CPU in
the tests).  Collection of generated ids is an all-gather of a few KB at the end.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int) -> "tuple[int, int]":
    """Contiguous block of items [lo, hi) for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n_items, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def broadcast_slab(slab: torch.Tensor, src: int = 0) -> None:
    """Weights generated/loaded on `src` -> every rank (one collective, whole slab)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(slab, src=src)


def gather_tokens(tokens: torch.Tensor) -> torch.Tensor:
    """All ranks' (B_rank, T) generated ids -> (sum B_rank, T) on every rank (equal B per rank)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return tokens
    out = [torch.empty_like(tokens) for _ in range(dist.get_world_size())]
    dist.all_gather(out, tokens)
    return torch.cat(out, 0)
