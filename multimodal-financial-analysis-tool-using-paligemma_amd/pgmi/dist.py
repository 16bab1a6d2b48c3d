"""Multi-GPU: one process per GPU, independent replicas.

The path does not exchange data per token: images are sharded across ranks and every rank
runs its own full replica.  The only collective is the load-time broadcast of the packed
bf16 weight slab from rank 0.  On GPUs it goes through libpgmi's C ABI
(pgmi_comm_init + pgmi_broadcast_weights: one in-place RCCL ncclBroadcast over xGMI), so a
non-Python host can do the same step; torch.distributed only carries the 128-byte RCCL id.  On
CPU (gloo, the tests) the slab is broadcast with torch.distributed.  Collection of generated
ids is an all-gather of a few KB at the end.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int) -> "tuple[int, int]":
    """Contiguous block of items [lo, hi) for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n_items, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_slab(slab: torch.Tensor, src: int = 0) -> None:
    """Weights generated/loaded on `src` -> every rank (one torch.distributed collective)."""
    if _world() > 1:
        dist.broadcast(slab, src=src)


def exchange_comm_id(device: torch.device, src: int = 0) -> bytes:
    """Rank `src` creates the RCCL unique id (pgmi_comm_unique_id, no GPU needed); the 128 bytes
    travel to every rank over the torch.distributed group (on the device for nccl, on the host for
    gloo).  Every rank returns the same bytes."""
    from . import _native as N
    lib = N.lib()
    uid = torch.zeros(128, dtype=torch.uint8)
    if dist.get_rank() == src:
        buf = (ctypes.c_uint8 * 128)()
        N.check(lib.pgmi_comm_unique_id(buf), "pgmi_comm_unique_id")
        uid = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
    t = uid.to(device) if dist.get_backend() == "nccl" else uid
    dist.broadcast(t, src=src)
    return bytes(t.cpu().tolist())


class WeightComm:
    """An RCCL communicator owned by libpgmi (pgmi_comm_init), one per process / GPU."""

    def __init__(self, device: torch.device, src: int = 0):
        from . import _native as N
        self.N, self.lib = N, N.lib()
        rank, world = dist.get_rank(), dist.get_world_size()
        # only the 128-byte id travels over torch.distributed
        raw = (ctypes.c_uint8 * 128)(*exchange_comm_id(device, src))
        h = ctypes.c_void_p()
        N.check(self.lib.pgmi_comm_init(device.index, world, rank, raw, ctypes.byref(h)), "pgmi_comm_init")
        self.comm = h

    def broadcast_weights(self, engine, src: int = 0) -> None:
        self.N.check(self.lib.pgmi_broadcast_weights(engine.ctx, self.comm, src, engine._s()), "pgmi_broadcast_weights")
        engine.prepared = False

    def close(self) -> None:
        if self.comm:
            self.N.check(self.lib.pgmi_comm_destroy(self.comm), "pgmi_comm_destroy")
            self.comm = None


def broadcast_weights(engine, src: int = 0, comm: "WeightComm | None" = None) -> "WeightComm | None":
    """Engine weights on `src` -> every rank's engine.  GPU ranks: libpgmi's RCCL broadcast
    (returns the communicator, reusable for later reloads); CPU/gloo: torch.distributed."""
    if _world() <= 1:
        return comm
    if engine.device.type == "cuda" and dist.get_backend() == "nccl":
        comm = comm or WeightComm(engine.device, src)
        comm.broadcast_weights(engine, src)
        return comm
    broadcast_slab(engine.slab, src)
    engine.prepared = False
    return comm


def gather_tokens(tokens: torch.Tensor) -> torch.Tensor:
    """All ranks' (B_rank, T) generated ids -> (sum B_rank, T) on every rank (equal B per rank)."""
    if _world() == 1:
        return tokens
    out = [torch.empty_like(tokens) for _ in range(dist.get_world_size())]
    dist.all_gather(out, tokens)
    return torch.cat(out, 0)
