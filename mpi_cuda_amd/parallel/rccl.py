"""Bootstrap of the native RCCL communicator from torch.distributed.

One process per GPU is launched by torchrun (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the env).
torch.distributed (gloo, CPU-only, so no second RCCL communicator is created by torch) carries the 128-byte
ncclUniqueId from rank 0 to the others; the C++ runtime then owns the RCCL communicator and drives every halo
exchange itself (csrc/src/solver_gpu.cpp). This replaces the reference's MPI_Init/Comm_rank/Comm_size
(SURVEY.md §2.6 M5, §5.8).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .._native import load


def env_rank_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_process_group(backend: str = "gloo", timeout_s: float = 600.0) -> tuple[int, int, int]:
    """Initialise torch.distributed from the torchrun env (idempotent). Returns (rank, world, local_rank)."""
    import datetime

    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return rank, world, local


def broadcast_bytes(data: bytes | None, src: int = 0, group=None) -> bytes:
    """Broadcast a short byte string from ``src`` over torch.distributed (CPU tensors)."""
    rank = dist.get_rank()
    n = torch.tensor([len(data) if rank == src else 0], dtype=torch.int64)
    dist.broadcast(n, src, group=group)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    dist.broadcast(buf, src, group=group)
    return bytes(buf.numpy().tobytes())


def make_comm(rank: int, world: int, group=None):
    """Create the native RCCL communicator (None for world == 1). torch.distributed must be initialised."""
    if world <= 1:
        return None
    C = load()
    uid = C.Comm.make_unique_id() if rank == 0 else None
    uid = broadcast_bytes(uid, 0, group)
    return C.Comm(rank, world, uid)
