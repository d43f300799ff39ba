"""Data-parallel training over RCCL: one process per GPU, contracts sharded, one all-reduce.

The reference is single-GPU (``models/torch.py:158-175``).  Contracts are independent, so the
step shards by contract: rank r of W draws the r-th slice of every step's W*B global batch
(engine.py) and the only exchange is the mean of the flat [gradients..., loss] buffer,
one ``all_reduce`` per step (backend "nccl" is RCCL on ROCm; "gloo" on CPU for tests).
Ring all-reduce delivers identical bits to every rank, so replicas stay bit-identical.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class DataParallel:
    world_size: int
    rank: int
    group: object | None = None

    def all_reduce_mean(self, flat: torch.Tensor) -> None:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        flat.div_(self.world_size)

    def shard(self, global_index0: int, local_batch: int) -> tuple[int, int]:
        """[start, stop) of this rank's contracts within a global batch starting at global_index0."""
        start = global_index0 + self.rank * local_batch
        return start, start + local_batch


def current() -> DataParallel | None:
    """The active data-parallel context, or None for a single-process run."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    world = dist.get_world_size()
    if world <= 1:
        return None
    return DataParallel(world_size=world, rank=dist.get_rank())


def init_from_env(backend: str | None = None) -> DataParallel | None:
    """torchrun-style initialisation (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*); binds the GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
    if not dist.is_initialized():
        kwargs = {"device_id": torch.device("cuda", local_rank)} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, **kwargs)
    return current()


__all__ = ["DataParallel", "current", "init_from_env"]
