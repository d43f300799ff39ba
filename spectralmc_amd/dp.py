"""Data-parallel training over RCCL: one process per GPU, contracts sharded, one all-reduce.

The reference is single-GPU (``models/torch.py:158-175``).  Contracts are independent, so the
step shards by contract: rank r of W draws the r-th slice of every step's W*B global batch
(engine.py) and the only exchange is the mean of the flat [gradients..., loss] buffer,
one all-reduce per step.  Ring all-reduce delivers identical bits to every rank, so replicas
stay bit-identical.

With backend "nccl" (= RCCL on ROCm) the all-reduce is issued on the CALLER's stream through a
communicator of this module's own (``RcclComm``: librccl's ``ncclAllReduce`` with an explicit
``hipStream_t``), not on torch's internal collective stream: the training step calls it on its
network stream, which is CU-masked, so RCCL's kernels run on the network's CUs and never take a CU
a persistent path launch needs.  "gloo" (CPU tests, one-GPU rehearsals) keeps
``torch.distributed.all_reduce``.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

_NCCL_FLOAT32, _NCCL_FLOAT64, _NCCL_SUM = 7, 8, 0  # ncclDataType_t / ncclRedOp_t (rccl.h)


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


def _librccl() -> ctypes.CDLL:
    """The RCCL torch itself loaded (torch/lib/librccl.so), else the ROCm one."""
    here = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    lib = ctypes.CDLL(here if os.path.exists(here) else "librccl.so")
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
    lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    return lib


class RcclComm:
    """An RCCL communicator over the default process group's ranks (its unique id broadcast through that
    group), whose all-reduce runs on an explicit HIP stream."""

    def __init__(self, rank: int, world: int) -> None:
        self.lib = _librccl()
        uid = _UniqueId()
        box: list[object] = [None]
        if rank == 0:
            rc = self.lib.ncclGetUniqueId(ctypes.byref(uid))
            # the raw 128 bytes (uid.internal would stop at the first NUL byte), or the failure for every rank
            box = [ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid)) if rc == 0 else
                   f"ncclGetUniqueId: {self.lib.ncclGetErrorString(rc).decode()} ({rc})"]
        dist.broadcast_object_list(box, src=0)  # every rank takes part, so a failure on rank 0 raises everywhere
        if isinstance(box[0], str):
            raise RuntimeError(box[0])
        uid = _UniqueId.from_buffer_copy(box[0])
        self.comm = ctypes.c_void_p()
        self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank), "ncclCommInitRank")
        self.world = world

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.ncclGetErrorString(rc).decode()} ({rc})")

    def all_reduce_sum(self, t: torch.Tensor, stream: int) -> None:
        if t.dtype not in (torch.float32, torch.float64) or not t.is_contiguous():
            raise ValueError("RcclComm.all_reduce_sum takes a contiguous f32 / f64 tensor")
        dtype = _NCCL_FLOAT32 if t.dtype == torch.float32 else _NCCL_FLOAT64
        self._check(self.lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype, _NCCL_SUM, self.comm,
                                           ctypes.c_void_p(stream)), "ncclAllReduce")

    def destroy(self) -> None:
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


_COMM: RcclComm | None = None  # this process's communicator (created once per process group)


@dataclass(frozen=True)
class DataParallel:
    world_size: int
    rank: int
    group: object | None = None
    comm: RcclComm | None = None

    def all_reduce_mean(self, flat: torch.Tensor) -> None:
        """Mean over the ranks, in place, on the current stream (RcclComm), or through torch.distributed."""
        if self.comm is not None:
            self.comm.all_reduce_sum(flat, torch.cuda.current_stream(flat.device).cuda_stream)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        flat.div_(self.world_size)

    def shard(self, global_index0: int, local_batch: int) -> tuple[int, int]:
        """[start, stop) of this rank's contracts within a global batch starting at global_index0."""
        start = global_index0 + self.rank * local_batch
        return start, start + local_batch


def _own_comm_wanted() -> bool:
    """The collective on the caller's stream (RcclComm) for the nccl backend; SMC_RCCL_OWN_COMM=0 keeps
    torch.distributed's all_reduce on its internal stream."""
    return dist.get_backend() == "nccl" and os.environ.get("SMC_RCCL_OWN_COMM", "1") != "0"


def current() -> DataParallel | None:
    """The active data-parallel context, or None for a single-process run."""
    global _COMM
    if not (dist.is_available() and dist.is_initialized()):
        return None
    world = dist.get_world_size()
    if world <= 1:
        return None
    rank = dist.get_rank()
    if _COMM is None and _own_comm_wanted():
        _COMM = RcclComm(rank, world)
    return DataParallel(world_size=world, rank=rank, comm=_COMM)


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


def shutdown() -> None:
    """Destroy this module's communicator (before torch.distributed.destroy_process_group)."""
    global _COMM
    if _COMM is not None:
        _COMM.destroy()
        _COMM = None


__all__ = ["DataParallel", "RcclComm", "current", "init_from_env", "shutdown"]
