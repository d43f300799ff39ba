"""Device/dtype inference for model and optimiser state
(reference ``src/spectralmc/models/cpu_gpu_transfer.py:480-526``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal, Mapping

import torch

from ..errors.numerical import TorchFacadeError
from ..result import Failure, Result, Success
from .torch import AnyDType, Device, any_dtype_from_torch


@dataclass(frozen=True)
class EmptyTensorTree:
    kind: Literal["EmptyTensorTree"] = "EmptyTensorTree"


@dataclass(frozen=True)
class HeterogeneousTensorTree:
    pairs: tuple[str, ...]
    kind: Literal["HeterogeneousTensorTree"] = "HeterogeneousTensorTree"


def get_tree_device_dtype(tensors: tuple[torch.Tensor, ...]) -> Result[tuple[Device, AnyDType], object]:
    if not tensors:
        return Failure(EmptyTensorTree())
    pairs = {(t.device, t.dtype) for t in tensors}
    if len(pairs) != 1:
        return Failure(HeterogeneousTensorTree(pairs=tuple(sorted(f"{d}/{t}" for d, t in pairs))))
    dev, dt = next(iter(pairs))
    dtype = any_dtype_from_torch(dt)
    if isinstance(dtype, Failure):
        return dtype
    device = Device.from_torch(dev)
    if isinstance(device, Failure):
        return device
    return Success((device.value, dtype.value))


def module_state_device_dtype(state: Mapping[str, torch.Tensor]) -> Result[tuple[Device, AnyDType], TorchFacadeError]:
    return get_tree_device_dtype(tuple(state.values()))


__all__ = ["module_state_device_dtype", "get_tree_device_dtype", "EmptyTensorTree", "HeterogeneousTensorTree"]
