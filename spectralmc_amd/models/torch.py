"""torch-facing dtype/device enums, tensor snapshots and Adam state
(reference ``src/spectralmc/models/torch.py``).

``AdamOptimizerState`` round-trips a ``torch.optim.Adam.state_dict()`` through CPU
SafeTensor blobs so snapshots carry no device artefacts (reference 579-735).
"""

from __future__ import annotations

import threading
from contextlib import contextmanager
from enum import Enum
from types import MappingProxyType
from typing import Iterable, Iterator, Mapping, Sequence

import torch
from pydantic import BaseModel, ConfigDict, ValidationError, field_serializer, model_validator
from safetensors.torch import load as _st_load
from safetensors.torch import save as _st_save

from ..errors.numerical import (
    InvalidAdamState,
    TensorStateConversionFailed,
    TorchFacadeError,
    UnsupportedTorchDevice,
    UnsupportedTorchDType,
)
from ..result import Failure, Result, Success
from ..validation import validate_model
from .numerical import Precision

_TORCH_BY_NAME: dict[str, torch.dtype] = {
    "float16": torch.float16,
    "bfloat16": torch.bfloat16,
    "float32": torch.float32,
    "float64": torch.float64,
    "complex64": torch.complex64,
    "complex128": torch.complex128,
}
_NAME_BY_TORCH = {v: k for k, v in _TORCH_BY_NAME.items()}
_FULL = ("float32", "float64", "complex64", "complex128")


class FullPrecisionDType(str, Enum):
    """Formats that have a simulation ``Precision`` counterpart."""

    float32 = "float32"
    float64 = "float64"
    complex64 = "complex64"
    complex128 = "complex128"

    def to_torch(self) -> torch.dtype:
        return _TORCH_BY_NAME[self.value]

    @classmethod
    def from_torch(cls, dt: torch.dtype) -> Result["FullPrecisionDType", UnsupportedTorchDType]:
        name = _NAME_BY_TORCH.get(dt)
        if name not in _FULL:
            return Failure(UnsupportedTorchDType(dtype_repr=str(dt)))
        return Success(cls(name))

    def to_precision(self) -> Precision:
        return Precision(self.value)

    @classmethod
    def from_precision(cls, p: Precision) -> "FullPrecisionDType":
        return cls(p.value)


class ReducedPrecisionDType(str, Enum):
    """Storage / mixed-precision formats without a simulation counterpart."""

    float16 = "float16"
    bfloat16 = "bfloat16"

    def to_torch(self) -> torch.dtype:
        return _TORCH_BY_NAME[self.value]

    @classmethod
    def from_torch(cls, dt: torch.dtype) -> Result["ReducedPrecisionDType", UnsupportedTorchDType]:
        name = _NAME_BY_TORCH.get(dt)
        if name not in ("float16", "bfloat16"):
            return Failure(UnsupportedTorchDType(dtype_repr=str(dt)))
        return Success(cls(name))


AnyDType = FullPrecisionDType | ReducedPrecisionDType


def any_dtype_from_torch(dt: torch.dtype) -> Result[AnyDType, UnsupportedTorchDType]:
    name = _NAME_BY_TORCH.get(dt)
    if name is None:
        return Failure(UnsupportedTorchDType(dtype_repr=str(dt)))
    return Success(FullPrecisionDType(name) if name in _FULL else ReducedPrecisionDType(name))


class Device(str, Enum):
    """``cuda`` is the process's GPU (reference ``models/torch.py:158-175``: the single-GPU policy
    "cuda:0").  One process per GPU: a rank bound with ``torch.cuda.set_device(LOCAL_RANK)``
    (spectralmc_amd/dp.py) maps ``cuda`` to ITS device, so tensors a rank reloads (storage/wire.py)
    land on its own GPU, not on rank 0's."""

    cpu = "cpu"
    cuda = "cuda:0"

    def to_torch(self) -> torch.device:
        if self is Device.cuda and torch.cuda.is_available():
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device(self.value)

    @classmethod
    def from_torch(cls, dev: torch.device) -> Result["Device", UnsupportedTorchDevice]:
        if dev.type == "cpu":
            return Success(cls.cpu)
        if dev.type == "cuda" and dev.index in (None, 0):
            return Success(cls.cuda)
        if dev.type == "cuda" and torch.cuda.is_available() and dev.index == torch.cuda.current_device():
            return Success(cls.cuda)  # rank-bound device of a multi-GPU node
        return Failure(UnsupportedTorchDevice(device_repr=str(dev)))


def _require_main_thread(what: str) -> None:
    if threading.current_thread() is not threading.main_thread():
        raise RuntimeError(f"{what} may only be used from the main thread")


@contextmanager
def default_dtype(dt: torch.dtype) -> Iterator[None]:
    _require_main_thread("default_dtype")
    saved = torch.get_default_dtype()
    torch.set_default_dtype(dt)
    try:
        yield
    finally:
        torch.set_default_dtype(saved)


def _default_device_setting() -> torch.device | None:
    """The device torch.set_default_device last installed, or None when no default-device mode is active.
    (torch.tensor([]).device reads "cpu" either way, and restoring "cpu" would leave a DeviceContext
    torch-function mode active that intercepts every later torch call: 2.5x slower tensor methods, measured.)"""
    ctx = getattr(getattr(torch, "_GLOBAL_DEVICE_CONTEXT", None), "device_context", None)
    return getattr(ctx, "device", None) if ctx is not None else None


@contextmanager
def default_device(dev: torch.device) -> Iterator[None]:
    _require_main_thread("default_device")
    saved = _default_device_setting()
    torch.set_default_device(dev)
    try:
        yield
    finally:
        torch.set_default_device(saved)


class TensorState(BaseModel):
    """CPU tensor frozen as a single-entry SafeTensor blob."""

    data: bytes
    shape: tuple[int, ...]
    dtype: FullPrecisionDType | ReducedPrecisionDType

    model_config = ConfigDict(extra="forbid")

    @staticmethod
    def from_torch(t: torch.Tensor) -> Result["TensorState", TensorStateConversionFailed]:
        if t.device.type != "cpu":
            return Failure(TensorStateConversionFailed(message="TensorState needs a CPU tensor"))
        dt = any_dtype_from_torch(t.dtype)
        if isinstance(dt, Failure):
            return Failure(TensorStateConversionFailed(message=f"unsupported dtype {t.dtype}"))
        blob = _st_save({"tensor": t.contiguous()})
        res = validate_model(TensorState, data=blob, shape=tuple(t.shape), dtype=dt.value)
        if isinstance(res, Failure):
            return Failure(TensorStateConversionFailed(message=str(res.error)))
        return res

    def to_torch(self) -> Result[torch.Tensor, TensorStateConversionFailed]:
        loaded = _st_load(self.data)
        t = loaded.get("tensor")
        if t is None:
            return Failure(TensorStateConversionFailed(message="blob has no 'tensor' entry"))
        if tuple(t.shape) != self.shape or t.dtype != self.dtype.to_torch():
            return Failure(TensorStateConversionFailed(message="tensor metadata mismatch"))
        return Success(t)

    @staticmethod
    def from_bytes(raw: bytes) -> Result["TensorState", TensorStateConversionFailed]:
        loaded = _st_load(raw)
        if set(loaded) != {"tensor"}:
            return Failure(TensorStateConversionFailed(message="blob must hold exactly one 'tensor'"))
        t = loaded["tensor"]
        dt = any_dtype_from_torch(t.dtype)
        if isinstance(dt, Failure):
            return Failure(TensorStateConversionFailed(message=f"unsupported dtype {t.dtype}"))
        return Success(TensorState(data=raw, shape=tuple(t.shape), dtype=dt.value))


class AdamParamState(BaseModel):
    step: int
    exp_avg: TensorState
    exp_avg_sq: TensorState
    max_exp_avg_sq: TensorState | None = None

    model_config = ConfigDict(extra="forbid")

    @classmethod
    def from_torch(cls, s: Mapping[str, object]) -> Result["AdamParamState", TorchFacadeError]:
        unknown = set(s) - {"step", "exp_avg", "exp_avg_sq", "max_exp_avg_sq"}
        if unknown:
            return Failure(InvalidAdamState(message=f"unexpected Adam state keys {sorted(unknown)}"))
        step = s.get("step")
        if isinstance(step, torch.Tensor):
            if step.ndim != 0 or step.device.type != "cpu":
                return Failure(InvalidAdamState(message="Adam 'step' must be a CPU scalar tensor"))
            step_i = int(step.item())
        elif isinstance(step, int):
            step_i = step
        else:
            return Failure(InvalidAdamState(message="Adam 'step' must be an int or a scalar tensor"))
        blobs: dict[str, TensorState | None] = {}
        for name in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
            t = s.get(name)
            if t is None and name == "max_exp_avg_sq":
                blobs[name] = None
                continue
            if not isinstance(t, torch.Tensor):
                return Failure(InvalidAdamState(message=f"Adam '{name}' must be a tensor"))
            if t.device.type != "cpu":
                return Failure(InvalidAdamState(message="Adam state tensors must be on the CPU"))
            ts = TensorState.from_torch(t)
            if isinstance(ts, Failure):
                return ts
            blobs[name] = ts.value
        return Success(cls(step=step_i, exp_avg=blobs["exp_avg"], exp_avg_sq=blobs["exp_avg_sq"],
                           max_exp_avg_sq=blobs["max_exp_avg_sq"]))

    def to_torch(self) -> Result[dict[str, object], TorchFacadeError]:
        out: dict[str, object] = {"step": self.step}
        for name in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
            ts = getattr(self, name)
            if ts is None:
                continue
            t = ts.to_torch()
            if isinstance(t, Failure):
                return t
            out[name] = t.value
        return Success(out)


class AdamParamGroup(BaseModel):
    params: list[int]
    lr: float
    betas: tuple[float, float]
    eps: float
    weight_decay: float
    amsgrad: bool = False
    maximize: bool = False
    foreach: bool | None = None
    capturable: bool = False
    differentiable: bool = False
    fused: bool | None = None
    decoupled_weight_decay: bool = False

    model_config = ConfigDict(extra="forbid")

    @classmethod
    def from_torch(cls, g: Mapping[str, object]) -> Result["AdamParamGroup", InvalidAdamState]:
        res = build_adam_param_group(g)
        if isinstance(res, Failure):
            return Failure(InvalidAdamState(message=f"invalid Adam param group: {res.error}"))
        return res

    def to_torch(self) -> dict[str, object]:
        return self.model_dump(mode="python")


def build_adam_param_group(data: Mapping[str, object]) -> Result[AdamParamGroup, ValidationError]:
    try:
        return Success(AdamParamGroup.model_validate(dict(data)))
    except ValidationError as exc:
        return Failure(exc)


class AdamOptimizerState(BaseModel):
    """Frozen, device-free image of an Adam ``state_dict``."""

    param_states: Mapping[int, AdamParamState]
    param_groups: tuple[AdamParamGroup, ...]

    model_config = ConfigDict(extra="forbid", arbitrary_types_allowed=True, frozen=True)

    @model_validator(mode="after")
    def _freeze(self) -> "AdamOptimizerState":
        if not isinstance(self.param_states, MappingProxyType):
            object.__setattr__(self, "param_states", MappingProxyType(dict(self.param_states)))
        if not isinstance(self.param_groups, tuple):
            object.__setattr__(self, "param_groups", tuple(self.param_groups))
        return self

    @field_serializer("param_states", when_used="always")
    def _dump_states(self, value: Mapping[int, AdamParamState]) -> dict[int, AdamParamState]:
        return dict(value)

    @classmethod
    def from_torch(cls, sd: Mapping[str, object]) -> Result["AdamOptimizerState", TorchFacadeError]:
        if set(sd) != {"state", "param_groups"}:
            return Failure(InvalidAdamState(message="state_dict needs exactly 'state' and 'param_groups'"))
        states = sd["state"]
        groups = sd["param_groups"]
        if not isinstance(states, Mapping) or not isinstance(groups, Iterable):
            return Failure(InvalidAdamState(message="malformed optimizer state_dict"))
        param_states: dict[int, AdamParamState] = {}
        for pid, st in states.items():
            res = AdamParamState.from_torch(st)
            if isinstance(res, Failure):
                return res
            param_states[int(pid)] = res.value
        param_groups: list[AdamParamGroup] = []
        for g in groups:
            res_g = AdamParamGroup.from_torch(g)
            if isinstance(res_g, Failure):
                return res_g
            param_groups.append(res_g.value)
        built = build_adam_optimizer_state(param_states, param_groups)
        if isinstance(built, Failure):
            return Failure(InvalidAdamState(message=f"invalid AdamOptimizerState: {built.error}"))
        return built

    def to_torch(self) -> Result[Mapping[str, object], TorchFacadeError]:
        state: dict[int, dict[str, object]] = {}
        for pid, ps in self.param_states.items():
            res = ps.to_torch()
            if isinstance(res, Failure):
                return res
            state[pid] = res.value
        return Success({"state": state, "param_groups": [g.to_torch() for g in self.param_groups]})


def build_adam_optimizer_state(
    param_states: Mapping[int, AdamParamState], param_groups: Sequence[AdamParamGroup]
) -> Result[AdamOptimizerState, ValidationError]:
    try:
        return Success(AdamOptimizerState.model_validate({"param_states": dict(param_states),
                                                          "param_groups": list(param_groups)}))
    except ValidationError as exc:
        return Failure(exc)


__all__ = (
    "FullPrecisionDType",
    "ReducedPrecisionDType",
    "AnyDType",
    "Device",
    "TensorState",
    "AdamParamState",
    "AdamParamGroup",
    "AdamOptimizerState",
    "build_adam_optimizer_state",
    "build_adam_param_group",
    "default_dtype",
    "default_device",
)
