"""Deterministic CVNN builder from a Pydantic config (reference ``src/spectralmc/cvnn_factory.py``).

``build_model`` constructs on the CPU inside ``torch.random.fork_rng()`` after
``torch.manual_seed(cfg.seed)`` and in the config's default dtype, so a given config
always yields the same weights and the caller's RNG stream is untouched
(reference cvnn_factory.py:343-367).  Modules are created in the reference's order —
it decides which uniform draws each ``xavier_uniform_`` consumes.
"""

from __future__ import annotations

from dataclasses import dataclass
from enum import Enum
from typing import Literal, TypeAlias

import torch
from pydantic import BaseModel, ConfigDict, PositiveInt, ValidationError

from .cvnn import (
    ComplexLinear,
    ComplexResidual,
    ComplexSequential,
    CovarianceComplexBatchNorm,
    NaiveComplexBatchNorm,
    modReLU,
    zReLU,
)
from .models.torch import AnyDType, Device, TensorState, default_device, default_dtype
from .result import Failure, Result, Success
from .validation import validate_model

nn = torch.nn


class ActivationKind(str, Enum):
    Z_RELU = "zReLU"
    MOD_RELU = "modReLU"


class LayerKind(str, Enum):
    LINEAR = "ComplexLinear"
    BN_NAIVE = "NaiveComplexBatchNorm"
    BN_COV = "CovarianceComplexBatchNorm"
    SEQ = "Sequential"
    RES = "Residual"


class WidthSpec(BaseModel):
    model_config = ConfigDict(frozen=True, extra="forbid")


class PreserveWidth(WidthSpec):
    model_config = ConfigDict(frozen=True, extra="forbid")


class ExplicitWidth(WidthSpec):
    value: PositiveInt
    model_config = ConfigDict(frozen=True, extra="forbid")


class ActivationCfg(BaseModel):
    kind: ActivationKind
    model_config = ConfigDict(frozen=True, extra="forbid")


class LinearCfg(BaseModel):
    kind: LayerKind = LayerKind.LINEAR
    width: WidthSpec = PreserveWidth()
    bias: bool = True
    activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


class NaiveBNCfg(BaseModel):
    kind: LayerKind = LayerKind.BN_NAIVE
    eps: float = 1e-5
    momentum: float = 0.1
    affine: bool = True
    track_running_stats: bool = True
    activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


class CovBNCfg(BaseModel):
    kind: LayerKind = LayerKind.BN_COV
    eps: float = 1e-5
    momentum: float = 0.1
    affine: bool = True
    track_running_stats: bool = True
    activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


class SequentialCfg(BaseModel):
    kind: LayerKind = LayerKind.SEQ
    layers: list["LayerCfg"]
    activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


class ResidualCfg(BaseModel):
    kind: LayerKind = LayerKind.RES
    body: SequentialCfg
    projection: LinearCfg | None = None
    activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


LayerCfg: TypeAlias = LinearCfg | NaiveBNCfg | CovBNCfg | SequentialCfg | ResidualCfg
SequentialCfg.model_rebuild()
ResidualCfg.model_rebuild()


class CVNNConfig(BaseModel):
    dtype: AnyDType
    layers: list[LayerCfg]
    seed: PositiveInt
    final_activation: ActivationCfg | None = None
    model_config = ConfigDict(frozen=True, extra="forbid")


def build_cvnn_config(*, dtype: AnyDType, layers: list[LayerCfg], seed: int,
                      final_activation: ActivationCfg | None = None) -> Result[CVNNConfig, ValidationError]:
    return validate_model(CVNNConfig, dtype=dtype, layers=layers, seed=seed, final_activation=final_activation)


@dataclass(frozen=True)
class ModelOnWrongDevice:
    device: str
    kind: Literal["ModelOnWrongDevice"] = "ModelOnWrongDevice"


@dataclass(frozen=True)
class SerializationDeviceMismatch:
    message: str
    kind: Literal["SerializationDeviceMismatch"] = "SerializationDeviceMismatch"


CVNNFactoryError = ModelOnWrongDevice | SerializationDeviceMismatch


# ----------------------------------------------------------------- construction
def _activation(kind: ActivationKind, width: int) -> nn.Module:
    return zReLU() if kind is ActivationKind.Z_RELU else modReLU(width)


def _chain(*mods: nn.Module) -> nn.Module:
    return mods[0] if len(mods) == 1 else ComplexSequential(*mods)


def _with_activation(mod: nn.Module, act: ActivationCfg | None, width: int) -> nn.Module:
    return _chain(mod, _activation(act.kind, width)) if act is not None else mod


def _build_layers(layers: list[LayerCfg], width: int) -> Result[tuple[list[nn.Module], int], CVNNFactoryError]:
    built: list[nn.Module] = []
    for layer in layers:
        res = _build(layer, width)
        if isinstance(res, Failure):
            return res
        mod, width = res.value
        built.append(mod)
    return Success((built, width))


def _build(cfg: LayerCfg, width: int) -> Result[tuple[nn.Module, int], CVNNFactoryError]:
    if isinstance(cfg, LinearCfg):
        out_w = cfg.width.value if isinstance(cfg.width, ExplicitWidth) else width
        lin = ComplexLinear(width, out_w, bias=cfg.bias)
        return Success((_with_activation(lin, cfg.activation, out_w), out_w))
    if isinstance(cfg, (NaiveBNCfg, CovBNCfg)):
        cls = NaiveComplexBatchNorm if isinstance(cfg, NaiveBNCfg) else CovarianceComplexBatchNorm
        bn = cls(width, eps=cfg.eps, momentum=cfg.momentum, affine=cfg.affine,
                 track_running_stats=cfg.track_running_stats)
        return Success((_with_activation(bn, cfg.activation, width), width))
    if isinstance(cfg, SequentialCfg):
        res = _build_layers(cfg.layers, width)
        if isinstance(res, Failure):
            return res
        mods, out_w = res.value
        return Success((_with_activation(_chain(*mods), cfg.activation, out_w), out_w))
    if isinstance(cfg, ResidualCfg):
        body = _build(cfg.body, width)
        if isinstance(body, Failure):
            return body
        body_mod, body_w = body.value
        if cfg.projection is None:
            proj, proj_w = (None, body_w) if body_w == width else (ComplexLinear(width, body_w), body_w)
        else:
            pres = _build(cfg.projection, width)
            if isinstance(pres, Failure):
                return pres
            proj, proj_w = pres.value
        if proj_w != body_w:
            return Failure(SerializationDeviceMismatch(
                message=f"Residual projection width {proj_w} does not match body width {body_w}."))
        post = _activation(cfg.activation.kind, body_w) if cfg.activation is not None else None
        return Success((ComplexResidual(body=body_mod, proj=proj, post_act=post), body_w))
    raise AssertionError(f"unknown layer config {type(cfg).__name__}")


def build_model(*, n_inputs: int, n_outputs: int, cfg: CVNNConfig) -> Result[nn.Module, CVNNFactoryError]:
    """Seeded CPU build; the caller's RNG state (CPU and GPU) is restored on exit."""
    with torch.random.fork_rng(), default_device(Device.cpu.to_torch()), default_dtype(cfg.dtype.to_torch()):
        torch.manual_seed(cfg.seed)
        res = _build_layers(cfg.layers, n_inputs)
        if isinstance(res, Failure):
            return res
        mods, width = res.value
        body = _chain(*mods)
        if width != n_outputs:
            body, width = _chain(body, ComplexLinear(width, n_outputs)), n_outputs
        return Success(_with_activation(body, cfg.final_activation, width))


def load_model(*, model: nn.Module, tensors: dict[str, TensorState]) -> Result[nn.Module, object]:
    off = next((p for p in model.parameters() if p.device.type != "cpu"), None)
    if off is not None:
        return Failure(ModelOnWrongDevice(device=str(off.device)))
    state: dict[str, torch.Tensor] = {}
    for name, ts in tensors.items():
        t = ts.to_torch()
        if isinstance(t, Failure):
            return t
        state[name] = t.value
    model.load_state_dict(state, assign=True)
    return Success(model)


def get_safetensors(model: nn.Module) -> Result[dict[str, TensorState], object]:
    off = next((p for p in model.parameters() if p.device.type != "cpu"), None)
    if off is not None:
        return Failure(ModelOnWrongDevice(device=str(off.device)))
    out: dict[str, TensorState] = {}
    for name, t in model.state_dict().items():
        ts = TensorState.from_torch(t)
        if isinstance(ts, Failure):
            return ts
        out[name] = ts.value
    return Success(out)


__all__ = ("ActivationKind", "LayerKind", "WidthSpec", "PreserveWidth", "ExplicitWidth", "ActivationCfg",
           "LinearCfg", "NaiveBNCfg", "CovBNCfg", "SequentialCfg", "ResidualCfg", "LayerCfg", "CVNNConfig",
           "build_cvnn_config", "build_model", "load_model", "get_safetensors")
