"""Precision conversion errors (reference ``src/spectralmc/errors/numerical.py``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal


@dataclass(frozen=True)
class UnsupportedNumPyDType:
    dtype_repr: str
    kind: Literal["UnsupportedNumPyDType"] = "UnsupportedNumPyDType"


@dataclass(frozen=True)
class InvalidComplexConversion:
    precision: str
    kind: Literal["InvalidComplexConversion"] = "InvalidComplexConversion"


@dataclass(frozen=True)
class UnsupportedTorchDType:
    dtype_repr: str
    kind: Literal["UnsupportedTorchDType"] = "UnsupportedTorchDType"


@dataclass(frozen=True)
class UnsupportedTorchDevice:
    device_repr: str
    kind: Literal["UnsupportedTorchDevice"] = "UnsupportedTorchDevice"


@dataclass(frozen=True)
class TensorStateConversionFailed:
    message: str
    kind: Literal["TensorStateConversionFailed"] = "TensorStateConversionFailed"


@dataclass(frozen=True)
class InvalidAdamState:
    message: str
    kind: Literal["InvalidAdamState"] = "InvalidAdamState"


TorchFacadeError = (
    UnsupportedTorchDType | UnsupportedTorchDevice | TensorStateConversionFailed | InvalidAdamState
)
