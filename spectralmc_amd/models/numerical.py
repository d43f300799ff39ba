"""Scalar formats of the engine (reference ``src/spectralmc/models/numerical.py``).

The reference maps each format to NumPy and CuPy dtypes; this build has no CuPy, so
``to_cupy`` is absent and ``to_torch`` is offered instead (device arrays are torch tensors).
"""

from __future__ import annotations

from enum import Enum

import numpy as np

from ..errors.numerical import InvalidComplexConversion, UnsupportedNumPyDType
from ..result import Failure, Result, Success

_NAMES = ("float32", "float64", "complex64", "complex128")
_TO_COMPLEX = {"float32": "complex64", "float64": "complex128"}
_TO_REAL = {v: k for k, v in _TO_COMPLEX.items()}


class Precision(str, Enum):
    float32 = "float32"
    float64 = "float64"
    complex64 = "complex64"
    complex128 = "complex128"

    def to_numpy(self) -> np.dtype:
        return np.dtype(self.value)

    @classmethod
    def from_numpy(cls, dtype: object) -> Result["Precision", UnsupportedNumPyDType]:
        try:
            name = np.dtype(dtype).name  # accepts scalar classes and dtype objects
        except TypeError:
            return Failure(UnsupportedNumPyDType(dtype_repr=repr(dtype)))
        if name not in _NAMES:
            return Failure(UnsupportedNumPyDType(dtype_repr=repr(dtype)))
        return Success(cls(name))

    def to_torch(self):  # noqa: ANN201 - torch imported lazily
        import torch

        return getattr(torch, self.value)

    def to_complex(self) -> Result["Precision", InvalidComplexConversion]:
        if self.value in _TO_COMPLEX:
            return Success(Precision(_TO_COMPLEX[self.value]))
        return Failure(InvalidComplexConversion(precision=self.value))

    @classmethod
    def from_complex(cls, p: "Precision") -> Result["Precision", InvalidComplexConversion]:
        if p.value in _TO_REAL:
            return Success(cls(_TO_REAL[p.value]))
        return Failure(InvalidComplexConversion(precision=p.value))

    @property
    def is_complex(self) -> bool:
        return self.value.startswith("complex")


__all__ = ["Precision"]
