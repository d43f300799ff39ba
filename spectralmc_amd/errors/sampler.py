"""Sampler errors (reference ``src/spectralmc/errors/sampler.py``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

from pydantic import ValidationError


@dataclass(frozen=True)
class DimensionMismatch:
    kind: Literal["DimensionMismatch"] = "DimensionMismatch"
    expected_fields: tuple[str, ...] = ()
    provided_fields: tuple[str, ...] = ()


@dataclass(frozen=True)
class InvalidBounds:
    message: str
    kind: Literal["InvalidBounds"] = "InvalidBounds"


@dataclass(frozen=True)
class NegativeSamples:
    n_samples: int
    kind: Literal["NegativeSamples"] = "NegativeSamples"


@dataclass(frozen=True)
class BoundSpecInvalid:
    lower: float
    upper: float
    kind: Literal["BoundSpecInvalid"] = "BoundSpecInvalid"


@dataclass(frozen=True)
class SamplerValidationFailed:
    error: ValidationError | str
    kind: Literal["SamplerValidationFailed"] = "SamplerValidationFailed"


@dataclass(frozen=True)
class SequenceExhausted:
    """Sobol index would pass 2^30 points (SciPy raises ValueError there)."""

    requested_end: int
    kind: Literal["SequenceExhausted"] = "SequenceExhausted"


SamplerError = DimensionMismatch | InvalidBounds | NegativeSamples | SamplerValidationFailed | SequenceExhausted
