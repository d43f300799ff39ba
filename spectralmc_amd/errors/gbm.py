"""GBM engine errors (reference ``src/spectralmc/errors/gbm.py``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

from pydantic import ValidationError

from .async_normals import NormGeneratorError


@dataclass(frozen=True)
class CudaRNGUnavailable:
    reason: str
    kind: Literal["CudaRNGUnavailable"] = "CudaRNGUnavailable"


@dataclass(frozen=True)
class InvalidSimulationParams:
    error: ValidationError
    kind: Literal["InvalidSimulationParams"] = "InvalidSimulationParams"


@dataclass(frozen=True)
class GPUMemoryLimitExceeded:
    total_paths: int
    max_paths: int
    network_size: int
    batches_per_mc_run: int
    kind: Literal["GPUMemoryLimitExceeded"] = "GPUMemoryLimitExceeded"


@dataclass(frozen=True)
class InvalidBlackScholesConfig:
    error: ValidationError
    kind: Literal["InvalidBlackScholesConfig"] = "InvalidBlackScholesConfig"


@dataclass(frozen=True)
class NormalsUnavailable:
    error: NormGeneratorError | CudaRNGUnavailable | object
    kind: Literal["NormalsUnavailable"] = "NormalsUnavailable"


@dataclass(frozen=True)
class NormalsGenerationFailed:
    error: NormGeneratorError | object
    kind: Literal["NormalsGenerationFailed"] = "NormalsGenerationFailed"


@dataclass(frozen=True)
class EngineFailure:
    """A status code returned by libspectralmc_hip (HIP launch / shape error)."""

    code: int
    message: str
    kind: Literal["EngineFailure"] = "EngineFailure"
