"""Trainer errors (reference ``src/spectralmc/errors/trainer.py``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

from .gbm import EngineFailure, NormalsGenerationFailed, NormalsUnavailable
from .sampler import SamplerError


@dataclass(frozen=True)
class SamplerInitFailed:
    error: SamplerError | object
    kind: Literal["SamplerInitFailed"] = "SamplerInitFailed"


@dataclass(frozen=True)
class InvalidTrainerConfig:
    message: str
    kind: Literal["InvalidTrainerConfig"] = "InvalidTrainerConfig"


@dataclass(frozen=True)
class InvalidTrainingConfig:
    num_batches: int
    batch_size: int
    learning_rate: float
    message: str
    kind: Literal["InvalidTrainingConfig"] = "InvalidTrainingConfig"


@dataclass(frozen=True)
class OptimizerStateSerializationFailed:
    message: str
    kind: Literal["OptimizerStateSerializationFailed"] = "OptimizerStateSerializationFailed"


@dataclass(frozen=True)
class PredictionFailed:
    message: str
    kind: Literal["PredictionFailed"] = "PredictionFailed"


TrainerError = (
    SamplerInitFailed
    | InvalidTrainerConfig
    | InvalidTrainingConfig
    | OptimizerStateSerializationFailed
    | PredictionFailed
    | NormalsUnavailable
    | NormalsGenerationFailed
    | EngineFailure
)
