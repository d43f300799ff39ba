"""Normal-stream errors (reference ``src/spectralmc/errors/async_normals.py``)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal


@dataclass(frozen=True)
class InvalidDType:
    requested: str
    kind: Literal["InvalidDType"] = "InvalidDType"


@dataclass(frozen=True)
class InvalidShape:
    rows: int
    cols: int
    kind: Literal["InvalidShape"] = "InvalidShape"


@dataclass(frozen=True)
class SeedOutOfRange:
    seed: int
    kind: Literal["SeedOutOfRange"] = "SeedOutOfRange"


@dataclass(frozen=True)
class QueueEmpty:
    kind: Literal["QueueEmpty"] = "QueueEmpty"


@dataclass(frozen=True)
class QueueBusy:
    kind: Literal["QueueBusy"] = "QueueBusy"


@dataclass(frozen=True)
class InvalidBufferSize:
    size: int
    matrix_rows: int
    matrix_cols: int
    kind: Literal["InvalidBufferSize"] = "InvalidBufferSize"


NormGeneratorError = InvalidDType | InvalidShape | SeedOutOfRange | QueueEmpty | QueueBusy | InvalidBufferSize
