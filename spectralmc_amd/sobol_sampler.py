"""Scrambled-Sobol contract sampler (reference ``src/spectralmc/sobol_sampler.py``).

The SciPy engine the reference wraps (``Sobol(d, scramble=True, seed)``, line 192) is
re-implemented bit-exactly in ``libspectralmc_hip.so`` (``smc_sobol_*``): the host handle
reproduces SciPy's LMS + digital-shift scramble, and points are direct-indexed through the
Gray code, so the same generator also runs as a device kernel (``draw_device``) that writes
the trainer's ``(B, 6)`` f64 contract batch straight into HBM.

``SobolSampler.sample`` keeps the reference semantics: a list of validated Pydantic points,
``Failure(NegativeSamples)`` for ``n < 0``, ``Failure(SamplerValidationFailed)`` when a
scaled row violates the model.
"""

from __future__ import annotations

import ctypes
from collections.abc import Mapping
from dataclasses import dataclass
from types import MappingProxyType
from typing import Generic, Iterator, TypeVar

import numpy as np
from pydantic import BaseModel, ValidationError

from . import _lib
from .errors.sampler import (
    BoundSpecInvalid,
    DimensionMismatch,
    InvalidBounds,
    NegativeSamples,
    SamplerValidationFailed,
)
from .result import Failure, Result, Success, collect_results
from .validation import validate_model

PointT = TypeVar("PointT", bound=BaseModel)

MAX_POINTS = 1 << _lib.SOBOL_BITS


@dataclass(frozen=True)
class SobolConfig:
    seed: int
    skip: int = 0


@dataclass(frozen=True)
class BoundSpec:
    """Inclusive [lower, upper] of one axis (build with ``build_bound_spec``)."""

    lower: float
    upper: float


@dataclass(frozen=True)
class DomainBounds(Generic[PointT], Mapping[str, BoundSpec]):
    """Bounds keyed by model field, frozen in the model's field order."""

    _fields: tuple[str, ...]
    _bounds: Mapping[str, BoundSpec]

    @property
    def fields(self) -> tuple[str, ...]:
        return self._fields

    def __getitem__(self, key: str) -> BoundSpec:
        return self._bounds[key]

    def __iter__(self) -> Iterator[str]:
        return iter(self._bounds)

    def __len__(self) -> int:
        return len(self._bounds)

    def arrays(self) -> tuple[np.ndarray, np.ndarray]:
        lo = np.array([self._bounds[f].lower for f in self._fields], dtype=np.float64)
        hi = np.array([self._bounds[f].upper for f in self._fields], dtype=np.float64)
        return lo, hi


def build_domain_bounds(pydantic_class: type[PointT], bounds: Mapping[str, BoundSpec]
                        ) -> Result[DomainBounds[PointT], DimensionMismatch]:
    fields = tuple(pydantic_class.model_fields)
    given = tuple(bounds.keys())
    if set(given) != set(fields):
        return Failure(DimensionMismatch(expected_fields=fields, provided_fields=given))
    return Success(DomainBounds(_fields=fields, _bounds=MappingProxyType({f: bounds[f] for f in fields})))


def build_bound_spec(lower: float, upper: float) -> Result[BoundSpec, BoundSpecInvalid]:
    if lower >= upper:
        return Failure(BoundSpecInvalid(lower=lower, upper=upper))
    return Success(BoundSpec(lower=lower, upper=upper))


def build_sobol_config(*, seed: int, skip: int = 0) -> Result[SobolConfig, ValidationError]:
    if seed < 0 or skip < 0:
        return Failure(ValidationError.from_exception_data("SobolConfig", []))
    return Success(SobolConfig(seed=seed, skip=skip))


class SobolEngine:
    """Owner of one ``smc_sobol`` handle: SciPy-identical scrambled Sobol stream."""

    def __init__(self, dim: int, seed: int, skip: int = 0) -> None:
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.smc_sobol_create(dim, seed, skip, ctypes.byref(h)))
        self._h = h
        self.dim = dim
        self.seed = seed

    def __del__(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib().smc_sobol_destroy(h)
            self._h = None

    @property
    def cursor(self) -> int:
        cur = ctypes.c_uint64()
        _lib.check(_lib.lib().smc_sobol_state(self._h, None, None, ctypes.byref(cur)))
        return int(cur.value)

    def fast_forward(self, n: int) -> None:
        _lib.check(_lib.lib().smc_sobol_fast_forward(self._h, n))

    def random(self, n: int) -> np.ndarray:
        out = np.empty((n, self.dim), dtype=np.float64)
        _lib.check(_lib.lib().smc_sobol_random_host(self._h, n, _lib.ptr(out)))
        return out

    def tables(self) -> np.ndarray:
        """Device table image: shift[dim] then sv[dim][30] (u32)."""
        out = np.empty(self.dim * (1 + _lib.SOBOL_BITS), dtype=np.uint32)
        _lib.check(_lib.lib().smc_sobol_export_tables(self._h, _lib.ptr(out)))
        return out

    def state(self) -> tuple[np.ndarray, np.ndarray]:
        shift = np.empty(self.dim, dtype=np.uint32)
        sv = np.empty((self.dim, _lib.SOBOL_BITS), dtype=np.uint32)
        _lib.check(_lib.lib().smc_sobol_state(self._h, _lib.ptr(shift), _lib.ptr(sv), None))
        return shift, sv


def draw_device(tables_dev, dim: int, index_dev, index0: int, n: int, lower_dev, upper_dev, out_f64,
                out_f32=None, stream=None) -> None:
    """Launch the Gray-code kernel: rows of ``lower + (upper - lower) * x`` into ``out_f64``."""
    _lib.check(_lib.lib().smc_sobol_draw(_lib.ptr(tables_dev), dim, _lib.ptr(index_dev), index0, n,
                                         _lib.ptr(lower_dev), _lib.ptr(upper_dev), _lib.ptr(out_f64),
                                         _lib.ptr(out_f32), _lib.stream_handle(stream)))


class SobolSampler(Generic[PointT]):
    """Draw Sobol points inside ``DomainBounds`` and validate them through a Pydantic model."""

    def __init__(self, *, fields: list[str], lower: np.ndarray, upper: np.ndarray, model: type[PointT],
                 engine: SobolEngine) -> None:
        self._fields = fields
        self._lower = lower
        self._upper = upper
        self._model = model
        self._engine = engine

    @classmethod
    def create(cls, pydantic_class: type[PointT], dimensions: DomainBounds[PointT], *, config: SobolConfig
               ) -> Result["SobolSampler[PointT]", DimensionMismatch | InvalidBounds]:
        fields = list(dimensions.fields)
        try:
            lower, upper = dimensions.arrays()
            engine = SobolEngine(len(fields), config.seed, config.skip)
        except (_lib.SmcError, ValueError) as exc:
            return Failure(InvalidBounds(message=str(exc)))
        return Success(cls(fields=fields, lower=lower, upper=upper, model=pydantic_class, engine=engine))

    # -- accessors used by the device trainer -------------------------------------------
    @property
    def engine(self) -> SobolEngine:
        return self._engine

    @property
    def bounds(self) -> tuple[np.ndarray, np.ndarray]:
        return self._lower, self._upper

    @property
    def fields(self) -> list[str]:
        return list(self._fields)

    @property
    def position(self) -> int:
        """Index of the next point (= skip + points drawn)."""
        return self._engine.cursor

    def skip(self, n: int) -> None:
        self._engine.fast_forward(n)

    def sample_array(self, n_samples: int) -> np.ndarray:
        """``lower + (upper - lower) * raw`` as an (n, d) f64 array (sobol_sampler.py:238-239)."""
        if n_samples < 0:
            raise ValueError("n_samples must be >= 0")
        if self._engine.cursor + n_samples > MAX_POINTS:
            raise ValueError(f"At most 2**{_lib.SOBOL_BITS}={MAX_POINTS} distinct points can be generated")
        raw = self._engine.random(n_samples)
        return self._lower + (self._upper - self._lower) * raw

    def _construct(self, row: np.ndarray) -> Result[PointT, SamplerValidationFailed]:
        res = validate_model(self._model, **{name: float(row[i]) for i, name in enumerate(self._fields)})
        if isinstance(res, Failure):
            return Failure(SamplerValidationFailed(error=res.error))
        return res

    def sample(self, n_samples: int) -> Result[list[PointT], NegativeSamples | SamplerValidationFailed]:
        if n_samples < 0:
            return Failure(NegativeSamples(n_samples=n_samples))
        if n_samples == 0:
            return Success([])
        scaled = self.sample_array(n_samples)
        return collect_results([self._construct(row) for row in scaled])


__all__ = ["BoundSpec", "DomainBounds", "SobolConfig", "SobolSampler", "SobolEngine", "build_bound_spec",
           "build_domain_bounds", "build_sobol_config", "draw_device"]
