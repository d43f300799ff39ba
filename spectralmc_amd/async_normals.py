"""Normal-matrix generator API (reference ``src/spectralmc/async_normals.py:106-470``).

The reference keeps a pool of CuPy workers that pre-generate ``(rows, cols)`` N(0,1)
matrices on their own streams; matrix m (the m-th served, ``skips`` restores the count) is
``cupy.random.default_rng(seed_m).standard_normal`` with ``seed_m`` the m-th draw of
``numpy.random.default_rng(seed).integers(0, 1e9)``.

Here matrix m is the normal matrix the HIP engine itself draws for contract ordinal m
(``smc_normals``: Philox-seeded MWC64X streams + Box-Muller, csrc/smc_rng.h), so the
generator and ``BlackScholes`` agree on every value, the matrices never cross PCIe, and
``skips`` restores a position in O(1).  The pool / stream / buffer-size structure, config
validation and error values are the reference's; the values are not CuPy's (normal-level
parity with CuPy is unpinned).
"""

from __future__ import annotations

from dataclasses import dataclass
from itertools import cycle
from time import time

import torch

from . import _lib
from .errors.async_normals import InvalidDType, InvalidShape, QueueBusy, QueueEmpty, SeedOutOfRange
from .models.numerical import Precision
from .result import Failure, Result, Success

_SEED_LIMIT = 1_000_000_000


@dataclass(frozen=True)
class BufferConfig:
    """Pool size, validated against the matrix shape (reference async_normals.py:106-126)."""

    size: int

    @classmethod
    def create(cls, size: int, matrix_rows: int, matrix_cols: int) -> Result["BufferConfig", InvalidShape]:
        bad = size > matrix_rows * matrix_cols or min(matrix_rows, matrix_cols) <= 0 or size <= 0
        return Failure(InvalidShape(rows=matrix_rows, cols=matrix_cols)) if bad else Success(cls(size=size))


@dataclass(frozen=True)
class ConcurrentNormGeneratorConfig:
    """Serialisable generator position (reference async_normals.py:129-170)."""

    rows: int
    cols: int
    seed: int
    dtype: Precision
    skips: int = 0

    @classmethod
    def create(cls, *, rows: int, cols: int, seed: int, dtype: Precision, skips: int = 0
               ) -> Result["ConcurrentNormGeneratorConfig", InvalidShape | SeedOutOfRange]:
        if rows <= 0 or cols <= 0:
            return Failure(InvalidShape(rows=rows, cols=cols))
        if seed <= 0:
            return Failure(SeedOutOfRange(seed=seed))
        if skips < 0:
            return Failure(SeedOutOfRange(seed=skips))
        return Success(cls(rows=rows, cols=cols, seed=seed, dtype=dtype, skips=skips))


def _dtype_code(dtype: object) -> Result[tuple[int, torch.dtype], InvalidDType]:
    if dtype in (Precision.float32, torch.float32):
        return Success((_lib.DTYPE_F32, torch.float32))
    if dtype in (Precision.float64, torch.float64):
        return Success((_lib.DTYPE_F64, torch.float64))
    return Failure(InvalidDType(requested=str(dtype)))


class _NormWorker:
    """One pre-generated matrix on a dedicated HIP stream (reference _NormGenerator 173-256)."""

    def __init__(self, rows: int, cols: int, seed: int, code: int, dtype: torch.dtype, device: torch.device) -> None:
        self._rows, self._cols, self._seed, self._code, self._dtype = rows, cols, seed, code, dtype
        self._device = device
        self._stream = torch.cuda.Stream(device=device)
        self._generated: torch.Tensor | None = None
        self._event: torch.cuda.Event | None = None
        self._sync_time = 0.0

    def enqueue(self, ordinal: int) -> Result[None, QueueBusy | SeedOutOfRange]:
        if self._generated is not None:
            return Failure(QueueBusy())
        if ordinal < 0:
            return Failure(SeedOutOfRange(seed=ordinal))
        out = torch.empty((self._rows, self._cols), dtype=self._dtype, device=self._device)
        out.record_stream(self._stream)
        self._stream.wait_stream(torch.cuda.current_stream(self._device))  # `out` allocated on the current stream
        _lib.check(_lib.lib().smc_normals(self._seed, ordinal, self._rows, self._cols, self._code, _lib.ptr(out),
                                          _lib.stream_handle(self._stream)))
        self._event = torch.cuda.Event()
        self._event.record(self._stream)
        self._generated = out
        return Success(None)

    def take(self, next_ordinal: int) -> Result[torch.Tensor, QueueEmpty | QueueBusy | SeedOutOfRange]:
        if self._generated is None:
            return Failure(QueueEmpty())
        t0 = time()
        torch.cuda.current_stream(self._device).wait_stream(self._stream)
        self._stream.synchronize()
        self._sync_time += time() - t0
        ready, self._generated = self._generated, None
        queued = self.enqueue(next_ordinal)
        return Success(ready) if isinstance(queued, Success) else queued

    def is_ready(self) -> bool:
        return self._event is not None and self._event.query()

    def get_time_spent_synchronizing(self) -> float:
        return self._sync_time


class ConcurrentNormGenerator:
    """Pool of ``buffer.size`` workers serving matrices m = skips, skips+1, ... in order."""

    def __init__(self, *, pool: list[_NormWorker], rows: int, cols: int, dtype: Precision, seed: int,
                 served: int) -> None:
        self._pool = pool
        self._it = cycle(pool)
        self._rows, self._cols, self._precision, self._seed = rows, cols, dtype, seed
        self._served = served
        self._idle_accum = 0.0
        self._idle_start: float | None = None
        self._update_idle_state()

    @classmethod
    def create(cls, buffer_result: Result[BufferConfig, InvalidShape], config: ConcurrentNormGeneratorConfig,
               *, math: str = "portable") -> Result["ConcurrentNormGenerator",
                                                    InvalidShape | InvalidDType | QueueBusy | SeedOutOfRange]:
        """``math="portable"``: the CPU-reproducible normals (bit-identical to the oracle);
        ``"hw"``: the hardware-transcendental normals of the engine's throughput mode."""
        if isinstance(buffer_result, Failure):
            return buffer_result
        dt = _dtype_code(config.dtype)
        if isinstance(dt, Failure):
            return dt
        code, tdtype = dt.value
        if math == "hw" and code == _lib.DTYPE_F32:
            code |= _lib.MATH_HW
        _lib.require_device()
        device = torch.device("cuda", torch.cuda.current_device())
        pool = []
        for i in range(buffer_result.value.size):
            w = _NormWorker(config.rows, config.cols, config.seed, code, tdtype, device)
            queued = w.enqueue(config.skips + i)
            if isinstance(queued, Failure):
                return queued
            pool.append(w)
        return Success(cls(pool=pool, rows=config.rows, cols=config.cols, dtype=config.dtype, seed=config.seed,
                           served=config.skips))

    def _update_idle_state(self) -> None:
        all_ready = all(w.is_ready() for w in self._pool)
        now = time()
        if all_ready and self._idle_start is None:
            self._idle_start = now
        elif not all_ready and self._idle_start is not None:
            self._idle_accum += now - self._idle_start
            self._idle_start = None

    def get_matrix(self) -> Result[torch.Tensor, QueueEmpty | QueueBusy | SeedOutOfRange]:
        """The next matrix (ordinal = number served so far); its worker queues ordinal + pool size."""
        w = next(self._it)
        got = w.take(self._served + len(self._pool))
        if isinstance(got, Failure):
            return got
        self._served += 1
        self._update_idle_state()
        return got

    def snapshot(self) -> ConcurrentNormGeneratorConfig:
        cfg = ConcurrentNormGeneratorConfig.create(rows=self._rows, cols=self._cols, seed=self._seed,
                                                   dtype=self._precision, skips=self._served)
        if isinstance(cfg, Failure):
            raise AssertionError(f"Invalid ConcurrentNormGeneratorConfig snapshot: {cfg.error}")
        return cfg.value

    def get_time_spent_synchronizing(self) -> float:
        return sum(w.get_time_spent_synchronizing() for w in self._pool)

    def get_idle_time(self) -> float:
        self._update_idle_state()
        return self._idle_accum + (time() - self._idle_start if self._idle_start is not None else 0.0)

    @property
    def dtype(self) -> torch.dtype:
        return _dtype_code(self._precision).value[1]


__all__ = ["BufferConfig", "ConcurrentNormGeneratorConfig", "ConcurrentNormGenerator"]
