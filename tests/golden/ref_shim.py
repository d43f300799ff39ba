"""CPU shims that let the reference's own ``spectralmc.gbm`` / ``async_normals`` run in the
build container (no CuPy, no Numba, no GPU).  Used only by ``make_golden.py`` to GENERATE
fixtures; nothing here is imported by the product, by the GPU tests or on the GPU box.

Recipe:
* ``spectralmc.runtime``: ``get_torch_handle`` returns torch (bypasses the CUDA-presence guard
  only, reference runtime/torch_runtime.py:83-97).
* ``cupy`` -> numpy: ``ndarray``/``dtype``/``linspace``/``exp``/``mean``/``maximum``/``fft``
  are numpy's (NEP 50 weak Python scalars, as CuPy's kernels cast them to the array dtype);
  streams and events are no-ops.  ``random.default_rng(seed).standard_normal((T, P), dtype)``
  returns the BUILD's normal matrix for the next contract ordinal (``oracle.normals``), so every
  op downstream of the normals is the reference's own code.  The k-th matrix the pool enqueues
  is the k-th matrix it serves (reference async_normals.py:319-398, any buffer size).
* ``numba.cuda.jit`` -> a serial grid emulator.  Array loads hand back Python floats and stores
  round into the array's dtype, which is Numba's typing of ``SimulateBlackScholes``
  (gbm.py:241-257: Python-float arguments make the recursion f64, only ``io`` is f32).
* ``spectralmc.effects``: the two enums loaded by file path from ``effects/montecarlo.py`` plus
  inert effect records (the interpreter package needs the whole storage stack).
"""

from __future__ import annotations

import importlib.util
import os
import sys
import types
from typing import Any, Callable

import numpy as np


class NormalSource:
    """Serves the build's normal matrices in contract-ordinal order."""

    def __init__(self, seed: int, ordinal0: int = 0) -> None:
        self.seed = seed
        self.next_ordinal = ordinal0

    def matrix(self, shape: tuple[int, int], dtype: Any) -> np.ndarray:
        import oracle  # noqa: PLC0415  (test infrastructure)

        name = "float64" if np.dtype(dtype) == np.float64 else "float32"
        out = oracle.normals(self.seed, self.next_ordinal, shape[0], shape[1], name)
        self.next_ordinal += 1
        return out


SOURCE = NormalSource(7)


# --------------------------------------------------------------------------- cupy -> numpy
class _Stream:
    def __init__(self, *_: Any, **__: Any) -> None:
        pass

    def __enter__(self) -> "_Stream":
        return self

    def __exit__(self, *_: Any) -> None:
        return None

    def synchronize(self) -> None:
        return None


class _Event:
    ptr = 0

    def __init__(self, *_: Any, **__: Any) -> None:
        pass

    def record(self, *_: Any) -> None:
        return None


class _Generator:
    def __init__(self, seed: int) -> None:
        self.seed = seed

    def standard_normal(self, shape: tuple[int, int], dtype: Any = np.float64) -> np.ndarray:
        return SOURCE.matrix(shape, dtype)


class _ArrayMeta(type):
    def __instancecheck__(cls, obj: Any) -> bool:
        # CuPy indexing gives 0-d arrays where numpy gives scalars (gbm.py:465-466)
        return isinstance(obj, (np.ndarray, np.generic))


class _NDArray(metaclass=_ArrayMeta):
    """``cupy.ndarray`` for Pydantic's isinstance checks: numpy arrays and numpy scalars."""


def _make_cupy() -> types.ModuleType:
    cp = types.ModuleType("cupy")
    cp.ndarray = _NDArray
    for name in ("dtype", "float32", "float64", "complex64", "complex128", "linspace", "exp",
                 "mean", "maximum", "expand_dims", "asarray", "fft", "zeros", "empty", "sqrt", "abs"):
        setattr(cp, name, getattr(np, name))
    cuda = types.ModuleType("cupy.cuda")
    cuda.Stream = _Stream
    cuda.Event = _Event
    runtime = types.ModuleType("cupy.cuda.runtime")
    runtime.eventQuery = lambda ptr: 0
    cuda.runtime = runtime
    cp.cuda = cuda
    rnd = types.ModuleType("cupy.random")
    rnd.default_rng = _Generator
    cp.random = rnd
    return cp


# --------------------------------------------------------------------------- numba.cuda
class _DeviceArray:
    """Numba device-array view: loads give Python floats (f64), stores round to the dtype."""

    def __init__(self, arr: np.ndarray) -> None:
        self._a = arr
        self.shape = arr.shape

    def __getitem__(self, ij: tuple[int, int]) -> float:
        return float(self._a[ij])

    def __setitem__(self, ij: tuple[int, int], value: float) -> None:
        self._a[ij] = value


class _Kernel:
    def __init__(self, fn: Callable[..., None]) -> None:
        self.fn = fn

    def __getitem__(self, launch: tuple[Any, ...]) -> Callable[..., None]:
        blocks, tpb = int(launch[0]), int(launch[1])

        def run(*args: Any) -> None:
            for idx in range(blocks * tpb):
                _CUDA_STATE["idx"] = idx
                self.fn(*args)

        return run


_CUDA_STATE = {"idx": 0}


def _make_numba() -> dict[str, types.ModuleType]:
    numba = types.ModuleType("numba")
    cuda = types.ModuleType("numba.cuda")
    cuda.jit = lambda fn: _Kernel(fn)
    cuda.grid = lambda ndim: _CUDA_STATE["idx"]
    cuda.stream = _Stream
    cuda.as_cuda_array = _DeviceArray
    numba.cuda = cuda
    cudadrv = types.ModuleType("numba.cuda.cudadrv")
    devicearray = types.ModuleType("numba.cuda.cudadrv.devicearray")
    devicearray.DeviceNDArray = _DeviceArray
    cudadrv.devicearray = devicearray
    cuda.cudadrv = cudadrv
    return {"numba": numba, "numba.cuda": cuda, "numba.cuda.cudadrv": cudadrv,
            "numba.cuda.cudadrv.devicearray": devicearray}


# --------------------------------------------------------------------------- effects
def _make_effects(ref_src: str) -> dict[str, types.ModuleType]:
    path = os.path.join(ref_src, "spectralmc", "effects", "montecarlo.py")
    spec = importlib.util.spec_from_file_location("spectralmc.effects.montecarlo", path)
    assert spec is not None and spec.loader is not None
    mc = importlib.util.module_from_spec(spec)
    sys.modules["spectralmc.effects.montecarlo"] = mc
    spec.loader.exec_module(mc)
    eff = types.ModuleType("spectralmc.effects")
    eff.__path__ = []  # package marker
    eff.PathScheme = mc.PathScheme
    eff.ForwardNormalization = mc.ForwardNormalization

    class _Inert:
        def __init__(self, *args: Any, **kwargs: Any) -> None:
            self.args, self.kwargs = args, kwargs

    for name in ("EffectSequence", "GenerateNormals", "SimulatePaths", "StreamSync", "CaptureRNGState"):
        setattr(eff, name, _Inert)
    eff.sequence_effects = lambda *effects: list(effects)
    return {"spectralmc.effects": eff, "spectralmc.effects.montecarlo": mc}


def install(ref_src: str) -> None:
    """Install every shim and put the reference source tree on sys.path."""
    import torch

    sys.dont_write_bytecode = True
    if ref_src not in sys.path:
        sys.path.insert(0, ref_src)
    guard = types.ModuleType("spectralmc.runtime")
    guard.get_torch_handle = lambda: torch
    sys.modules["spectralmc.runtime"] = guard
    sys.modules["cupy"] = _make_cupy()
    sys.modules.update(_make_numba())
    sys.modules.update(_make_effects(ref_src))
