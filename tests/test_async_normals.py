"""ConcurrentNormGenerator API (reference async_normals.py; tests/test_async_normals.py:94-123
restore semantics).  CPU: validation; GPU: values = the engine's normals = the oracle's."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from spectralmc_amd.async_normals import BufferConfig, ConcurrentNormGenerator, ConcurrentNormGeneratorConfig
from spectralmc_amd.errors.async_normals import InvalidShape, SeedOutOfRange
from spectralmc_amd.models.numerical import Precision
from spectralmc_amd.result import Failure, Success


def test_buffer_config_validation() -> None:
    assert isinstance(BufferConfig.create(4, 2, 3), Success)
    for args in ((7, 2, 3), (0, 2, 3), (1, 0, 3), (1, 2, -1)):
        r = BufferConfig.create(*args)
        assert isinstance(r, Failure) and isinstance(r.error, InvalidShape)


def test_generator_config_validation() -> None:
    assert isinstance(ConcurrentNormGeneratorConfig.create(rows=2, cols=3, seed=1, dtype=Precision.float32), Success)
    assert isinstance(ConcurrentNormGeneratorConfig.create(rows=0, cols=3, seed=1, dtype=Precision.float32).error,
                      InvalidShape)
    assert isinstance(ConcurrentNormGeneratorConfig.create(rows=2, cols=3, seed=0, dtype=Precision.float32).error,
                      SeedOutOfRange)
    assert isinstance(ConcurrentNormGeneratorConfig.create(rows=2, cols=3, seed=5, dtype=Precision.float32,
                                                           skips=-1).error, SeedOutOfRange)


def _gen(rows, cols, seed, dtype, skips=0, size=3, math="portable"):
    cfg = ConcurrentNormGeneratorConfig.create(rows=rows, cols=cols, seed=seed, dtype=dtype, skips=skips).value
    res = ConcurrentNormGenerator.create(BufferConfig.create(size, rows, cols), cfg, math=math)
    assert isinstance(res, Success), res
    return res.value


@pytest.mark.gpu
@pytest.mark.parametrize("prec,dt", [(Precision.float32, "float32"), (Precision.float64, "float64")])
def test_matrices_are_the_engine_normals(oracle, prec, dt) -> None:
    g = _gen(6, 40, 11, prec)
    for m in range(5):
        got = g.get_matrix().value.cpu().numpy()
        want = oracle.normals(11, m, 6, 40, dt)
        if dt == "float32":
            np.testing.assert_array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    assert g.snapshot().skips == 5
    assert g.dtype == (torch.float32 if dt == "float32" else torch.float64)


@pytest.mark.gpu
def test_restore_continues_stream_with_other_buffer_size() -> None:
    a = _gen(4, 16, 3, Precision.float32, size=2)
    first = [a.get_matrix().value.clone() for _ in range(3)]
    snap = a.snapshot()
    rest = [a.get_matrix().value.clone() for _ in range(4)]
    b = ConcurrentNormGenerator.create(BufferConfig.create(5, 4, 16), snap).value
    again = [b.get_matrix().value for _ in range(4)]
    for x, y in zip(rest, again):
        assert torch.equal(x, y)
    assert not torch.equal(first[0], first[1])
    assert a.get_time_spent_synchronizing() >= 0.0 and a.get_idle_time() >= 0.0


@pytest.mark.gpu
def test_hw_math_normals_close_to_portable() -> None:
    p = _gen(8, 256, 9, Precision.float32).get_matrix().value
    h = _gen(8, 256, 9, Precision.float32, math="hw").get_matrix().value
    torch.testing.assert_close(h, p, rtol=2e-5, atol=2e-5)
    z = _gen(64, 4096, 21, Precision.float32).get_matrix().value.double()
    assert abs(float(z.mean())) < 0.01 and abs(float(z.var()) - 1.0) < 0.01
