"""Lowering of CVNN modules to the fused kernels' layer table (CPU, no launches)."""

from __future__ import annotations

import pytest
import torch

from spectralmc_amd import _lib
from spectralmc_amd.cvnn import ComplexLinear, ComplexSequential, NaiveComplexBatchNorm, modReLU, zReLU
from spectralmc_amd.net import UnsupportedNetwork, lower
from tests.helpers import make_test_cvnn


def test_lower_benchmark_architecture() -> None:
    model = make_test_cvnn(n_inputs=6, n_outputs=256, seed=123, dtype=torch.float32, device="cpu", hidden_layers=2)
    params = list(model.parameters())
    table = lower(model, params)
    assert [(t.in_features, t.out_features, t.activation) for t in table] == [
        (6, 32, _lib.ACT_MODRELU), (32, 32, _lib.ACT_MODRELU), (32, 256, _lib.ACT_NONE)]
    offs = {}
    o = 0
    for name, p in model.named_parameters():
        offs[name] = o
        o += p.numel()
    assert table[0].w_re == offs["layers.0.layers.0.real_weight"]
    assert table[2].w_im in offs.values() and table[2].w_re in offs.values()
    covered = set()
    for t in table:
        for f, n in (("w_re", t.in_features * t.out_features), ("w_im", t.in_features * t.out_features),
                     ("b_re", t.out_features), ("b_im", t.out_features), ("act_bias", t.out_features)):
            start = getattr(t, f)
            if start >= 0:
                covered.update(range(start, start + n))
    assert covered == set(range(o))


def test_lower_zrelu_and_no_bias() -> None:
    m = ComplexSequential(ComplexLinear(4, 8, bias=False), zReLU(), ComplexLinear(8, 3))
    t = lower(m, list(m.parameters()))
    assert t[0].activation == _lib.ACT_ZRELU and t[0].b_re == -1 and t[0].b_im == -1 and t[1].b_re >= 0


@pytest.mark.parametrize("bad", [
    lambda: ComplexSequential(ComplexLinear(4, 8), NaiveComplexBatchNorm(8), ComplexLinear(8, 3)),
    lambda: ComplexSequential(modReLU(4), ComplexLinear(4, 3)),
])
def test_lower_rejects_unsupported(bad) -> None:
    m = bad()
    with pytest.raises(UnsupportedNetwork):
        lower(m, list(m.parameters()))
