"""Basket (multi-asset) extension on the CPU: host config validation and the oracle's
kernel-mode restatement against an independent numpy statement of the same step."""

from __future__ import annotations

import numpy as np
import pytest

from spectralmc_amd.basket import BasketConfig, basket_fields, default_basket_bounds


def test_fields_and_bounds_order() -> None:
    f = basket_fields(4)
    assert f[:4] == ("K", "T", "r", "rho") and len(f) == 16
    assert f[4:8] == ("X0_0", "X0_1", "X0_2", "X0_3") and f[-1] == "v_3"
    cfg = BasketConfig(n_assets=4)
    lo, hi = cfg.arrays()
    assert lo.shape == (16,) and (hi > lo).all()
    assert set(default_basket_bounds(4)) == set(f)


@pytest.mark.parametrize("kw", [dict(n_assets=0), dict(n_assets=9), dict(network_size=66),
                                dict(network_size=64, batches_per_mc_run=3), dict(math="fast"),
                                dict(n_assets=4, bounds={"rho": (-0.5, 0.9)}), dict(bounds={"nope": (0, 1)})])
def test_config_rejects(kw) -> None:
    with pytest.raises(ValueError):
        BasketConfig(**kw)


@pytest.mark.parametrize("A,rho", [(1, 0.0), (2, -0.5), (4, 0.3), (8, 0.9), (5, -0.2)])
def test_oracle_cholesky(oracle, A, rho) -> None:
    L = oracle.basket_cholesky(A, rho)
    C = np.full((A, A), rho)
    np.fill_diagonal(C, 1.0)
    np.testing.assert_allclose(L @ L.T, C, atol=1e-14)
    assert np.allclose(np.triu(L, 1), 0.0)


@pytest.mark.parametrize("A", [1, 3, 4])
def test_oracle_kernel_matches_numpy_statement(oracle, A) -> None:
    """Kernel-mode f32 targets vs numpy (f64 payoff + FFT per batch row, then mean) on the same
    terminal values: the two orders agree to f32 accuracy (1e-5 of the row scale)."""
    cfg = BasketConfig(n_assets=A, timesteps=8, network_size=64, batches_per_mc_run=32)
    lo, hi = cfg.arrays()
    c = oracle.sobol_contracts(7, 0, 6, lo, hi)
    paths, tsum, targets = oracle.basket_kernel(c, A, 8, 64, 32, 7, want_paths=True)
    term = paths[:, :, -1, :].astype(np.float64)
    np.testing.assert_allclose(tsum, term.sum(axis=2), rtol=1e-6)  # f32 4-path partials
    ref = oracle.basket_reference_targets(c, A, term, 64, 32)
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-30
    assert float((np.abs(targets - ref) / scale).max()) < 1e-5


def test_oracle_is_deterministic_and_ordinal_keyed(oracle) -> None:
    cfg = BasketConfig(n_assets=2, timesteps=4, network_size=64, batches_per_mc_run=32)
    lo, hi = cfg.arrays()
    c = oracle.sobol_contracts(7, 0, 3, lo, hi)
    _, _, a = oracle.basket_kernel(c, 2, 4, 64, 32, 7, ordinal0=0)
    _, _, b = oracle.basket_kernel(c, 2, 4, 64, 32, 7, ordinal0=0)
    np.testing.assert_array_equal(a, b)
    # contract i at ordinal0 = i alone equals row i of the batch (streams keyed by global ordinal)
    _, _, one = oracle.basket_kernel(c[1:2], 2, 4, 64, 32, 7, ordinal0=1)
    np.testing.assert_array_equal(one[0], a[1])
