"""The oracle (CPU restatement) pinned against the reference's golden vectors, published
known-answer vectors and closed-form cases.  CPU only."""

from __future__ import annotations

import math

import numpy as np
import pytest

# Random123 kat_vectors, philox4x32 R=10 (Salmon et al. 2011)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expected", PHILOX_KAT)
def test_philox_known_answers(oracle, ctr, key, expected) -> None:
    assert oracle.philox4x32_10(ctr, key) == expected


@pytest.mark.parametrize("seed", [7, 31, 42, 123])
@pytest.mark.parametrize("skip", [0, 8, 4096])
def test_oracle_sobol_matches_reference_sampler(oracle, golden, seed, skip) -> None:
    lo, hi = golden["bounds_lower"], golden["bounds_upper"]
    got = oracle.sobol_contracts(seed, skip, 64, lo, hi)
    np.testing.assert_array_equal(got, golden[f"sobol_s{seed}_k{skip}"])
    nxt = oracle.sobol_contracts(seed, skip + 64, 32, lo, hi)
    np.testing.assert_array_equal(nxt, golden[f"sobol_s{seed}_k{skip}_next"])


def test_oracle_normals_are_standard(oracle) -> None:
    z = oracle.normals(7, 3, 16, 65536).astype(np.float64)
    assert abs(z.mean()) < 5e-3
    assert abs(z.std() - 1.0) < 5e-3
    # independent streams per path and per ordinal
    z2 = oracle.normals(7, 4, 16, 65536)
    assert abs(np.corrcoef(z.ravel(), z2.ravel().astype(np.float64))[0, 1]) < 5e-3


def test_oracle_zero_vol_paths_are_forwards(oracle) -> None:
    """v = 0: every path is the deterministic forward X0 e^{(r-d) t} (gbm.py:245-250)."""
    c = np.array([[100.0, 95.0, 2.0, 0.05, 0.01, 0.0]])
    T = 8
    paths, term, rowsum = oracle.gbm_paths(c, T, 64, 7, dtype="float64", want_paths=True)
    t = np.linspace(2.0 / T, 2.0, T)
    fwd = 100.0 * np.exp(0.04 * t)
    np.testing.assert_allclose(paths[0], np.broadcast_to(fwd[:, None], (T, 64)), rtol=1e-13)
    np.testing.assert_allclose(rowsum[0] / 64, fwd, rtol=1e-13)


def test_oracle_zero_maturity(oracle) -> None:
    c = np.array([[50.0, 40.0, 0.0, 0.1, 0.0, 0.7]])
    _, term, _ = oracle.gbm_paths(c, 4, 128, 9, dtype="float32")
    assert np.all(term == np.float32(50.0))


def test_oracle_mc_price_matches_black(oracle) -> None:
    """Reference tests/test_gbm.py:103-139 acceptance on a few contracts: MC put vs Black."""
    rng = np.random.default_rng(3)
    rel = []
    for i in range(8):
        X0, K = rng.uniform(50, 150), rng.uniform(50, 150)
        T, r, d, v = rng.uniform(0.2, 2.0), rng.uniform(-0.05, 0.08), rng.uniform(0, 0.05), rng.uniform(0.1, 0.5)
        c = np.array([[X0, K, T, r, d, v]])
        tgt = oracle.training_targets(c, 1, 256, 256, seed=11, ordinal0=i)
        put_mc = float(tgt[0, 0].real) / 256  # DC bin / N = mean payoff (gbm_trainer.py:1729-1748)
        ref = oracle.black_put(X0, K, T, r, d, v)
        if ref > 1.0:
            rel.append(abs(put_mc - ref) / ref)
    assert rel and max(rel) < 0.05


def test_black_formula_put_call_parity(oracle) -> None:
    X0, K, T, r, d, v = 100.0, 90.0, 1.3, 0.03, 0.01, 0.4
    put = oracle.black_put(X0, K, T, r, d, v)
    # call by parity must be positive and above intrinsic
    call = put + X0 * math.exp(-d * T) - K * math.exp(-r * T)
    assert call > max(X0 * math.exp(-d * T) - K * math.exp(-r * T), 0.0)
