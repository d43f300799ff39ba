"""The oracle (CPU restatement) pinned against the reference's golden vectors, published
known-answer vectors and closed-form cases.  CPU only."""

from __future__ import annotations

import math
import os

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


MWC_A = 4294883355  # MWC64X multiplier (D. B. Thomas, "The MWC64X random number generator", 2011)


def _mwc64x_reference(seed: int, ordinal: int, group: int, n: int) -> list[int]:
    """The path stream restated in Python integers: Philox4x32-10 (KAT-pinned above) of
    counter (group, ordinal) under key seed gives the MWC64X state (x, c) = (w0, w1 mod-reduced
    below A, absorbing states moved off); each output is x ^ c, then x + c 2^32 <- A x + c."""
    w = (group & 0xFFFFFFFF, group >> 32, ordinal & 0xFFFFFFFF, ordinal >> 32)
    import oracle as _o
    p = _o.philox4x32_10(w, (seed & 0xFFFFFFFF, seed >> 32))
    x, c = p[0], p[1] - MWC_A if p[1] >= MWC_A else p[1]
    if x == 0 and c == 0:
        x = 1
    if x == 0xFFFFFFFF and c == MWC_A - 1:
        x = 0xFFFFFFFE
    out = []
    for _ in range(n):
        out.append(x ^ c)
        t = MWC_A * x + c
        x, c = t & 0xFFFFFFFF, t >> 32
    return out


@pytest.mark.parametrize("seed,ordinal,group", [(7, 0, 0), (7, 3, 16383), (123, 1 << 33, 5), ((1 << 64) - 1, 99, 1 << 40)])
def test_oracle_stream_is_mwc64x(oracle, seed, ordinal, group) -> None:
    got = oracle.stream_u32(seed, ordinal, group, 200)
    assert got.tolist() == _mwc64x_reference(seed, ordinal, group, 200)


@pytest.mark.parametrize("rows", [1, 2, 3])
def test_oracle_stream_span_at_small_t(oracle, rows) -> None:
    """Stream span (smc_rng.h, round 4): at T <= 2 group g (paths 4g .. 4g + 3) takes the (g mod 4)-th run
    of 4 T draws of the stream of g / 4 (one Philox-10 seed per 16 paths); T >= 3: one stream per group.
    Restated here from the raw streams and the f64 Box-Muller pieces: pair k of a group is
    (a, b) -> sqrt(-2 ln u(a)) (cos, sin)(angle(b)); T = 1 takes pairs 0, 1 for paths (0, 1), (2, 3);
    T = 2 one pair per path (z0 -> row 0, z1 -> row 1)."""
    seed, ordinal, cols = 7, 3, 64
    z = oracle.normals(seed, ordinal, rows, cols, "float64")
    for grp in range(cols // 4):
        span = rows <= 2
        words = oracle.stream_u32(seed, ordinal, grp // 4 if span else grp, 64).tolist()
        if span:
            words = words[4 * rows * (grp % 4):]
        pairs = []
        for k in range(0, 2 * (4 if rows >= 2 else 2), 2):
            a, b = words[k], words[k + 1]
            r = math.sqrt(oracle.m2log_u32(a))
            sn, cs = oracle.sincos2pi_u32(b)
            pairs.append((r * cs, r * sn))
        for j in range(4):
            if rows == 1:
                want = pairs[j // 2][j % 2]
                assert z[0, 4 * grp + j] == want, (grp, j)
            else:
                assert (z[0, 4 * grp + j], z[1, 4 * grp + j]) == pairs[j], (grp, j)


def test_oracle_stream_bits_are_uniform(oracle) -> None:
    """Top-23-bit uniforms of 4096 streams x 64 draws (the draws of one C2 chunk): mean, variance and
    lag-1 / cross-stream correlation at the level a 262,144-sample test resolves."""
    u = np.stack([oracle.stream_u32(7, 11, g, 64) for g in range(4096)]).astype(np.float64) / 2.0**32
    assert abs(u.mean() - 0.5) < 3e-3
    assert abs(u.var() - 1.0 / 12.0) < 2e-3
    assert abs(np.corrcoef(u[:, :-1].ravel(), u[:, 1:].ravel())[0, 1]) < 8e-3
    assert abs(np.corrcoef(u[:-1].ravel(), u[1:].ravel())[0, 1]) < 8e-3
    # every bit position (the kernels use bits 9..31) is a fair coin
    bits = np.stack([oracle.stream_u32(7, 11, g, 64) for g in range(4096)]).ravel()
    for b in range(32):
        assert abs(((bits >> b) & 1).mean() - 0.5) < 4e-3, b


def test_f64_uniform_transcendentals_are_accurate(oracle) -> None:
    """The f64 normals' ln / sin / cos of 32-bit uniforms and the f64 recursion's exp (csrc/smc_math.h,
    restated in the oracle) against numpy's libm at the edges of their domains and on random points:
    within 2 ulp (log, exp); sin / cos within 2^-52 absolute of an x87 long-double evaluation of the
    exactly reduced angle.  The angle of b is 2 pi B 2^-32 with B = (b mod 1024) 2^22 + (b >> 10 as a signed
    22-bit integer) mod 2^32 (smc_math.h v4: the low bits pick the table angle); the integer B is reduced to
    the nearest quarter turn before any rounding."""
    two_pi = np.longdouble("6.283185307179586476925286766559005768")

    def sincos_ld(b: int) -> tuple[float, float]:
        y = (b >> 10) - (2**22 if b >= 2**31 else 0)
        b = ((b & 1023) * 2**22 + y) % 2**32
        k = (b + 2**29) // 2**30
        x = two_pi * np.longdouble(b - k * 2**30) / np.longdouble(2**32)
        s_, c_ = np.sin(x), np.cos(x)
        for _ in range(k % 4):
            s_, c_ = c_, -s_
        return float(s_), float(c_)

    rng = np.random.default_rng(5)
    a_vals = [0, 1, 2, 3, 0x7FFFFFFF, 0xB504F333, 0xFFFFFFFE, 0xFFFFFFFF] + [int(x) for x in rng.integers(0, 2**32, 2000)]
    for a in a_vals:
        want = -2.0 * math.log((a + 0.5) / 2.0**32)  # (a + 1/2) 2^-32: exact in double, never 0 or 1
        got = oracle.m2log_u32(a)
        assert abs(got - want) <= 2 * math.ulp(want), a
    for b in [0, 1, 2**29 - 1, 2**29, 2**30, 3 * 2**29, 2**31, 2**32 - 2**29, 2**32 - 1] + \
            [int(x) for x in rng.integers(0, 2**32, 2000)]:
        s, c = oracle.sincos2pi_u32(b)
        ws, wc = sincos_ld(b)
        assert abs(s - ws) <= 2.0**-52 and abs(c - wc) <= 2.0**-52, b
    # 2^(ys / 256): ys / 256 is exact, so libm's 2.0 ** (ys / 256) is the correctly rounded value to 1 ulp
    for ys in [-258000.0, -18000.5, -0.5, -1e-300, 0.0, 1e-12, 0.5, 127.49, 128.0, 18000.0, 258000.0] + \
            list(rng.uniform(-22000, 22000, 2000)):
        want = 2.0 ** (ys / 256.0)
        assert abs(oracle.exp2s_f64(float(ys)) - want) <= 2 * math.ulp(want), ys


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


@pytest.mark.parametrize("scheme", [0, 1])
@pytest.mark.parametrize("T", [1, 5, 16, 33])
def test_reference_math_mode_reproduces_the_reference_arithmetic(oracle, T, scheme) -> None:
    """Kernel mode with MATH_REF (gbm.hip rows_ref_kernel: the f64 engine's step of the portable f32
    normals, state in f64, stores rounded to f32) against the reference mode (gbm.py:224-257's own typing
    under Numba: f64 state, libm exp, f32 stores; pinned to the reference's output by gbm_golden.npz): the
    stored f32 paths agree to the bit except where the two f64 exps (within 2 ulp of each other) round to
    different floats -- none in these 32 x 2048 x T values -- while the f32 recursion differs in most."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"), allow_pickle=False)
    c = oracle.sobol_contracts(7, 0, 32, g["bounds_lower"], g["bounds_upper"])
    P = 2048
    ref, _, _ = oracle.gbm_paths(c, T, P, 7, 3, scheme, "float32", want_paths=True)
    k64, term, rowsum = oracle.kernel_paths(c, T, P, 7, 3, scheme | oracle.MATH_REF, want_paths=True)
    k32, _, _ = oracle.kernel_paths(c, T, P, 7, 3, scheme, want_paths=True)
    fin = np.isfinite(ref)
    assert int(((k64 != ref) & fin).sum()) == 0
    assert ((k32 != ref) & fin).mean() > 0.3
    np.testing.assert_array_equal(term, k64[:, -1])


@pytest.mark.parametrize("scheme", [0, 1])
def test_reference_math_mismatch_rate_at_the_c2_shape(oracle, scheme) -> None:
    """The exception the equality above allows, bounded at C2's per-contract shape (T = 16, P = 65,536, 8
    contracts = 8.4 M stored values): MATH_REF kernel mode against the reference arithmetic differs in at
    most 1e-6 of the values, each by one f32 ulp (measured: 0 for log-Euler, 1 value for simple Euler),
    where the f64 engine's exp (within 2 ulp of libm) and libm's exp round to different floats."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"), allow_pickle=False)
    c = oracle.sobol_contracts(7, 0, 8, g["bounds_lower"], g["bounds_upper"])
    ref, _, _ = oracle.gbm_paths(c, 16, 65536, 7, 3, scheme, "float32", want_paths=True)
    k64, _, _ = oracle.kernel_paths(c, 16, 65536, 7, 3, scheme | oracle.MATH_REF, want_paths=True)
    diff = (k64 != ref) & np.isfinite(ref)
    assert diff.mean() <= 1e-6, int(diff.sum())
    ulps = np.abs(k64.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))[diff]
    assert ulps.size == 0 or int(ulps.max()) == 1

