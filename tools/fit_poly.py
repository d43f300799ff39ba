"""Fit the f32 polynomial coefficients of the portable transcendental kernels
(spectralmc_amd/csrc/smc_math.h, mirrored in oracle/gbm_oracle.c).

Weighted least squares on Chebyshev nodes in f64 (near-minimax), coefficients rounded to
f32, error measured by evaluating the rounded polynomial with f32 Horner/fma emulation.
Usage: python tools/fit_poly.py
"""
import numpy as np


def f32(x):
    return np.float32(x)


def fma32(a, b, c):
    # exact product of two f32 fits in f64; one rounding of the sum to f32 (double rounding is
    # negligible for an error estimate)
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def horner32(coeffs, x):
    acc = np.float32(coeffs[-1])
    for c in coeffs[-2::-1]:
        acc = fma32(acc, x, np.float32(c))
    return acc


def fit(fn, lo, hi, basis_powers, weight, n=4000):
    k = np.arange(n)
    x = 0.5 * (lo + hi) + 0.5 * (hi - lo) * np.cos(np.pi * (k + 0.5) / n)
    A = np.stack([x ** p for p in basis_powers], axis=1)
    w = weight(x)
    coef, *_ = np.linalg.lstsq(A * w[:, None], fn(x) * w, rcond=None)
    return coef


def main():
    # ln(1+f) = f * q(f), f in [sqrt(1/2)-1, sqrt(2)-1]
    lo, hi = np.sqrt(0.5) - 1, np.sqrt(2.0) - 1
    c = fit(lambda f: np.where(f == 0, 1.0, np.log1p(f) / np.where(f == 0, 1, f)), lo, hi, range(9),
            lambda f: np.ones_like(f))
    c32 = [f32(v) for v in c]
    xs = np.linspace(lo, hi, 200001).astype(np.float32)
    got = np.array([np.float32(x) * horner32(c32, x) for x in xs[::50]])
    ref = np.log1p(xs[::50].astype(np.float64))
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)
    print("LOG1P_Q =", [float(v) for v in c32], "max rel err", err[np.abs(ref) > 1e-6].max())

    # sin(2 pi r) = r * s(r^2), cos(2 pi r) = c(r^2), r in [-1/8, 1/8]
    u = lambda r: r * r  # noqa: E731
    cs = fit(lambda r: np.sin(2 * np.pi * r) / np.where(r == 0, 1, r), 0, 0.125, [0, 2, 4, 6, 8],
             lambda r: np.ones_like(r))
    cc = fit(lambda r: np.cos(2 * np.pi * r), 0, 0.125, [0, 2, 4, 6, 8], lambda r: np.ones_like(r))
    s32 = [f32(v) for v in cs]
    k32 = [f32(v) for v in cc]
    rs = np.linspace(-0.125, 0.125, 20001).astype(np.float32)
    gs = np.array([np.float32(r) * horner32(s32, np.float32(r * r)) for r in rs])
    gc = np.array([horner32(k32, np.float32(r * r)) for r in rs])
    print("SIN2PI_S =", [float(v) for v in s32], "max abs err", np.abs(gs - np.sin(2 * np.pi * rs.astype(np.float64))).max())
    print("COS2PI_C =", [float(v) for v in k32], "max abs err", np.abs(gc - np.cos(2 * np.pi * rs.astype(np.float64))).max())

    # 2^f, f in [-1/2, 1/2]
    ce = fit(lambda f: 2.0 ** f, -0.5, 0.5, range(7), lambda f: 2.0 ** -f)
    e32 = [f32(v) for v in ce]
    fs = np.linspace(-0.5, 0.5, 20001).astype(np.float32)
    ge = np.array([horner32(e32, f) for f in fs])
    print("EXP2_P =", [float(v) for v in e32], "max rel err", (np.abs(ge - 2.0 ** fs.astype(np.float64)) / 2.0 ** fs).max())


if __name__ == "__main__":
    main()
