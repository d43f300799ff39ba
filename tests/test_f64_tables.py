"""The f64 path-math tables (round 3; round-4 v3 forms; round-5 v4 forms): the device header (spectralmc_amd/csrc/smc_f64_tables.h) and
the oracle's copy (oracle/f64_tables.h) hold the same bits, and both are what tools/gen_f64_tables.py
generates (60-digit decimal arithmetic rounded to double), so a hand edit of either breaks parity here
rather than as an unexplained f64 mismatch on the GPU."""

from __future__ import annotations

import importlib.util
import math
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_f64_tables", os.path.join(ROOT, "tools", "gen_f64_tables.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _values(path: str) -> dict[str, list[float]]:
    text = open(path).read()
    out = {}
    for name in ("kF64LogTab", "kF64SinCosTab", "kF64Exp2Tab"):
        body = re.search(name + r"[^=]*=\s*\{(.*?)\n\};", text, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        out[name] = [float.fromhex(t) for t in re.findall(r"-?0x[0-9a-fA-Fp.+-]+", body)]
    return out


def _consts(path: str) -> dict[str, float]:
    return {m.group(1): float.fromhex(m.group(2))
            for m in re.finditer(r"#define (kF64\w+) (-?0x[0-9a-fA-Fp.+-]+)", open(path).read())}


def test_device_and_oracle_tables_hold_the_same_bits() -> None:
    dev = _values(os.path.join(ROOT, "spectralmc_amd", "csrc", "smc_f64_tables.h"))
    orc = _values(os.path.join(ROOT, "oracle", "f64_tables.h"))
    assert dev == orc
    assert [len(dev[k]) for k in ("kF64LogTab", "kF64SinCosTab", "kF64Exp2Tab")] == [1025 * 4, 1024 * 2, 256]
    assert _consts(os.path.join(ROOT, "spectralmc_amd", "csrc", "smc_f64_tables.h")) == \
        _consts(os.path.join(ROOT, "oracle", "f64_tables.h")) == _gen().constants()


def test_tables_are_the_generator_output() -> None:
    log, sc, ex = _gen().tables()
    dev = _values(os.path.join(ROOT, "spectralmc_amd", "csrc", "smc_f64_tables.h"))
    assert dev["kF64LogTab"] == [v for row in log for v in row]
    assert dev["kF64SinCosTab"] == [v for row in sc for v in row]
    assert dev["kF64Exp2Tab"] == ex


def test_table_entries_are_near_libm() -> None:
    """Independent sanity check of the generator against libm (ln and 2^x within 1-2 ulp; sin / cos
    within 2^-50 absolute, which covers the rounding of the double argument 2 pi j / 256 libm is given;
    the tables themselves are the correctly rounded 60-digit values)."""
    log, sc, ex = _gen().tables()
    consts = _gen().constants()
    l2hi, l2lo = -consts["kF64M2Ln2Hi"] / 2, -consts["kF64M2Ln2Lo"] / 2
    assert l2hi == round(l2hi * 2.0**43) / 2.0**43 and abs(l2hi + l2lo - math.log(2)) <= 2 * math.ulp(math.log(2))
    m2hi_c, m2lo_c = consts["kF64M2Ln2Hi"], consts["kF64M2Ln2Lo"]
    for i, (m4inv, hi2, lo2, pad) in zip(range(0, 1025), log):
        # v4 rows: -4 INV (exact scaling), -2 T_HI - 33 (-2 LN2_HI) (exact), -2 T_LO - 33 (-2 LN2_LO) (rounded)
        assert pad == 0.0 and hi2 == round(hi2 * 2.0**42) / 2.0**42 and abs(hi2) < 64
        m2hi = hi2 + 33 * m2hi_c
        assert m2hi - 33 * m2hi_c == hi2  # exact both ways
        m2lo = lo2 + 33 * m2lo_c
        inv, hi, lo = -m4inv / 4, -m2hi / 2, -m2lo / 2
        assert inv == 1.0 / (1.0 + i / 1024.0)
        assert hi == round(hi * 2.0**43) / 2.0**43  # k LN2_HI + T_HI exact for |k| <= 33
        # (i = 0: T = 0; the LO entry's one rounding leaves |lo| <= 2^-85)
        assert abs((hi + lo) - (-math.log(inv))) <= 2 * math.ulp(max(abs(hi), 1e-300)) if hi else abs(lo) <= 2.0**-85
        assert abs(lo) <= 2.0**-43 + 2.0**-80
    # c = 2: T = ln 2 exactly as LN2_HI + LN2_LO, so at e = 32 both sums vanish exactly
    assert log[1024][1] == -32 * m2hi_c and log[1024][2] == -32 * m2lo_c
    for j, (s, c) in enumerate(sc):
        assert abs(s - math.sin(2 * math.pi * j / 1024)) <= 2 ** -50
        assert abs(c - math.cos(2 * math.pi * j / 1024)) <= 2 ** -50
    for j, v in enumerate(ex):
        assert abs(v - 2.0 ** (j / 256)) <= math.ulp(v)
    for k in range(1, 5):  # (ln 2 / 256)^k / k!
        assert abs(consts[f"kF64ExpE{k}"] - (math.log(2) / 256) ** k / math.factorial(k)) <= \
            2 * math.ulp(consts[f"kF64ExpE{k}"])
    K = 2 * math.pi / 2.0**32  # sin / cos coefficients in integer angle units
    for name, want in (("kF64SinS1", K), ("kF64SinS3", -K**3 / 6), ("kF64SinS5", K**5 / 120),
                       ("kF64CosC2", -K**2 / 2), ("kF64CosC4", K**4 / 24)):
        assert abs(consts[name] - want) <= 4 * math.ulp(want), name
