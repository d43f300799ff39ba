"""The f64 path-math tables (round 3; round-4 sizes): the device header (spectralmc_amd/csrc/smc_f64_tables.h) and
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


def test_device_and_oracle_tables_hold_the_same_bits() -> None:
    dev = _values(os.path.join(ROOT, "spectralmc_amd", "csrc", "smc_f64_tables.h"))
    orc = _values(os.path.join(ROOT, "oracle", "f64_tables.h"))
    assert dev == orc
    assert [len(dev[k]) for k in ("kF64LogTab", "kF64SinCosTab", "kF64Exp2Tab")] == [256 * 3, 1024 * 2, 64]


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
    for i, (inv, hi, lo) in zip(range(-128, 128), log):
        assert inv == 1.0 / (1.0 + i / 256.0)
        assert abs(hi - (-math.log(inv))) <= 2 * math.ulp(max(abs(hi), 1e-300))
        assert abs(lo) <= math.ulp(hi) if hi != 0.0 else lo == 0.0
    for j, (s, c) in enumerate(sc):
        assert abs(s - math.sin(2 * math.pi * j / 1024)) <= 2 ** -50
        assert abs(c - math.cos(2 * math.pi * j / 1024)) <= 2 ** -50
    for j, v in enumerate(ex):
        assert abs(v - 2.0 ** (j / 64)) <= math.ulp(v)
