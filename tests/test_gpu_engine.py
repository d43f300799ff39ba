"""HIP engine parity: every kernel through the C ABI vs the oracle (CPU restatement) on the
same seeded inputs.  Bit-exact for integer/index work (Sobol, Philox-seeded streams via the
normals they produce within float tolerance), fp tolerances stated per test."""

from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from spectralmc_amd import _lib
from spectralmc_amd.sobol_sampler import SobolEngine, draw_device
from tests.helpers import assert_rows_equal, poisoned, poisoned_like

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _L():
    return _lib.lib()


def _contracts(oracle, golden, n: int, seed: int = 7, skip: int = 0) -> np.ndarray:
    return oracle.sobol_contracts(seed, skip, n, golden["bounds_lower"], golden["bounds_upper"])


def _norm_rel(a: np.ndarray, b: np.ndarray, floor: float = 0.0) -> float:
    den = max(float(np.linalg.norm(b)), floor)
    return float(np.linalg.norm(a - b)) / den if den > 0 else float(np.linalg.norm(a - b))


def _assert_close(got: np.ndarray, want: np.ndarray, tol: float) -> None:
    """Batch norm-relative error below tol; a failure names the worst contracts (row, row mod 8, rel)."""
    rel = _norm_rel(got, want)
    if rel < tol:
        return
    g = got.reshape(got.shape[0], -1) if got.ndim > 1 else got[None]
    w = want.reshape(want.shape[0], -1) if want.ndim > 1 else want[None]
    per = np.linalg.norm(g - w, axis=1) / max(float(np.linalg.norm(w)), 1e-300)
    worst = np.argsort(per)[::-1][:12]
    raise AssertionError(f"batch norm-relative error {rel:.3e} >= {tol}; worst rows (row, row mod 8, share): "
                         f"{[(int(i), int(i) % 8, float(per[i])) for i in worst]}")


# ------------------------------------------------------------------------------ Sobol
@pytest.mark.parametrize("seed", [7, 31, 42, 123])
@pytest.mark.parametrize("skip", [0, 8, 4096])
def test_device_sobol_bit_exact(golden, seed, skip) -> None:
    eng = SobolEngine(6, seed, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    out = poisoned((96, 6), torch.float64, DEV)
    out32 = poisoned((96, 6), torch.float32, DEV)
    idx = torch.tensor([skip], dtype=torch.int64, device=DEV)
    draw_device(tables, 6, idx, 0, 96, lo, hi, out, out32)
    torch.cuda.synchronize()
    want = np.concatenate([golden[f"sobol_s{seed}_k{skip}"], golden[f"sobol_s{seed}_k{skip}_next"]])
    assert_rows_equal(out.cpu().numpy(), want)
    assert_rows_equal(out32.cpu().numpy(), want.astype(np.float32))


def test_device_sobol_far_index_matches_host() -> None:
    start = (1 << 29) + 12345
    eng = SobolEngine(6, 99, start)
    host = eng.random(1000)
    tables = torch.from_numpy(SobolEngine(6, 99).tables().view(np.int32)).to(DEV)
    lo = torch.zeros(6, dtype=torch.float64, device=DEV)
    hi = torch.ones(6, dtype=torch.float64, device=DEV)
    out = poisoned((1000, 6), torch.float64, DEV)
    draw_device(tables, 6, None, start, 1000, lo, hi, out)
    torch.cuda.synchronize()
    assert_rows_equal(out.cpu().numpy(), host)


# ------------------------------------------------------------------------------ RNG
@pytest.mark.parametrize("rows", [17, 1, 2])
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_normals_match_oracle(oracle, dtype, rows) -> None:
    """f32: bit-exact (portable Box-Muller); f64: the table-driven f64 math restated, 1e-12 (bit-exact in
    practice).  rows 1, 2: the stream span of small T (4 groups per Philox-seeded stream)."""
    cols = 5003
    tdt = torch.float32 if dtype == "float32" else torch.float64
    z = poisoned((rows, cols), tdt, DEV)
    _lib.check(_L().smc_normals(7, 5, rows, cols, 0 if dtype == "float32" else 1, _lib.ptr(z), None))
    torch.cuda.synchronize()
    want = oracle.normals(7, 5, rows, cols, dtype)
    got = z.cpu().numpy()
    if dtype == "float32":
        assert_rows_equal(got, want)
    else:
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-12 * np.abs(want).max())
    assert abs(float(got.mean())) < 0.02 and abs(float(got.std()) - 1) < 0.02


# ------------------------------------------------------------------------------ paths
PATH_CASES = [
    # (T, P, scheme, dtype)
    (16, 1024, 0, "float32"),     # T specialised kernel, C1 paths
    (16, 3000, 1, "float32"),     # simple Euler, ragged last chunk
    (16, 4096, 0, "float32"),     # straight-line 16-row block, two full chunks, all row sums
    (16, 4096, 0, "float64"),     # the same block in f64
    (1, 513, 0, "float32"),       # T = 1, P % 4 != 0 -> scalar stores
    (20, 4196, 0, "float32"),     # two row blocks (16 + 4), ragged paths
    (100, 64, 1, "float32"),      # seven row blocks with step replay
    (7, 4096, 0, "float64"),      # generic T, f64
    (100, 64, 1, "float64"),      # long generic T, tiny P
]


@pytest.mark.parametrize("T,P,scheme,dtype", PATH_CASES)
def test_paths_match_oracle(oracle, golden, T, P, scheme, dtype) -> None:
    c = _contracts(oracle, golden, 6)
    c[:, 2] = np.minimum(c[:, 2], 3.0)  # keep the extreme-variance corner out of a 1e-5 check
    tdt = torch.float32 if dtype == "float32" else torch.float64
    cd = torch.from_numpy(c).to(DEV)
    paths = poisoned((6, T, P), tdt, DEV)
    rowsum = poisoned((6, T), torch.float64, DEV)
    _lib.check(_L().smc_gbm_simulate(_lib.ptr(cd), 6, T, P, 7, None, 3, scheme, 0 if dtype == "float32" else 1,
                                     _lib.ptr(paths), _lib.ptr(rowsum), None))
    torch.cuda.synchronize()
    got = paths.cpu().numpy()
    if dtype == "float32":  # bit-exact vs the kernel-mode restatement
        kp, _, krs = oracle.kernel_paths(c, T, P, 7, ordinal0=3, scheme=scheme, want_paths=True)
        assert_rows_equal(got, kp)
        assert_rows_equal(rowsum.cpu().numpy(), krs)
    # reference semantics (Numba kernel: f64 recursion, dtype stores), stated tolerance
    want, _, want_rs = oracle.gbm_paths(c, T, P, 7, ordinal0=3, scheme=scheme, dtype=dtype, want_paths=True)
    tol = 2e-5 if dtype == "float32" else 1e-11
    for b in range(6):
        assert _norm_rel(got[b], want[b]) < tol, b
    np.testing.assert_allclose(rowsum.cpu().numpy(), want_rs, rtol=5 * tol)


def test_zero_vol_and_zero_maturity_exact() -> None:
    c = torch.tensor([[100.0, 95.0, 2.0, 0.05, 0.01, 0.0], [50.0, 40.0, 0.0, 0.1, 0.0, 0.7]],
                     dtype=torch.float64, device=DEV)
    T, P = 8, 256
    paths = poisoned((2, T, P), torch.float64, DEV)
    _lib.check(_L().smc_gbm_simulate(_lib.ptr(c), 2, T, P, 7, None, 0, 0, 1, _lib.ptr(paths), None, None))
    torch.cuda.synchronize()
    p = paths.cpu().numpy()
    t = np.linspace(2.0 / T, 2.0, T)
    np.testing.assert_allclose(p[0], np.broadcast_to((100 * np.exp(0.04 * t))[:, None], (T, P)), rtol=1e-13)
    assert np.all(p[1] == 50.0)


# ------------------------------------------------------------------------------ CF targets
TARGET_CASES = [
    # (B, T, N, M, scheme, normalize, dtype)
    (64, 16, 256, 4, 0, 1, "float32"),    # C1
    (8, 16, 128, 4, 0, 1, "float32"),     # e2e test shape
    (16, 1, 16, 256, 0, 1, "float32"),    # T = 1, many batches
    (5, 5, 100, 7, 1, 1, "float32"),      # non power-of-two N, simple Euler
    (4, 3, 1024, 2, 0, 0, "float32"),     # N > workgroup, RAW
    (6, 16, 64, 16, 0, 1, "float64"),     # f64
]


def _run_targets(c: np.ndarray, T: int, N: int, M: int, scheme: int, normalize: int, dtype: str, store: int,
                 chunk: int | None = None, ordinal0: int = 0, with_rowsum: bool = True, flags: int = 0,
                 pitch: int | None = None, sliced: bool = False, workspace: torch.Tensor | None = None):
    B = c.shape[0]
    P = N * M
    tdt = torch.float32 if dtype == "float32" else torch.float64
    cdt = torch.complex64 if dtype == "float32" else torch.complex128
    cd = torch.from_numpy(c).to(DEV)
    chunk = chunk or B
    pitch = pitch or P
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, tdt, DEV)
    rowsum = poisoned((B, T), torch.float64, DEV)
    tg = poisoned((B, N), cdt, DEV)
    wsb = int(_L().smc_engine_workspace_bytes(chunk, T, P, int(with_rowsum))) if sliced else 0
    if sliced and workspace is None:
        workspace = torch.zeros(max(wsb, 8), dtype=torch.uint8, device=DEV)
    _lib.check(_L().smc_train_targets(_lib.ptr(cd), B, T, N, M, 7, None, ordinal0, scheme | flags, normalize,
                                      0 if dtype == "float32" else 1, store, _lib.ptr(paths), pitch, chunk,
                                      _lib.ptr(rowsum) if with_rowsum else None, _lib.ptr(tg),
                                      _lib.ptr(workspace) if sliced else None, wsb, None))
    torch.cuda.synchronize()
    return tg.cpu().numpy(), rowsum.cpu().numpy(), paths[..., :P]


@pytest.mark.parametrize("B,T,N,M,scheme,normalize,dtype", TARGET_CASES)
def test_targets_match_oracle(oracle, golden, B, T, N, M, scheme, normalize, dtype) -> None:
    c = _contracts(oracle, golden, B, seed=31)
    got, rowsum, _ = _run_targets(c, T, N, M, scheme, normalize, dtype, _lib.STORE_ALL, ordinal0=11)
    if dtype == "float32":  # the f32 engine is restated exactly: bit-identical targets
        kt, krs = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=11, scheme=scheme, normalize=bool(normalize))
        assert_rows_equal(rowsum, krs)
        assert_rows_equal(got, kt)
    # reference semantics (f64 path recursion as the Numba kernel; FFT per batch then mean):
    # whole-batch norm-relative error <= 1e-5 (f32) / 1e-10 (f64)
    want = oracle.training_targets(c, T, N, M, seed=7, ordinal0=11, scheme=scheme, normalize=bool(normalize),
                                   dtype=dtype)
    tol = 1e-5 if dtype == "float32" else 1e-10
    _assert_close(got, want, tol)


SLICED_CASES = [
    # (B, T, N, M, scheme, normalize, dtype): P > 8192, so a contract runs as several workgroups
    (3, 16, 256, 64, 0, 1, "float32"),    # 2 whole slices
    (3, 20, 100, 250, 0, 1, "float32"),   # 4 slices, ragged last chunk, T > 16 (row-block replay)
    (2, 4, 99, 101, 1, 1, "float32"),     # P % 4 != 0: every chunk masked; simple Euler
    (2, 16, 1024, 24, 0, 0, "float32"),   # N > workgroup, RAW, 3 slices
]


@pytest.mark.parametrize("B,T,N,M,scheme,normalize,dtype", SLICED_CASES)
@pytest.mark.parametrize("with_rowsum", [True, False])
def test_sliced_contracts_match_oracle(oracle, golden, B, T, N, M, scheme, normalize, dtype, with_rowsum) -> None:
    """Several workgroups per contract + last-arriver CF phase: bit-identical to the oracle's
    sliced reduction order, run-to-run identical, counters left at zero."""
    c = _contracts(oracle, golden, B, seed=42)
    P = N * M
    wsb = int(_L().smc_engine_workspace_bytes(B, T, P, int(with_rowsum)))
    assert wsb > 0
    ws = torch.zeros(wsb, dtype=torch.uint8, device=DEV)
    got, rowsum, _ = _run_targets(c, T, N, M, scheme, normalize, dtype, _lib.STORE_ALL, ordinal0=5,
                                  with_rowsum=with_rowsum, sliced=True, workspace=ws)
    kt, krs = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=5, scheme=scheme, normalize=bool(normalize),
                                    sliced=True)
    assert_rows_equal(got, kt)
    if with_rowsum:
        assert_rows_equal(rowsum, krs)
    assert int(ws[-4 * (B + 16):].view(torch.int32).abs().sum()) == 0  # arrival + queue counters reset
    again, _, _ = _run_targets(c, T, N, M, scheme, normalize, dtype, _lib.STORE_TERMINAL, ordinal0=5,
                               with_rowsum=with_rowsum, sliced=True, workspace=ws)
    assert_rows_equal(again, got)
    # unsliced: same paths, row sums associated differently -> targets within f32 rounding
    flat, _, _ = _run_targets(c, T, N, M, scheme, normalize, dtype, _lib.STORE_ALL, ordinal0=5,
                              with_rowsum=with_rowsum)
    _assert_close(got, flat, 1e-6)


def test_sliced_f64_and_chunked_launches(oracle, golden) -> None:
    """f64 sliced engine within the reference tolerance; several launches share one workspace."""
    c = _contracts(oracle, golden, 5, seed=7)
    got, _, _ = _run_targets(c, 16, 128, 80, 0, 1, "float64", _lib.STORE_ALL, sliced=True)
    want = oracle.training_targets(c, 16, 128, 80, seed=7, dtype="float64")
    _assert_close(got, want, 1e-10)
    a, _, _ = _run_targets(c, 16, 256, 40, 0, 1, "float32", _lib.STORE_ALL, sliced=True)
    b, _, _ = _run_targets(c, 16, 256, 40, 0, 1, "float32", _lib.STORE_ALL, sliced=True, chunk=2)
    assert_rows_equal(a, b)


ROWS_CASES = [  # (B, T, N, M, scheme, normalize, dtype, store, hw): shapes rows_kernel + cf_kernel take
    (7, 17, 2048, 32, 0, 1, "float32", _lib.STORE_ALL, 0),    # f32, T != 16, N > 1024
    (6, 17, 2048, 32, 0, 1, "float32", _lib.STORE_ALL, 1),    # the same in hw math
    (5, 16, 64, 64, 0, 1, "float64", _lib.STORE_ALL, 0),      # f64 (any f64 shape with whole chunks)
    (5, 5, 128, 32, 1, 0, "float64", _lib.STORE_TERMINAL, 0),  # f64, odd T, simple Euler, RAW, terminal rows
    (3, 33, 64, 64, 0, 1, "float64", _lib.STORE_ALL, 0),      # f64, T > 16
]


@pytest.mark.parametrize("B,T,N,M,scheme,normalize,dtype,store,hw", ROWS_CASES)
def test_rows_kernel_matches_oracle_and_contract_kernel(oracle, golden, B, T, N, M, scheme, normalize, dtype, store,
                                                        hw) -> None:
    """rows_kernel + cf_kernel (persistent, every row in registers, terminal sum through the row
    padding): f32 portable bit-exact with the kernel-mode oracle (512-lane order) and hw within 1e-5 of
    the reference mode; f64 within 1e-10 of the reference mode (its exp differs from libm by <= 2 ulp)
    and bit-identical to contract_kernel at an unpadded pitch (same paths, same reduction order)."""
    c = _contracts(oracle, golden, B, seed=3)
    P = N * M
    dcode = 0 if dtype == "float32" else 1
    pitch = int(_L().smc_path_pitch(P, dcode))
    assert _L().smc_train_targets_kernel(T, N, P, dcode, pitch, 0) == b"rows_kernel+cf_kernel"
    flags = _lib.MATH_HW if hw else 0
    got, _, paths = _run_targets(c, T, N, M, scheme, normalize, dtype, store, ordinal0=9, with_rowsum=False,
                                 flags=flags, pitch=pitch)
    want = oracle.training_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme, normalize=bool(normalize),
                                   dtype=dtype)
    _assert_close(got, want, (1e-5 if dtype == "float32" else 1e-10))
    if dtype == "float32" and not hw:
        kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme, normalize=bool(normalize))
        assert_rows_equal(got, kt)
    if dtype == "float64":
        assert _L().smc_train_targets_kernel(T, N, P, dcode, 0, 0) == b"contract_kernel"
        ref, _, ref_paths = _run_targets(c, T, N, M, scheme, normalize, dtype, store, ordinal0=9, with_rowsum=False)
        assert_rows_equal(got, ref)
        assert_rows_equal(paths.cpu().numpy(), ref_paths.cpu().numpy())


MANY_CONTRACT_CASES = [
    # (B, T, N, M, scheme, normalize): more contracts than the resident grid (512 workgroups on
    # MI355X), so the one-workgroup-per-contract launch runs several rounds
    (600, 16, 128, 16, 0, 1),
    (1100, 5, 256, 8, 1, 1),     # T < 16, simple Euler
    (520, 16, 2048, 2, 0, 0),    # N = 2048 (4 x the workgroup: 4-column quads), RAW
    (513, 16, 4, 1024, 0, 1),    # N = 4
]


@pytest.mark.parametrize("B,T,N,M,scheme,normalize", MANY_CONTRACT_CASES)
@pytest.mark.parametrize("store", [_lib.STORE_ALL, _lib.STORE_TERMINAL])
def test_multi_round_launches_match_oracle(oracle, golden, B, T, N, M, scheme, normalize, store) -> None:
    c = _contracts(oracle, golden, B, seed=7, skip=3)
    got, _, _ = _run_targets(c, T, N, M, scheme, normalize, "float32", store, ordinal0=9, with_rowsum=False)
    kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme, normalize=bool(normalize),
                                  wg=oracle.engine_wg(T, N, N * M, normalize=bool(normalize)))
    assert_rows_equal(got, kt)
    # padded pitch and chunked launches: same bits
    pitch = int(_L().smc_path_pitch(N * M, 0))
    again, _, _ = _run_targets(c, T, N, M, scheme, normalize, "float32", store, ordinal0=9, with_rowsum=False,
                               pitch=pitch, chunk=B // 2 + 1)
    assert_rows_equal(again, kt, "padded pitch, two chunk launches", chunk=B // 2 + 1)


def test_store_modes_and_chunking_bit_identical(oracle, golden) -> None:
    c = _contracts(oracle, golden, 12, seed=42)
    a, rs_a, _ = _run_targets(c, 16, 64, 8, 0, 1, "float32", _lib.STORE_ALL)
    b, rs_b, _ = _run_targets(c, 16, 64, 8, 0, 1, "float32", _lib.STORE_TERMINAL)
    d, rs_d, _ = _run_targets(c, 16, 64, 8, 0, 1, "float32", _lib.STORE_ALL, chunk=5)
    assert_rows_equal(a, b)
    assert_rows_equal(a, d)
    assert_rows_equal(rs_a, rs_b)
    assert_rows_equal(rs_a, rs_d)
    # run-to-run determinism (fixed-order reductions, no atomics)
    e, _, _ = _run_targets(c, 16, 64, 8, 0, 1, "float32", _lib.STORE_ALL)
    assert_rows_equal(a, e)


@pytest.mark.parametrize("store", [_lib.STORE_ALL, _lib.STORE_TERMINAL])
def test_padded_row_pitch_bit_identical(oracle, golden, store) -> None:
    """A padded scratch pitch (smc_path_pitch, or any multiple of 4 >= P) changes nothing."""
    c = _contracts(oracle, golden, 9, seed=7)
    P = 64 * 8
    a, rs_a, pa = _run_targets(c, 20, 64, 8, 0, 1, "float32", store)
    for pitch in (int(_L().smc_path_pitch(P, 0)), P + 4, P + 1024):
        b, rs_b, pb = _run_targets(c, 20, 64, 8, 0, 1, "float32", store, chunk=4, pitch=pitch)
        assert_rows_equal(a, b)
        assert_rows_equal(rs_a, rs_b)
        if store == _lib.STORE_ALL:  # last chunk of 4 holds contracts 8.. of 9 in slot 0
            torch.testing.assert_close(pb[0], pa[8], rtol=0, atol=0)


def test_cf_targets_from_stored_paths_equal_fused(oracle, golden) -> None:
    c = _contracts(oracle, golden, 7, seed=123)
    T, N, M = 16, 32, 8
    fused, rowsum, paths = _run_targets(c, T, N, M, 0, 1, "float32", _lib.STORE_ALL)
    cd = torch.from_numpy(c).to(DEV)
    rs = torch.from_numpy(rowsum).to(DEV)
    tg = poisoned((7, N), torch.complex64, DEV)
    _lib.check(_L().smc_cf_targets(_lib.ptr(cd), 7, T, N, M, 1, 0, _lib.ptr(paths), _lib.ptr(rs), _lib.ptr(tg), None))
    torch.cuda.synchronize()
    assert_rows_equal(tg.cpu().numpy(), fused)


def test_partition_invariance_of_ordinals(oracle, golden) -> None:
    """Contract b of a batch starting at ordinal o equals contract 0 of a batch at o + b
    (the property the data-parallel shard relies on)."""
    c = _contracts(oracle, golden, 8, seed=7)
    full, _, _ = _run_targets(c, 16, 32, 4, 0, 1, "float32", _lib.STORE_ALL, ordinal0=100)
    part, _, _ = _run_targets(c[5:], 16, 32, 4, 0, 1, "float32", _lib.STORE_ALL, ordinal0=105)
    assert_rows_equal(full[5:], part)


def test_fft_linearity_property(oracle, golden) -> None:
    """Size-independent check at a large shape: DC bin / N = discounted mean payoff, and the
    spectrum of a real signal is Hermitian."""
    c = _contracts(oracle, golden, 32, seed=7)
    got, _, _ = _run_targets(c, 16, 256, 256, 0, 1, "float32", _lib.STORE_TERMINAL)
    np.testing.assert_allclose(got[:, 1:], np.conj(got[:, :0:-1]), rtol=1e-6, atol=1e-3)
    assert np.all(got[:, 0].real >= 0) and np.allclose(got[:, 0].imag, 0.0)


def test_terminal_only_row_sum_mode_identical(oracle, golden) -> None:
    """Training passes rowsum=NULL (terminal-row sum only, kept on chip): same targets, same bits."""
    c = _contracts(oracle, golden, 9, seed=7)
    for T in (16, 20):
        a, _, _ = _run_targets(c, T, 64, 8, 0, 1, "float32", _lib.STORE_ALL)
        b, _, _ = _run_targets(c, T, 64, 8, 0, 1, "float32", _lib.STORE_ALL, with_rowsum=False)
        assert_rows_equal(a, b)


@pytest.mark.parametrize("scheme", [0, 1])
def test_hw_math_mode_within_fp32_tolerance(oracle, golden, scheme) -> None:
    """SMC_MATH_HW (hardware transcendentals): not bit-reproducible; the reference-semantics
    targets agree to 1e-5 norm-relative over the batch and the normals to ~1e-5 absolute."""
    c = _contracts(oracle, golden, 32, seed=31)
    got, _, _ = _run_targets(c, 16, 256, 4, scheme, 1, "float32", _lib.STORE_ALL, flags=_lib.MATH_HW)
    want = oracle.training_targets(c, 16, 256, 4, seed=7, scheme=scheme)
    _assert_close(got, want, 1e-5)
    z = poisoned((16, 4096), torch.float32, DEV)
    _lib.check(_L().smc_normals(7, 3, 16, 4096, _lib.DTYPE_F32 | _lib.MATH_HW, _lib.ptr(z), None))
    torch.cuda.synchronize()
    np.testing.assert_allclose(z.cpu().numpy(), oracle.normals(7, 3, 16, 4096), rtol=0, atol=2e-5)


RESIDENT_CASES = [
    # (B, N, M, store): resident_kernel shapes (T = 16, 4096 | P <= 65,536, N | 4096, N <= 1024)
    (300, 256, 256, _lib.STORE_ALL),      # C2 per-contract shape, > 1 contract on some workgroups
    (40, 64, 64, _lib.STORE_ALL),         # one chunk (all terminal values in LDS), B < #CUs
    (33, 1024, 16, _lib.STORE_TERMINAL),  # 4 chunks, G = 4, terminal-only scratch
    (17, 4, 2048, _lib.STORE_ALL),        # N = 4: one column quad, G = 1024
    (9, 512, 96, _lib.STORE_ALL),         # 12 chunks: 8 in LDS + 4 in registers
]


@pytest.mark.parametrize("B,N,M,store", RESIDENT_CASES)
def test_resident_kernel_bit_exact(oracle, golden, B, N, M, store) -> None:
    """resident_kernel (terminal rows kept on chip, no re-read): portable math bit-exact with the
    kernel-mode oracle in 1024-lane order, hw math within 1e-5 of the reference-mode targets."""
    P = N * M
    pitch = int(_L().smc_path_pitch(P, 0))
    assert _L().smc_train_targets_kernel(16, N, P, 0, pitch, 0) == b"resident_kernel"
    assert oracle.engine_wg(16, N, P) == 1024
    c = _contracts(oracle, golden, B, seed=42, skip=11)
    got, _, _ = _run_targets(c, 16, N, M, 0, 1, "float32", store, ordinal0=21, with_rowsum=False, pitch=pitch)
    kt, _ = oracle.kernel_targets(c, 16, N, M, seed=7, ordinal0=21, wg=1024)
    assert_rows_equal(got, kt)
    hw, _, _ = _run_targets(c, 16, N, M, 0, 1, "float32", store, ordinal0=21, with_rowsum=False, pitch=pitch,
                            flags=_lib.MATH_HW)
    want = oracle.training_targets(c, 16, N, M, seed=7, ordinal0=21)
    _assert_close(hw, want, 1e-5)
    # contiguous rows (pitch = P) and launches of a few contracts: same bits
    again, _, _ = _run_targets(c, 16, N, M, 0, 1, "float32", store, ordinal0=21, with_rowsum=False,
                               chunk=max(1, B // 3))
    assert_rows_equal(again, kt)


# ------------------------------------------------------------------------------ fused step
STEP_CASES = [  # (B, T, N, M, math, store, chunk): resident shapes (fused launch) and fallback shapes
    (None, 16, 256, 256, _lib.MATH_HW, _lib.STORE_ALL, None),   # C2 per-contract shape, 2 rounds + 3
    (37, 16, 64, 64, 0, _lib.STORE_TERMINAL, None),             # resident, portable math, terminal rows
    (37, 16, 64, 64, 0, _lib.STORE_ALL, 10),                    # resident, four chunk launches per step
    (9, 5, 64, 4, 0, _lib.STORE_ALL, None),                     # T != 16: contract_kernel fallback
    (7, 16, 1000, 4, 0, _lib.STORE_ALL, None),                  # N does not divide 4096: split pair fallback
]


def _sync(L, T, N, M, pitch):
    n = int(L.smc_train_step_sync_bytes(T, N, M, _lib.DTYPE_F32, pitch))
    assert n > 0
    return torch.zeros(n, dtype=torch.uint8, device=DEV), n


@pytest.mark.parametrize("B,T,N,M,math,store,chunk", STEP_CASES)
def test_train_step_equals_draw_then_targets(golden, B, T, N, M, math, store, chunk) -> None:
    """smc_train_step (Sobol draw + targets + cursor advance; one resident_kernel launch per chunk
    where the shape allows) is bit-identical to smc_sobol_draw + smc_train_targets + the cursor
    update, over three consecutive steps of a rank-1-of-2 shard; the sync area is left zeroed."""
    L = _L()
    if B is None:
        B = 2 * torch.cuda.get_device_properties(0).multi_processor_count + 3
    chunk = chunk or B
    P = N * M
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    pitch = int(L.smc_path_pitch(P, 0))
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, torch.float32, DEV)
    scheme = _lib.SCHEME_LOG_EULER | math
    offset, adv = B, 2 * B  # rank 1 of 2
    cur_a = torch.tensor([100, 50], dtype=torch.int64, device=DEV)
    cur_b = cur_a.clone()
    sync, nsync = _sync(L, T, N, M, pitch)
    assert nsync == 128  # whole-contract shapes: done counter, status word, contract queue
    for _ in range(3):
        ca = poisoned((B, 6), torch.float64, DEV)
        fa = poisoned((B, 6), torch.float32, DEV)
        ta = poisoned((B, N), torch.complex64, DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur_a), offset, adv,
                                    _lib.ptr(ca), _lib.ptr(fa), B, T, N, M, 7, scheme, _lib.NORM_NORMALIZE,
                                    _lib.DTYPE_F32, store, _lib.ptr(paths), pitch, chunk, _lib.ptr(ta),
                                    _lib.ptr(sync), nsync, None))
        cb = poisoned_like(ca)
        fb = poisoned_like(fa)
        tb = poisoned_like(ta)
        draw_device(tables, 6, cur_b[0:1], offset, B, lo, hi, cb, fb)
        _lib.check(L.smc_train_targets(_lib.ptr(cb), B, T, N, M, 7, _lib.ptr(cur_b[1:2]), offset, scheme,
                                       _lib.NORM_NORMALIZE, _lib.DTYPE_F32, store, _lib.ptr(paths), pitch, chunk,
                                       None, _lib.ptr(tb), None, 0, None))
        cur_b.add_(adv)
        torch.cuda.synchronize()
        assert_rows_equal(ca.cpu().numpy(), cb.cpu().numpy())
        assert_rows_equal(fa.cpu().numpy(), fb.cpu().numpy())
        assert_rows_equal(ta.cpu().numpy(), tb.cpu().numpy())
        assert cur_a.tolist() == cur_b.tolist()
        assert not sync.view(torch.int32).any()  # done counter, status word and contract queue


ROWS_STEP_CASES = [  # (B, T, N, M, dtype, store, chunk): smc_train_step shapes on rows_kernel + cf_kernel
    (None, 16, 64, 64, _lib.DTYPE_F64, _lib.STORE_ALL, None),      # f64, > 4 contracts per workgroup slot
    (2500, 5, 32, 64, _lib.DTYPE_F64, _lib.STORE_TERMINAL, 900),   # f64, three chunk launches, odd T
    (None, 3, 64, 96, _lib.DTYPE_F32, _lib.STORE_ALL, None),       # f32, P = 6144 (neither resident nor packed)
]


@pytest.mark.parametrize("B,T,N,M,dtype,store,chunk", ROWS_STEP_CASES)
def test_rows_train_step_equals_targets(golden, B, T, N, M, dtype, store, chunk) -> None:
    """smc_train_step on the rows_kernel shapes (Sobol draw, rows_kernel + cf_kernel, cursor update;
    contracts striped statically over the persistent workgroups since round 4) is bit-identical to the
    separate draw + smc_train_targets (the oracle-checked path) over three steps, and leaves the sync
    area zeroed."""
    L = _L()
    if B is None:
        B = 4 * 4 * torch.cuda.get_device_properties(0).multi_processor_count + 5
    chunk = chunk or B
    P = N * M
    f64 = dtype == _lib.DTYPE_F64
    pitch = int(L.smc_path_pitch(P, dtype))
    assert L.smc_train_step_kernel(T, N, M, dtype, pitch) == b"rows_kernel+cf_kernel"
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, torch.float64 if f64 else torch.float32, DEV)
    ctype = torch.complex128 if f64 else torch.complex64
    cur_a = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
    cur_b = cur_a.clone()
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, dtype, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    for _ in range(3):
        ca = poisoned((B, 6), torch.float64, DEV)
        fa = poisoned((B, 6), torch.float32, DEV)
        ta = poisoned((B, N), ctype, DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur_a), 0, B,
                                    _lib.ptr(ca), _lib.ptr(fa), B, T, N, M, 7, _lib.SCHEME_LOG_EULER | _lib.MATH_HW,
                                    _lib.NORM_NORMALIZE, dtype, store, _lib.ptr(paths), pitch, chunk, _lib.ptr(ta),
                                    _lib.ptr(sync), nsync, None))
        tb = poisoned_like(ta)
        _lib.check(L.smc_train_targets(_lib.ptr(ca), B, T, N, M, 7, _lib.ptr(cur_b[1:2]), 0,
                                       _lib.SCHEME_LOG_EULER | _lib.MATH_HW, _lib.NORM_NORMALIZE, dtype, store,
                                       _lib.ptr(paths), pitch, chunk, None, _lib.ptr(tb), None, 0, None))
        cur_b.add_(B)
        torch.cuda.synchronize()
        assert_rows_equal(ta.cpu().numpy(), tb.cpu().numpy())
        assert cur_a.tolist() == cur_b.tolist()
        assert not sync.view(torch.int32).any()


def test_c2_f64_timed_call_matches_oracle(oracle, golden) -> None:
    """The f64 C2 MC part exactly as the bench times it: smc_train_step at T = 16, N = M = 256
    (P = 65,536: rows_kernel with contracts striped over the persistent grid + cf_kernel), B = 2500
    contracts (more than two rounds of the persistent grid), two steps; every 80th contract against the oracle's reference-mode f64
    targets (the reference's f64 recursion with libm exp on this build's f64 normals, numpy-order FFT)
    at 1e-10 norm-relative (reference gbm.py:241-250 computes the recursion in f64)."""
    L = _L()
    B, T, N, M = 2500, 16, 256, 256
    P = N * M
    dtype = _lib.DTYPE_F64
    pitch = int(L.smc_path_pitch(P, dtype))
    assert L.smc_train_step_kernel(T, N, M, dtype, pitch) == b"rows_kernel+cf_kernel"
    slots = 4 * torch.cuda.get_device_properties(0).multi_processor_count  # 4 workgroups per CU
    assert B > 2 * slots
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    paths = poisoned((B, T, pitch), torch.float64, DEV)
    cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, dtype, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    for step in range(2):
        c = poisoned((B, 6), torch.float64, DEV)
        t = poisoned((B, N), torch.complex128, DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                    _lib.ptr(c), None, B, T, N, M, 7, _lib.SCHEME_LOG_EULER | _lib.MATH_HW,
                                    _lib.NORM_NORMALIZE, dtype, _lib.STORE_ALL, _lib.ptr(paths), pitch, B,
                                    _lib.ptr(t), _lib.ptr(sync), nsync, None))
        torch.cuda.synchronize()
        assert cur.tolist() == [(step + 1) * B] * 2
        assert not sync.view(torch.int32).any()
        idx = np.arange(step, B, 80)
        contracts = c.cpu().numpy()
        assert_rows_equal(contracts, oracle.sobol_contracts(7, step * B, B, golden["bounds_lower"],
                                                                        golden["bounds_upper"]))
        got = t.cpu().numpy()[idx]
        for k, b in enumerate(idx):  # one contract at a time: each keeps its own normal ordinal
            want = oracle.training_targets(contracts[b:b + 1], T, N, M, seed=7, ordinal0=step * B + int(b),
                                           dtype="float64")
            assert _norm_rel(got[k:k + 1], want) < 1e-10, (step, b, b % 8)


PACKED_CASES = [  # (B, T, N, M, normalize, store, chunk): P < 4096 -> packed_kernel, K = 4096 / P per workgroup
    (4096, 16, 128, 4, 1, _lib.STORE_ALL, None),    # the reference's e2e shape (P = 512, K = 8) at a full batch
    (1001, 16, 64, 4, 1, _lib.STORE_ALL, None),     # P = 256 (K = 16, one wave per contract), ragged last group
    (300, 5, 256, 8, 0, _lib.STORE_TERMINAL, None),  # P = 2048 (K = 2), odd T (rolled rows), RAW, terminal rows
    (77, 1, 16, 64, 1, _lib.STORE_ALL, None),       # T = 1, N = 16, P = 1024
    (1000, 16, 128, 4, 1, _lib.STORE_ALL, 334),     # e2e shape in 3 chunk launches (ragged last: 332)
]


@pytest.mark.parametrize("B,T,N,M,normalize,store,chunk", PACKED_CASES)
def test_packed_train_step_matches_oracle(oracle, golden, B, T, N, M, normalize, store, chunk) -> None:
    """Small P: smc_train_step runs K = 4096 / P whole contracts per 1024-thread
    workgroup (packed_kernel, Sobol draw and cursor advance fused).  Portable math bit-exact with the
    kernel-mode oracle in the packed order (one chunk of P / 4 lanes per contract: oracle.engine_wg);
    hw math within 1e-5 of the reference mode; contracts equal the Sobol draw; the sync area is left
    zeroed."""
    L = _L()
    P = N * M
    pitch = int(L.smc_path_pitch(P, 0))
    assert L.smc_train_step_kernel(T, N, M, 0, pitch) == b"packed_kernel"
    assert oracle.engine_wg(T, N, P) == P // 4
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    chunk = chunk or B  # chunk < B: several launches (per-chunk Sobol index and ordinal, last one advances)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, torch.float32, DEV)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, 0, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    norm = _lib.NORM_NORMALIZE if normalize else _lib.NORM_RAW
    for math in (0, _lib.MATH_HW):
        cur = torch.tensor([40, 9], dtype=torch.int64, device=DEV)
        c = poisoned((B, 6), torch.float64, DEV)
        f = poisoned((B, 6), torch.float32, DEV)
        t = torch.full((B, N), float("nan"), dtype=torch.complex64, device=DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                    _lib.ptr(c), _lib.ptr(f), B, T, N, M, 7, _lib.SCHEME_LOG_EULER | math, norm,
                                    _lib.DTYPE_F32, store, _lib.ptr(paths), pitch, chunk, _lib.ptr(t),
                                    _lib.ptr(sync), nsync, None))
        torch.cuda.synchronize()
        assert cur.tolist() == [40 + B, 9 + B]
        assert not sync.view(torch.int32).any()
        contracts = c.cpu().numpy()
        assert_rows_equal(contracts, oracle.sobol_contracts(7, 40, B, golden["bounds_lower"],
                                                                        golden["bounds_upper"]))
        assert_rows_equal(f.cpu().numpy(), contracts.astype(np.float32))
        got = t.cpu().numpy()
        if math == 0:
            kt, _ = oracle.kernel_targets(contracts, T, N, M, seed=7, ordinal0=9, normalize=bool(normalize),
                                          wg=P // 4)
            assert_rows_equal(got, kt)
            if store == _lib.STORE_ALL:  # the stored rows (the last chunk's) are the kernel-mode paths
                b0 = (B - 1) // chunk * chunk
                kp, _, _ = oracle.kernel_paths(contracts[b0:b0 + 3], T, P, 7, ordinal0=9 + b0, want_paths=True,
                                               wg=P // 4)
                assert_rows_equal(paths[:len(kp), :, :P].cpu().numpy(), kp)
        else:
            want = oracle.training_targets(contracts[:24], T, N, M, seed=7, ordinal0=9, normalize=bool(normalize))
            _assert_close(got[:24], want, 1e-5)


WAVE_CASES = [  # (B, T, N, M, store, chunk): RAW, T <= 2 -> wave_kernel, one wave per contract
    (4096, 1, 16, 4096, _lib.STORE_ALL, None),      # the reference's lock-step shape at C2's batch (bench "lockstep")
    (333, 2, 64, 64, _lib.STORE_ALL, None),          # T = 2: 8 draws per group, 4 groups per stream span
    (5000, 1, 256, 16, _lib.STORE_TERMINAL, None),   # more contracts than resident waves: two rounds; N = 256
    (70, 2, 1024, 2, _lib.STORE_TERMINAL, None),     # N = 1024: one batch row per chunk
    (333, 2, 64, 64, _lib.STORE_ALL, 130),           # three chunk launches (ragged last: 73)
    (40, 1, 16, 8192, _lib.STORE_TERMINAL, None),    # P = 131,072 > 65,536: still one wave (not the sliced kernel)
]


@pytest.mark.parametrize("B,T,N,M,store,chunk", WAVE_CASES)
def test_wave_train_step_matches_oracle(oracle, golden, B, T, N, M, store, chunk) -> None:
    """RAW targets at T <= 2 (the reference's lock-step trainer shape, tests/test_gbm_trainer.py:122-142):
    smc_train_step runs one wave per contract (wave_kernel: 16 paths = one stream span per lane,
    payoffs added as the chunks finish, the M-mean and FFT by the wave alone).  Portable math bit-exact
    with the kernel-mode oracle in the wave's order (wg = 256); hw math within 1e-5 of the reference mode; contracts equal the Sobol draw; the
    stored terminal rows equal the kernel-mode paths; the sync area is left zeroed."""
    L = _L()
    P = N * M
    pitch = int(L.smc_path_pitch(P, 0))
    assert L.smc_train_step_kernel(T, N, M, _lib.QUERY_RAW, pitch) == b"wave_kernel"
    assert L.smc_train_step_kernel(T, N, M, 0, pitch) != b"wave_kernel"  # NORMALIZE needs the terminal sum first
    assert oracle.train_step_order(T, N, P, normalize=False) == (256, 1)
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    chunk = chunk or B  # chunk < B: several launches (per-chunk Sobol index and ordinal, last one advances)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, torch.float32, DEV)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, 0, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    for math in (0, _lib.MATH_HW):
        cur = torch.tensor([17, 3], dtype=torch.int64, device=DEV)
        c = poisoned((B, 6), torch.float64, DEV)
        f = poisoned((B, 6), torch.float32, DEV)
        t = torch.full((B, N), float("nan"), dtype=torch.complex64, device=DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                    _lib.ptr(c), _lib.ptr(f), B, T, N, M, 43, _lib.SCHEME_LOG_EULER | math,
                                    _lib.NORM_RAW, _lib.DTYPE_F32, store, _lib.ptr(paths), pitch, chunk, _lib.ptr(t),
                                    _lib.ptr(sync), nsync, None))
        torch.cuda.synchronize()
        assert cur.tolist() == [17 + B, 3 + B]
        assert not sync.view(torch.int32).any()
        contracts = c.cpu().numpy()
        assert_rows_equal(contracts, oracle.sobol_contracts(7, 17, B, golden["bounds_lower"],
                                                                        golden["bounds_upper"]))
        got = t.cpu().numpy()
        if math == 0:
            sub = np.arange(0, B, 7)  # every 7th contract (its own normal ordinal): the oracle loops per contract
            for b in sub[:64]:
                kt, _ = oracle.kernel_targets(contracts[b:b + 1], T, N, M, seed=43, ordinal0=3 + int(b),
                                              normalize=False, wg=256)
                assert_rows_equal(got[b:b + 1], kt)
            b0 = (B - 1) // chunk * chunk  # the scratch holds the last chunk's rows
            kp, _, _ = oracle.kernel_paths(contracts[b0:b0 + 2], T, P, 43, ordinal0=3 + b0, want_paths=True, wg=256)
            if store == _lib.STORE_ALL:
                assert_rows_equal(paths[:2, :, :P].cpu().numpy(), kp)
            else:
                assert_rows_equal(paths[:2, :P].cpu().numpy(), kp[:, -1])
        else:
            want = oracle.training_targets(contracts[:16], T, N, M, seed=43, ordinal0=3, normalize=False)
            _assert_close(got[:16], want, 1e-5)


SLICED_CASES = [  # (B, N, M, store, chunk): shapes with P > 65,536 (W = P / 65,536 slices)
    (None, 1024, 256, _lib.STORE_ALL, None),   # C3 per-contract shape, W = 4, > 1 contract per group
    (70, 1024, 256, _lib.STORE_ALL, 24),       # C3 shape in three chunk launches
    (23, 128, 1024, _lib.STORE_TERMINAL, None),  # W = 2, terminal rows only
    (11, 512, 1024, _lib.STORE_ALL, None),     # W = 8, N = 512
]


@pytest.mark.parametrize("B,N,M,store,chunk", SLICED_CASES)
def test_sliced_train_step_bit_exact(oracle, golden, B, N, M, store, chunk) -> None:
    """smc_train_step at P > 65,536: W co-resident resident_kernel workgroups per contract that
    exchange their terminal and column sums.  Portable math is bit-exact with the kernel-mode
    oracle in the slice order (oracle.train_step_order); hw math within 1e-5 of the reference-mode
    targets; contracts and CVNN input bit-equal to the Sobol draw; the cursor advances; the
    arrival counters are left zeroed."""
    L = _L()
    T, P = 16, N * M
    if B is None:
        B = 2 * torch.cuda.get_device_properties(0).multi_processor_count // 4 + 3
    chunk = chunk or B
    wg, W = oracle.train_step_order(T, N, P)
    assert wg == 1024 and W == P // 65536
    pitch = int(L.smc_path_pitch(P, 0))
    assert L.smc_train_step_kernel(T, N, M, 0, pitch) == b"resident_kernel(sliced)"
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = poisoned(shape, torch.float32, DEV)
    sync, nsync = _sync(L, T, N, M, pitch)
    assert nsync > 4
    start = [40, 9]
    for math in (0, _lib.MATH_HW):
        cur = torch.tensor(start, dtype=torch.int64, device=DEV)
        c = poisoned((B, 6), torch.float64, DEV)
        f = poisoned((B, 6), torch.float32, DEV)
        t = torch.full((B, N), float("nan"), dtype=torch.complex64, device=DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                    _lib.ptr(c), _lib.ptr(f), B, T, N, M, 7, _lib.SCHEME_LOG_EULER | math,
                                    _lib.NORM_NORMALIZE, _lib.DTYPE_F32, store, _lib.ptr(paths), pitch, chunk,
                                    _lib.ptr(t), _lib.ptr(sync), nsync, None))
        cb = poisoned_like(c)
        fb = poisoned_like(f)
        draw_device(tables, 6, torch.tensor(start[:1], dtype=torch.int64, device=DEV), 0, B, lo, hi, cb, fb)
        torch.cuda.synchronize()
        assert_rows_equal(c.cpu().numpy(), cb.cpu().numpy())
        assert_rows_equal(f.cpu().numpy(), fb.cpu().numpy())
        assert cur.tolist() == [start[0] + B, start[1] + B]
        # the done counter and the group counters are back at zero (the second pass depends on it:
        # its exchanges wait for W arrivals per contract round from zero)
        words = sync.view(torch.int32).cpu().numpy()
        groups = -(-2 * torch.cuda.get_device_properties(0).multi_processor_count // W)  # sync-area capacity
        # done counter, status word, launch failure flag, contract queue and every group's two counter lines
        assert words[0] == 0 and words[8] == 0 and words[12] == 0 and words[16] == 0
        assert not words[32:32 + 64 * groups].any()
        contracts = c.cpu().numpy()
        got = t.cpu().numpy()
        if math == 0:
            kt, _ = oracle.kernel_targets(contracts, T, N, M, seed=7, ordinal0=start[1], wg=wg, slices=W)
            assert_rows_equal(got, kt)
        else:
            want = oracle.training_targets(contracts[:12], T, N, M, seed=7, ordinal0=start[1])
            _assert_close(got[:12], want, 1e-5)


def test_exchange_timeout_sets_status_not_silent_nan(oracle, golden) -> None:
    """A sliced contract whose partner slice never arrives (test hook: slice W-1 of group 0 withholds
    its first arrival, 20,000-poll budget) ends the launch with NaN targets AND the sticky status word
    SMC_SYNC_EXCHANGE_TIMEOUT, which smc_sync_status reports (and clears) and TrainingEngine maps to
    SmcError(SMC_ERR_EXCHANGE_TIMEOUT).  With the hook cleared the next step is bit-exact again, also
    when it runs before anyone has read the status (the failure flag is per launch; only the status
    word is sticky)."""
    from spectralmc_amd.engine import check_sync_status

    L = _L()
    T, N, M = 16, 128, 1024  # P = 131,072: W = 2 slices per contract
    P = N * M
    B = 9
    pitch = int(L.smc_path_pitch(P, 0))
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    paths = poisoned((B, pitch), torch.float32, DEV)
    sync, nsync = _sync(L, T, N, M, pitch)

    def step(cur):
        c = poisoned((B, 6), torch.float64, DEV)
        t = torch.zeros((B, N), dtype=torch.complex64, device=DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                    _lib.ptr(c), None, B, T, N, M, 7, _lib.SCHEME_LOG_EULER, _lib.NORM_NORMALIZE,
                                    _lib.DTYPE_F32, _lib.STORE_TERMINAL, _lib.ptr(paths), pitch, B, _lib.ptr(t),
                                    _lib.ptr(sync), nsync, None))
        return c, t

    _lib.check(L.smc_test_exchange_fault(1, 20000))
    try:
        cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
        _, t = step(cur)
        torch.cuda.synchronize()
    finally:
        _lib.check(L.smc_test_exchange_fault(0, 0))
    assert np.isnan(t[0].cpu().numpy()).all()  # group 0's first contract could not finish
    assert cur.tolist() == [B, B]                # the launch still completed and advanced the cursor
    assert int(sync.view(torch.int32)[12]) == 0  # the launch's own failure flag is cleared at its end
    wg, W = oracle.train_step_order(T, N, P)
    # the next launch, status not yet read: waits normally, bit-exact
    cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
    c, t = step(cur)
    kt, _ = oracle.kernel_targets(c.cpu().numpy(), T, N, M, seed=7, ordinal0=0, wg=wg, slices=W)
    assert_rows_equal(t.cpu().numpy(), kt)
    with pytest.raises(_lib.SmcError) as exc:  # the first launch's failure is still reported (sticky)
        check_sync_status(sync)
    assert exc.value.code == _lib.SMC_ERR_EXCHANGE_TIMEOUT
    assert _lib.sync_status(sync) == 0  # read-and-clear
    cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
    c, t = step(cur)
    check_sync_status(sync)
    assert_rows_equal(t.cpu().numpy(), kt)


def test_time_launches_spans_the_call_kernels(golden) -> None:
    """smc_time_launches: the armed events take the first kernel's start and the last kernel's end of the
    calls that follow (hipExtLaunchKernel), so they span less than stream events around the same call and
    more than zero; disarmed, later calls leave them alone; the targets are unchanged."""
    L = _L()
    B, T, N, M = 64, 16, 128, 4  # packed_kernel: one launch per call
    P = N * M
    pitch = int(L.smc_path_pitch(P, 0))
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    paths = poisoned((B, T, pitch), torch.float32, DEV)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, 0, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    outs = []
    for timed in (False, True):
        cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
        c = poisoned((B, 6), torch.float64, DEV)
        t = poisoned((B, N), torch.complex64, DEV)
        s0, s1, k0, k1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        k0.record()
        k1.record()
        torch.cuda.synchronize()
        s0.record()
        if timed:
            _lib.check(L.smc_time_launches(k0.cuda_event, k1.cuda_event))
        try:
            _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur), 0, B,
                                        _lib.ptr(c), None, B, T, N, M, 7, _lib.SCHEME_LOG_EULER, _lib.NORM_NORMALIZE,
                                        _lib.DTYPE_F32, _lib.STORE_ALL, _lib.ptr(paths), pitch, B, _lib.ptr(t),
                                        _lib.ptr(sync), nsync, None))
        finally:
            _lib.check(L.smc_time_launches(None, None))
        s1.record()
        torch.cuda.synchronize()
        outs.append(t.cpu().numpy())
        if timed:
            kernel, around = k0.elapsed_time(k1), s0.elapsed_time(s1)
            assert 0.0 < kernel <= around, (kernel, around)
    assert_rows_equal(outs[1], outs[0], "timed launch")
