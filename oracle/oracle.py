"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference GbmCVNNPricer training step (Tuee22/SpectralMC @
2026-01-02), used as the parity checker by ``tests/``, by ``__graft_entry__.smoke()`` and
as the CPU baseline in ``bench.py``.  The product package ``spectralmc_amd`` never imports
this module; its HIP path fails loudly when its extension is missing instead of falling back
here.

Pieces and what pins them
-------------------------
* Sobol contracts  -> ``scipy.stats.qmc.Sobol`` itself (the reference's own dependency,
  scipy 1.15.3 here; ``sobol_sampler.py:192,197,238-239``).  Pinned by golden vectors made
  with the reference's ``SobolSampler`` (tests/golden/make_golden.py).
* Normals + paths  -> ``oracle/gbm_oracle.c`` (f64 recursion / dtype stores as the Numba
  kernel, ``gbm.py:241-257``).  Philox pinned by Random123 KAT vectors, the MWC64X stream by a
  Python restatement of its recurrence (tests/test_oracle.py); normal-level parity
  with CuPy XORWOW is unpinned (CuPy absent).  The path arithmetic is additionally pinned by
  closed-form cases (v = 0, T = 0) and the reference test's Black-price acceptance
  (``tests/test_gbm.py:103-139``).
* Normalisation, payoff, FFT, batch mean -> numpy in the sim dtype, in the reference's order
  (``gbm.py:428-438,464-474``; ``gbm_trainer.py:814-817``: FFT each batch row, then mean).
* CVNN step -> torch-cpu restatement of ``_torch_step`` (``gbm_trainer.py:819-835``) on a CPU
  copy of the model; the model's weights/forward are pinned by golden vectors made with the
  reference's ``cvnn_factory.build_model``.
"""

from __future__ import annotations

import ctypes
import math
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsmc_oracle.so")
_lib: ctypes.CDLL | None = None

FIELDS = ("X0", "K", "T", "r", "d", "v")  # BlackScholes.Inputs order, gbm.py:270-275


def build() -> str:
    """Compile the C restatement (gcc, no GPU)."""
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_philox4x32_10.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_stream_u32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64,
                                        ctypes.c_void_p]
        L.oracle_normals.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_void_p]
        L.oracle_gbm_paths.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                       ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        L.oracle_num_threads.restype = ctypes.c_int32
        L.oracle_kernel_paths.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                          ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                          ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_kernel_cf.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_basket_kernel.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_basket_cholesky.argtypes = [ctypes.c_int32, ctypes.c_double, ctypes.c_void_p]
        L.oracle_m2log_u32.argtypes = [ctypes.c_uint32]
        L.oracle_m2log_u32.restype = ctypes.c_double
        L.oracle_exp2s_f64.argtypes = [ctypes.c_double]
        L.oracle_exp2s_f64.restype = ctypes.c_double
        L.oracle_sincos2pi_u32.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_log_pos.argtypes = [ctypes.c_float]
        L.oracle_log_pos.restype = ctypes.c_float
        L.oracle_exp2.argtypes = [ctypes.c_float]
        L.oracle_exp2.restype = ctypes.c_float
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None) -> int | None:
    return None if a is None else a.ctypes.data


def _np_dtype(dtype: str) -> type:
    return {"float32": np.float32, "float64": np.float64}[dtype]


# --------------------------------------------------------------------------- RNG
def philox4x32_10(ctr: tuple[int, int, int, int], key: tuple[int, int]) -> tuple[int, ...]:
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return tuple(int(x) for x in out)


def stream_u32(seed: int, ordinal: int, group: int, n: int) -> np.ndarray:
    """The first n u32 outputs of the (seed, ordinal, group) path stream (csrc/smc_rng.h)."""
    out = np.empty(n, dtype=np.uint32)
    lib().oracle_stream_u32(seed, ordinal, group, n, _ptr(out))
    return out


def m2log_u32(a: int) -> float:
    """-2 ln((a + 1/2) 2^-32): the f64 Box-Muller radius squared (csrc/smc_math.h m2log_u32)."""
    return float(lib().oracle_m2log_u32(a))


def sincos2pi_u32(b: int) -> tuple[float, float]:
    """(sin, cos) of the f64 Box-Muller angle of the 32-bit uniform b, 2 pi ((b mod 1024) / 1024 + y 2^-32) with
    y = b >> 10 as a signed 22-bit integer (csrc/smc_math.h sincos2pi_u32)."""
    s, c = ctypes.c_double(), ctypes.c_double()
    lib().oracle_sincos2pi_u32(b, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def exp2s_f64(ys: float) -> float:
    """2^(ys / 256) as the f64 device path recursion computes it, the exponent in units of ln 2 / 256
    (csrc/smc_math.h exp2s_f64)."""
    return float(lib().oracle_exp2s_f64(ys))


def normals(seed: int, ordinal: int, rows: int, cols: int, dtype: str = "float32") -> np.ndarray:
    out = np.empty((rows, cols), dtype=_np_dtype(dtype))
    lib().oracle_normals(seed, ordinal, rows, cols, 1 if dtype == "float64" else 0, _ptr(out))
    return out


# --------------------------------------------------------------------------- Sobol
def sobol_contracts(seed: int, skip: int, n: int, lower: np.ndarray, upper: np.ndarray) -> np.ndarray:
    """SobolSampler._sample_nonzero arithmetic (sobol_sampler.py:238-239) on SciPy's engine."""
    import warnings

    from scipy.stats.qmc import Sobol

    eng = Sobol(d=len(lower), scramble=True, seed=seed)
    if skip:
        eng.fast_forward(skip)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        raw = eng.random(n)
    return lower + (upper - lower) * raw


# --------------------------------------------------------------------------- paths
def gbm_paths(contracts: np.ndarray, timesteps: int, n_paths: int, seed: int, ordinal0: int = 0,
              scheme: int = 0, dtype: str = "float32", want_paths: bool = False,
              threads: int = 0) -> tuple[np.ndarray | None, np.ndarray, np.ndarray]:
    """(paths [B,T,P] or None, terminal [B,P], rowsum [B,T] f64) of the raw paths."""
    contracts = np.ascontiguousarray(contracts, dtype=np.float64)
    B = contracts.shape[0]
    dt = _np_dtype(dtype)
    paths = np.empty((B, timesteps, n_paths), dtype=dt) if want_paths else None
    terminal = np.empty((B, n_paths), dtype=dt)
    rowsum = np.empty((B, timesteps), dtype=np.float64)
    lib().oracle_gbm_paths(_ptr(contracts), B, timesteps, n_paths, seed, ordinal0, scheme,
                           1 if dtype == "float64" else 0, _ptr(paths), _ptr(terminal), _ptr(rowsum), threads)
    return paths, terminal, rowsum


def _times(Tm: float, timesteps: int, dt_np: type) -> np.ndarray:
    """cp.linspace(dt, T, timesteps, dtype) (gbm.py:429): f64 grid cast, last point exact."""
    dt = Tm / timesteps
    grid = np.linspace(dt, Tm, timesteps, dtype=np.float64)
    return grid.astype(dt_np)


def normalize_paths(contracts: np.ndarray, paths: np.ndarray, rowsum: np.ndarray) -> np.ndarray:
    """sims *= forwards / row_means (gbm.py:428-438) in the sim dtype."""
    out = paths.copy()
    dt_np = paths.dtype.type
    B, T, P = paths.shape
    for b in range(B):
        X0, _, Tm, r, d, _ = (float(x) for x in contracts[b])
        times = _times(Tm, T, dt_np)
        forwards = dt_np(X0) * np.exp(dt_np(r - d) * times)
        means = (rowsum[b] / P).astype(dt_np)
        out[b] *= (forwards / means)[:, None]
    return out


def cf_targets(contracts: np.ndarray, terminal: np.ndarray, terminal_sum: np.ndarray | None, network_size: int,
               batches: int, normalize: bool = True) -> np.ndarray:
    """Per contract: put payoff on the (normalised) terminal row, FFT of each of the M batch
    rows of length N, mean over batches (gbm.py:464-474, gbm_trainer.py:814-817).

    terminal_sum None: the row mean is ``numpy.mean`` of the stored terminal row in the sim
    dtype (gbm.py:437 ``cp.mean(sims, axis=1)`` on the CPU path: pairwise, dtype accumulator)."""
    dt_np = terminal.dtype.type
    B, P = terminal.shape
    assert P == network_size * batches
    X0 = contracts[:, 0]
    K = contracts[:, 1].astype(dt_np)
    Tm = contracts[:, 2].astype(dt_np)
    r = contracts[:, 3]
    d = contracts[:, 4]
    F = X0.astype(dt_np) * np.exp((r - d).astype(dt_np) * Tm)
    df = np.exp((-r).astype(dt_np) * Tm)
    if normalize:
        mean = terminal.mean(axis=1) if terminal_sum is None else (terminal_sum / P).astype(dt_np)
        scale = (F / mean).astype(dt_np)
        sims_T = (terminal * scale[:, None]).astype(dt_np)
    else:
        sims_T = terminal
    put = df[:, None] * np.maximum(K[:, None] - sims_T, dt_np(0))
    mat = put.reshape(B, batches, network_size)
    spec = np.fft.fft(mat, axis=2).mean(axis=1)
    return spec.astype(np.complex64 if dt_np is np.float32 else np.complex128)


def training_targets(contracts: np.ndarray, timesteps: int, network_size: int, batches: int, seed: int,
                     ordinal0: int = 0, scheme: int = 0, normalize: bool = True, dtype: str = "float32",
                     threads: int = 0) -> np.ndarray:
    """The Monte-Carlo side of one training step for a batch of contracts, as the reference CPU
    path computes it (pinned bit-for-bit by tests/golden/gbm_golden.npz, made by the
    reference's own gbm.py + _simulate_fft on these normals)."""
    _, terminal, _ = gbm_paths(contracts, timesteps, network_size * batches, seed, ordinal0, scheme, dtype,
                               want_paths=False, threads=threads)
    return cf_targets(contracts, terminal, None, network_size, batches, normalize)


# --------------------------------------------------------------------------- kernel mode
# paths per workgroup slice when smc_train_targets gets a workspace (gbm.hip kSliceChunks * kChunk)
SLICE_PATHS = 8192
# scheme flag (spectralmc_hip.h SMC_MATH_REF): kernel mode of rows_ref_kernel -- the reference kernel's
# typing, f64 state and step (the f64 engine's exp) of the portable f32 normals, f32 stores
MATH_REF = 0x400


def kernel_paths(contracts: np.ndarray, timesteps: int, n_paths: int, seed: int, ordinal0: int = 0,
                 scheme: int = 0, want_paths: bool = False, sliced: bool = False,
                 wg: int = 512, slices: int = 1) -> tuple[np.ndarray | None, np.ndarray, np.ndarray]:
    """f32 KERNEL mode: exact restatement of the HIP engine (paths, terminal, rowsum in its order).
    sliced: row sums in the sliced-contract order (engine with a workspace); wg: lanes of the
    engine workgroup whose reduction order to follow (1024 = resident_kernel); slices: workgroups
    per contract of the sliced resident_kernel (slices of n_paths / slices paths, added in order)."""
    contracts = np.ascontiguousarray(contracts, dtype=np.float64)
    B = contracts.shape[0]
    paths = np.empty((B, timesteps, n_paths), dtype=np.float32) if want_paths else None
    terminal = np.empty((B, n_paths), dtype=np.float32)
    rowsum = np.empty((B, timesteps), dtype=np.float64)
    span = SLICE_PATHS if sliced else (n_paths // slices if slices > 1 else 0)
    lib().oracle_kernel_paths(_ptr(contracts), B, timesteps, n_paths, seed, ordinal0, scheme,
                              span, wg, _ptr(paths), _ptr(terminal), _ptr(rowsum))
    return paths, terminal, rowsum


def kernel_cf(contracts: np.ndarray, terminal: np.ndarray, terminal_sum: np.ndarray, network_size: int,
              batches: int, normalize: bool = True, wg: int = 512, slices: int = 1) -> np.ndarray:
    contracts = np.ascontiguousarray(contracts, dtype=np.float64)
    terminal = np.ascontiguousarray(terminal, dtype=np.float32)
    terminal_sum = np.ascontiguousarray(terminal_sum, dtype=np.float64)
    out = np.empty((contracts.shape[0], network_size), dtype=np.complex64)
    lib().oracle_kernel_cf(_ptr(contracts), contracts.shape[0], network_size, batches, int(normalize), wg,
                           slices, _ptr(terminal), _ptr(terminal_sum), _ptr(out))
    return out


def _wave_shape(timesteps: int, N: int, P: int, normalize: bool) -> bool:
    """gbm.hip wave_ok: RAW, T <= 2, 1024 | P, 16 | N, N | 1024 (a lane's 16 paths = one stream span of
    16 adjacent columns)."""
    return not normalize and timesteps <= 2 and P % 1024 == 0 and N >= 16 and N % 16 == 0 and 1024 % N == 0


def engine_wg(timesteps: int, network_size: int, n_paths: int, with_rowsum: bool = False,
              sliced: bool = False, normalize: bool = True) -> int:
    """Lanes whose reduction order an f32 training launch of smc_train_targets follows: 1024 for
    resident_kernel (1 <= T <= 65,536, 4096 | P <= 65,536, N | 4096, 4 <= N <= 1024, no row sums, no
    workspace; gbm.hip resident_ok), P / 4 for packed_kernel (256 <= P <= 2048, P | 4096, 4 | N, N | P:
    one chunk of P / 4 lanes per contract; gbm.hip packed_ok), 256 for wave_kernel (one wave per contract
    walking 1024-path chunks, 16 paths per lane: the column-sum order of 256 four-path lanes, G = 1024 / N
    batch-row groups; _wave_shape), 512 otherwise."""
    N, P = network_size, n_paths
    if with_rowsum or sliced or not 1 <= timesteps <= 65536:
        return 512
    if _wave_shape(timesteps, N, P, normalize):
        return 256
    if P % 4096 == 0 and P // 4096 <= 16 and 4 <= N <= 1024 and 4096 % N == 0:
        return 1024
    if 256 <= P <= 2048 and 4096 % P == 0 and N >= 4 and N % 4 == 0 and P % N == 0:
        return P // 4
    return 512


def train_step_order(timesteps: int, network_size: int, n_paths: int, normalize: bool = True) -> tuple[int, int]:
    """(wg, slices) of the f32 resident launch smc_train_step makes for this shape (gbm.hip
    resident_slices / resident_ok: W = the fewest power-of-two slices of <= 65,536 paths, W <= 8),
    or (engine_wg(...), 1) where it falls back to the separate draw + smc_train_targets calls."""
    N, P = network_size, n_paths
    W = 1
    while W < 8 and P > W * 65536:
        W *= 2
    if _wave_shape(timesteps, N, P, normalize):
        return 256, 1
    ok = (1 <= timesteps <= 65536 and P % (W * 4096) == 0 and P // (W * 4096) <= 16 and 4 <= N <= 1024
          and 4096 % N == 0)
    return (1024, W) if ok else (engine_wg(timesteps, N, P, normalize=normalize), 1)


def kernel_targets(contracts: np.ndarray, timesteps: int, network_size: int, batches: int, seed: int,
                   ordinal0: int = 0, scheme: int = 0, normalize: bool = True,
                   sliced: bool = False, wg: int = 512, slices: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """(targets [B,N] complex64, rowsum [B,T]) exactly as the f32 HIP engine computes them
    (wg: engine_wg(...) of the launch; slices: train_step_order(...) for smc_train_step)."""
    _, terminal, rowsum = kernel_paths(contracts, timesteps, network_size * batches, seed, ordinal0, scheme,
                                       sliced=sliced, wg=wg, slices=slices)
    return kernel_cf(contracts, terminal, rowsum[:, -1], network_size, batches, normalize, wg=wg,
                     slices=slices), rowsum


# --------------------------------------------------------------------------- basket (extension)
def basket_fields(n_assets: int) -> tuple[str, ...]:
    """Contract row of the basket engine (spectralmc_amd/basket.py BasketInputs order)."""
    return ("K", "T", "r", "rho") + tuple(f"X0_{i}" for i in range(n_assets)) + tuple(
        f"d_{i}" for i in range(n_assets)) + tuple(f"v_{i}" for i in range(n_assets))


def basket_cholesky(n_assets: int, rho: float) -> np.ndarray:
    L = np.zeros((8, 8), dtype=np.float64)
    lib().oracle_basket_cholesky(n_assets, float(rho), _ptr(L))
    return L[:n_assets, :n_assets].copy()


def basket_order(n_assets: int, timesteps: int, network_size: int, batches: int, resident: bool = True) -> tuple[int, int]:
    """(wg, slices) of the basket launch smc_basket_train_targets makes for this shape (basket.hip
    basket_res_slices): basket_resident_kernel (1024 lanes, W = N*M / 4096 workgroups per contract)
    when a sync area is passed and T = 16, N | 4096, 4 <= N <= 2048, 4096 | N*M, W <= 32 and the LDS
    plan fits 160 KiB; else basket_kernel (512 lanes, one workgroup per contract)."""
    N, P, A = network_size, network_size * batches, n_assets
    lds = A * 1024 * 16 + (4096 + 16 * 8 + 16) * 8 + (2 * 64 + 2) * (2 * A + A * A) * 4
    ok = (resident and timesteps == 16 and 4 <= N <= 2048 and N % 4 == 0 and 4096 % N == 0 and P % 4096 == 0
          and P // 4096 <= 32 and lds <= 160 * 1024)
    return (1024, P // 4096) if ok else (512, 1)


def basket_kernel(contracts: np.ndarray, n_assets: int, timesteps: int, network_size: int, batches: int,
                  seed: int, ordinal0: int = 0, normalize: bool = True,
                  want_paths: bool = False, wg: int = 512, slices: int = 1) -> tuple[np.ndarray | None, np.ndarray, np.ndarray]:
    """KERNEL mode restatement of the f32 basket engine (csrc/basket.hip, portable math):
    (paths [B,A,T,P] or None, terminal sums [B,A] f64, targets [B,N] complex64).
    (wg, slices): the launch's reduction orders, basket_order(...)."""
    contracts = np.ascontiguousarray(contracts, dtype=np.float64)
    B = contracts.shape[0]
    assert contracts.shape[1] == 3 * n_assets + 4
    P = network_size * batches
    paths = np.empty((B, n_assets, timesteps, P), dtype=np.float32) if want_paths else None
    tsum = np.empty((B, n_assets), dtype=np.float64)
    out = np.empty((B, network_size), dtype=np.complex64)
    lib().oracle_basket_kernel(_ptr(contracts), B, n_assets, timesteps, network_size, batches, seed, ordinal0,
                               int(normalize), wg, slices, _ptr(paths), _ptr(tsum), _ptr(out))
    return paths, tsum, out


def basket_reference_targets(contracts: np.ndarray, n_assets: int, terminal: np.ndarray, network_size: int,
                             batches: int) -> np.ndarray:
    """numpy statement of the basket payoff + FFT (reference gbm_trainer.py:806-817 shape:
    FFT of each batch row, then the mean) from given terminal values [B,A,P] (f64)."""
    contracts = np.asarray(contracts, dtype=np.float64)
    B, A = contracts.shape[0], n_assets
    K, T, r = contracts[:, 0], contracts[:, 1], contracts[:, 2]
    X0, d = contracts[:, 4:4 + A], contracts[:, 4 + A:4 + 2 * A]
    F = X0 * np.exp((r[:, None] - d) * T[:, None])
    scale = F / terminal.mean(axis=2)
    basket = (terminal * scale[:, :, None]).mean(axis=1)
    put = np.exp(-r * T)[:, None] * np.maximum(K[:, None] - basket, 0.0)
    return np.fft.fft(put.reshape(B, batches, network_size), axis=2).mean(axis=1)


# --------------------------------------------------------------------------- CVNN step
@dataclass
class StepResult:
    loss: float
    grad_norm: float


def torch_step(model, real_in, imag_in, targets, optimizer) -> StepResult:
    """_torch_step (gbm_trainer.py:819-835) on whatever device the tensors live on (CPU here)."""
    import torch

    pred_r, pred_i = model(real_in, imag_in)
    loss = torch.nn.functional.mse_loss(pred_r, torch.real(targets)) + torch.nn.functional.mse_loss(
        pred_i, torch.imag(targets))
    optimizer.zero_grad(set_to_none=True)
    loss.backward()
    optimizer.step()
    grad_norm = float(torch.nn.utils.clip_grad_norm_(model.parameters(), float("inf")))
    return StepResult(float(loss.item()), grad_norm)


# --------------------------------------------------------------------------- KAT
def black_put(X0: float, K: float, T: float, r: float, d: float, v: float) -> float:
    """Closed-form Black-Scholes put (QuantLib blackFormula as used in quantlib.py:19-42)."""
    df = math.exp(-r * T)
    fwd = X0 * math.exp((r - d) * T)
    if T <= 0 or v <= 0:
        return df * max(K - fwd, 0.0)
    sd = v * math.sqrt(T)
    d1 = (math.log(fwd / K) + 0.5 * sd * sd) / sd
    d2 = d1 - sd
    ncdf = lambda x: 0.5 * math.erfc(-x / math.sqrt(2.0))  # noqa: E731
    return df * (K * ncdf(-d2) - fwd * ncdf(-d1))


def num_threads() -> int:
    return int(lib().oracle_num_threads())
