"""ORACLE — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The reference's CPU path as BASELINE.json ``north_star`` names it — torch-cpu + numpy.fft — for
one GbmCVNNPricer training step, vectorised over a batch of contracts.  Used by ``bench.py``'s
``cpu_baseline`` leg (timed on the GPU box's host cores) and by the CPU tests (checked against the
reference-generated fixtures).  Never imported by ``spectralmc_amd``.

Per contract, in the reference's order (Tuee22/SpectralMC @ 2026-01-02):
  normals  (T, P) of the contract ordinal                 async_normals.py:212-216 (values: this
                                                          build's streams, oracle.normals)
  paths    X_t = X_{t-1} exp((r - d - v^2/2) dt + v sqrt(dt) Z_t)  in f64, stored in the sim dtype
           (log-Euler; Numba's f64 arithmetic, gbm.py:241-250) — a running product over t
  forwards times = linspace(dt, T, T) (sim dtype); F = X0 exp((r - d) times); df = exp(-r times)
                                                          gbm.py:428-431
  NORMALIZE sims *= F / mean_p(sims)  (sim-dtype mean)    gbm.py:435-438
  payoff   put = df_T max(K - S_T, 0)                     gbm.py:464-473
  targets  mean_m fft(put.reshape(M, N), axis=1)          gbm_trainer.py:814-817 (numpy.fft)
and the network half is oracle.torch_step (gbm_trainer.py:819-835) on torch-cpu.
"""

from __future__ import annotations

import math

import numpy as np
import torch

from . import oracle as _o


_SEED_LIMIT = 1_000_000_000  # async_normals.py _SEED_LIMIT


def numpy_seed_stream(mc_seed: int, skip: int, count: int) -> list[int]:
    """Per-matrix seeds of ConcurrentNormGenerator: the k-th draw of
    np.random.default_rng(mc_seed).integers(0, 1e9) (async_normals.py:319-326, 391)."""
    rng = np.random.default_rng(mc_seed)
    rng.integers(0, _SEED_LIMIT, size=skip)
    return [int(x) for x in rng.integers(0, _SEED_LIMIT, size=count)]


def cpu_path_targets(contracts: np.ndarray, timesteps: int, network_size: int, batches: int, seed: int,
                     ordinal0: int = 0, dtype: str = "float32", normals: str = "build",
                     workers: int | None = None, normalize: bool = True) -> np.ndarray:
    """CF targets (B, N) of B contracts on the torch-cpu + numpy.fft path (log-Euler; NORMALIZE, or RAW
    with normalize=False).

    normals "build": this build's stream for each contract ordinal (oracle.normals), so the
    result is comparable with the GPU and the reference fixtures; "numpy": the reference
    generator's CPU analogue, numpy ``default_rng(seed_m).standard_normal((T, P), dtype)`` with
    the pool's seed stream (async_normals.py:212-216, 319-326) — the timing leg of bench.py.
    Contracts are simulated one after another on reused buffers (torch intra-op threads); the
    next contracts' normals are drawn meanwhile on a thread pool (numpy releases the GIL), as
    the reference's pool pre-generates matrices."""
    from concurrent.futures import ThreadPoolExecutor

    contracts = np.ascontiguousarray(contracts, dtype=np.float64)
    B = contracts.shape[0]
    T, N, M = timesteps, network_size, batches
    P = N * M
    sim = torch.float32 if dtype == "float32" else torch.float64
    np_sim = np.float32 if dtype == "float32" else np.float64
    seeds = numpy_seed_stream(seed, ordinal0, B) if normals == "numpy" else None

    def draw(b: int) -> np.ndarray:  # the pool's matrix for contract ordinal ordinal0 + b
        if seeds is not None:
            return np.random.default_rng(seeds[b]).standard_normal((T, P), dtype=np_sim)
        return _o.normals(seed, ordinal0 + b, T, P, dtype)

    w = torch.empty((T, P), dtype=torch.float64)
    x = torch.empty((T, P), dtype=torch.float64)
    paths = torch.empty((T, P), dtype=sim)
    out = np.empty((B, N), dtype=np.complex64 if dtype == "float32" else np.complex128)
    workers = workers or max(1, torch.get_num_threads())
    with ThreadPoolExecutor(max_workers=workers) as pool:
        futures = [pool.submit(draw, b) for b in range(min(B, 2 * workers))]
        for b in range(B):
            z = futures[b].result()
            futures[b] = None
            if b + 2 * workers < B:
                futures.append(pool.submit(draw, b + 2 * workers))
            X0, K, Tm, r, d, v = (float(q) for q in contracts[b])
            dt = Tm / T
            # Numba's f64 arithmetic (gbm.py:241-250): dW = Z sqrt(dt); X *= exp(drift dt + v dW)
            w.copy_(torch.from_numpy(z))
            w.mul_(math.sqrt(dt)).mul_(v).add_((r - d - 0.5 * v * v) * dt).exp_()
            w[0].mul_(X0)  # X = X0; X *= e_1; X *= e_2 ...: the recursion's association
            torch.cumprod(w, 0, out=x)
            paths.copy_(x)  # stored in the sim dtype
            times = np.linspace(dt, Tm, T).astype(np_sim)  # cp.linspace(dt, T, T, dtype)
            fwd = np_sim(X0) * np.exp(np_sim(r - d) * times)
            df = np.exp(np_sim(-r) * times)
            terminal = paths[-1].numpy()
            # sims *= F / cp.mean(sims) (terminal row; RAW keeps the simulated values)
            s_T = terminal * (fwd[-1] / terminal.mean()) if normalize else terminal
            put = (df[-1] * np.maximum(np_sim(K) - s_T, np_sim(0))).astype(np_sim)
            out[b] = np.fft.fft(put.reshape(M, N), axis=1).mean(axis=0)
    return out


def cpu_training_step(model, adam, contracts: np.ndarray, timesteps: int, network_size: int, batches: int,
                      seed: int, ordinal0: int = 0, normals: str = "build") -> tuple[np.ndarray, "_o.StepResult"]:
    """One full training step on the CPU path: targets, then _torch_step on torch-cpu."""
    targets = cpu_path_targets(contracts, timesteps, network_size, batches, seed, ordinal0, normals=normals)
    x = torch.tensor(contracts, dtype=torch.float32)
    return targets, _o.torch_step(model, x, torch.zeros_like(x), torch.from_numpy(targets), adam)
