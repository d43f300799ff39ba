"""Correlated multi-asset GBM (basket) engine — BASELINE.json configs[4] extension.

The reference prices one asset per contract (``src/spectralmc/gbm.py``).  This module adds
the builder-defined multi-asset case the benchmark names ("multi-asset correlated GBM, 4
assets, Cholesky in LDS"): each asset follows the reference log-Euler dynamics
(gbm.py:224-257) and forward normalisation (gbm.py:428-440), the assets' Brownian drivers
are equicorrelated with a per-contract rho, the payoff is an equal-weight basket put, and
the training target is mean_m FFT_N(put.reshape(M, N)) as ``_simulate_fft``
(gbm_trainer.py:806-817).

Contract row (Sobol dimensions, in order): K, T, r, rho, X0_0..X0_{A-1}, d_0..d_{A-1},
v_0..v_{A-1}.  All device work is one launch of ``smc_basket_train_targets`` (csrc/basket.hip)
per chunk of contracts, after the Sobol draw; no host synchronisation.

``BasketEngine`` has the interface of ``engine.TrainingEngine`` (``buffers``,
``enqueue_step``, ``set_position``, ``global_batch``), so a ``GbmCVNNPricer`` whose CVNN has
3A+4 inputs trains on baskets through ``use_basket_engine``.  Snapshots of such a pricer
record the network, optimizer and Sobol/normal positions as usual but not the basket
configuration: call ``use_basket_engine`` again on the restored pricer.  ``predict_price``
stays single-asset (the reference has no basket pricing API).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import engine as _engine
from .engine import StepBuffers, check_sync_status
from .sobol_sampler import SobolEngine, draw_device

MAX_ASSETS = 8


def basket_fields(n_assets: int) -> tuple[str, ...]:
    return ("K", "T", "r", "rho") + tuple(f"X0_{i}" for i in range(n_assets)) + tuple(
        f"d_{i}" for i in range(n_assets)) + tuple(f"v_{i}" for i in range(n_assets))


def default_basket_bounds(n_assets: int, *, x0=(0.001, 10_000.0), k=(0.001, 20_000.0), t=(0.0, 10.0),
                          r=(-0.20, 0.20), d=(-0.20, 0.20), v=(0.0, 2.0),
                          rho=None) -> dict[str, tuple[float, float]]:
    """Per-field (lower, upper): the single-asset defaults of tests/helpers/factories.py:108-161
    per asset, plus the correlation range (default [max(-0.2, -0.9/(A-1)), 0.9]: the
    equicorrelation matrix is positive definite for rho > -1/(A-1))."""
    if rho is None:
        rho = (max(-0.20, -0.9 / (n_assets - 1)) if n_assets > 1 else -0.20, 0.90)
    out = {"K": k, "T": t, "r": r, "rho": rho}
    for i in range(n_assets):
        out[f"X0_{i}"] = x0
    for i in range(n_assets):
        out[f"d_{i}"] = d
    for i in range(n_assets):
        out[f"v_{i}"] = v
    return out


@dataclass(frozen=True)
class BasketConfig:
    n_assets: int = 4
    timesteps: int = 16
    network_size: int = 256
    batches_per_mc_run: int = 512
    mc_seed: int = 7
    normalize: bool = True
    math: str = "hw"  # "hw" (hardware transcendentals) or "portable" (bit-identical to the oracle)
    bounds: dict[str, tuple[float, float]] | None = field(default=None)

    def __post_init__(self) -> None:
        if not 1 <= self.n_assets <= MAX_ASSETS:
            raise ValueError(f"n_assets must be in 1..{MAX_ASSETS}, got {self.n_assets}")
        if self.timesteps <= 0 or self.network_size <= 0 or self.batches_per_mc_run <= 0:
            raise ValueError("timesteps, network_size and batches_per_mc_run must be positive")
        if self.network_size % 4 or self.network_size > 4096:
            raise ValueError("network_size must be a multiple of 4 and <= 4096")
        if self.total_paths % 2048:
            raise ValueError("network_size * batches_per_mc_run must be a multiple of 2048")
        if self.math not in ("hw", "portable"):
            raise ValueError(f"math must be 'hw' or 'portable', got {self.math!r}")
        lo_rho = self.resolved_bounds()["rho"][0]
        if self.n_assets > 1 and lo_rho <= -1.0 / (self.n_assets - 1):
            raise ValueError(f"rho lower bound {lo_rho} makes the correlation matrix indefinite")

    @property
    def total_paths(self) -> int:
        return self.network_size * self.batches_per_mc_run

    @property
    def dim(self) -> int:
        return 3 * self.n_assets + 4

    def resolved_bounds(self) -> dict[str, tuple[float, float]]:
        b = default_basket_bounds(self.n_assets)
        if self.bounds:
            unknown = set(self.bounds) - set(b)
            if unknown:
                raise ValueError(f"unknown basket fields {sorted(unknown)}")
            b.update(self.bounds)
        return b

    def arrays(self) -> tuple[np.ndarray, np.ndarray]:
        b = self.resolved_bounds()
        names = basket_fields(self.n_assets)
        return (np.array([b[n][0] for n in names], dtype=np.float64),
                np.array([b[n][1] for n in names], dtype=np.float64))


def sync_bytes(cfg: BasketConfig, chunk_contracts: int) -> int:
    """Bytes of the sync area the resident basket kernel needs for this shape and launch size (0: it
    does not take the shape)."""
    n = int(_lib.lib().smc_basket_sync_bytes(cfg.n_assets, cfg.timesteps, cfg.network_size, cfg.batches_per_mc_run,
                                             chunk_contracts))
    if n < 0:
        raise RuntimeError("smc_basket_sync_bytes: bad shape or device query failed")
    return n


def basket_targets(contracts: torch.Tensor, cfg: BasketConfig, *, ordinal0: int = 0, paths: torch.Tensor | None = None,
                   terminal_sum: torch.Tensor | None = None, targets: torch.Tensor | None = None,
                   pitch: int = 0, resident: bool = True) -> torch.Tensor:
    """One call of the basket engine on explicit device contracts [B, 3A+4] f64.
    ``paths``: [B, A, T, pitch] f32 to keep every row, else only terminal rows are kept (scratch).
    ``resident``: pass a sync area, so shapes basket_resident_kernel takes run it (reduction orders:
    oracle.basket_order(...))."""
    _lib.require_device()
    B = contracts.shape[0]
    if contracts.dtype != torch.float64 or contracts.shape[1] != cfg.dim or not contracts.is_contiguous():
        raise ValueError(f"contracts must be a contiguous (B, {cfg.dim}) float64 tensor")
    P = cfg.total_paths
    pitch = pitch or P
    store = _lib.STORE_ALL if paths is not None else _lib.STORE_TERMINAL
    if paths is None:
        paths = torch.empty((B, cfg.n_assets, pitch), dtype=torch.float32, device=contracts.device)
    elif paths.dtype != torch.float32 or paths.numel() < B * cfg.n_assets * cfg.timesteps * pitch:
        raise ValueError("paths must be float32 with room for [B, A, T, pitch]")
    if targets is None:
        targets = torch.empty((B, cfg.network_size), dtype=torch.complex64, device=contracts.device)
    nsync = sync_bytes(cfg, max(B, 1)) if resident else 0
    sync = torch.zeros(nsync, dtype=torch.uint8, device=contracts.device) if nsync else None
    _lib.check(_lib.lib().smc_basket_train_targets(
        _lib.ptr(contracts), B, cfg.n_assets, cfg.timesteps, cfg.network_size, cfg.batches_per_mc_run, cfg.mc_seed,
        None, ordinal0, _lib.MATH_HW if cfg.math == "hw" else 0, 1 if cfg.normalize else 0, store, _lib.ptr(paths),
        pitch, max(B, 1), _lib.ptr(terminal_sum), _lib.ptr(targets), _lib.ptr(sync), nsync, _lib.stream_handle()))
    return targets


class BasketEngine:
    """Device buffers + launches of the basket Monte-Carlo side of one training step
    (the ``TrainingEngine`` interface)."""

    def __init__(self, cfg: BasketConfig, batch_size: int, *, device: torch.device, sobol_skip: int = 0,
                 model_dtype: torch.dtype = torch.float32, rank: int = 0, world_size: int = 1,
                 store_paths: bool = True, path_buffer_bytes: int | None = None) -> None:
        _lib.require_device()
        self.cfg = cfg
        self.B = batch_size
        self.A = cfg.n_assets
        self.T = cfg.timesteps
        self.N = cfg.network_size
        self.M = cfg.batches_per_mc_run
        self.P = cfg.total_paths
        self.rank = rank
        self.world_size = world_size
        self.device = device
        self.dim = cfg.dim
        self._math = _lib.MATH_HW if cfg.math == "hw" else 0
        self.store_mode = _lib.STORE_ALL if store_paths else _lib.STORE_TERMINAL
        self._sobol = SobolEngine(self.dim, cfg.mc_seed, sobol_skip)
        lo, hi = cfg.arrays()
        self.tables = torch.from_numpy(self._sobol.tables().view("int32")).to(device)
        self.lower = torch.from_numpy(lo).to(device)
        self.upper = torch.from_numpy(hi).to(device)
        self.cursor = torch.zeros(2, dtype=torch.int64, device=device)
        B = batch_size
        contracts = torch.empty((B, self.dim), dtype=torch.float64, device=device)
        real_in = torch.empty((B, self.dim), dtype=model_dtype, device=device)
        self.buffers = StepBuffers(contracts=contracts, real_in=real_in, imag_in=torch.zeros_like(real_in),
                                   targets=torch.empty((B, self.N), dtype=torch.complex64, device=device))
        self.terminal_sum = torch.empty((B, self.A), dtype=torch.float64, device=device)
        self.pitch = int(_lib.lib().smc_path_pitch(self.P, 0))
        rows = self.T if store_paths else 1
        per_contract = self.A * rows * self.pitch * 4
        budget = path_buffer_bytes if path_buffer_bytes is not None else _engine.path_buffer_budget(device)
        max_chunk = max(1, min(B, budget // per_contract))
        if max_chunk < B:
            # several launches: whole rounds of resident workgroups, so no launch ends in a
            # part-filled round (C5: 1171 -> 1024 contracts per launch, 2 full rounds each)
            slots = int(_lib.lib().smc_basket_resident_slots(self.A, self.N, self._math))
            if 0 < slots <= max_chunk:
                max_chunk -= max_chunk % slots
        launches = -(-B // max_chunk)
        self.chunk = -(-B // launches)  # equal launches
        shape = (self.chunk, self.A, rows, self.pitch)
        self._paths_buf = torch.empty(shape, dtype=torch.float32, device=device)
        self.paths = self._paths_buf[..., :self.P]
        self._f32_in = model_dtype == torch.float32
        # sync area of the resident kernel (zero-filled once; every launch leaves its counters zeroed);
        # the engine keeps the terminal sums, so other shapes run the split pair (simulate, then CF)
        self._sync_bytes = sync_bytes(cfg, self.chunk)
        self._sync = torch.zeros(self._sync_bytes, dtype=torch.uint8, device=device) if self._sync_bytes else None
        self.kernel_name = _lib.lib().smc_basket_train_targets_kernel(
            self.A, self.T, self.N, self.M, 1 if self._sync is not None else 0, 1).decode()

    @property
    def exchanges(self) -> bool:
        """The step's path launch has workgroups that wait for each other (the resident basket kernel)."""
        return self.kernel_name == "basket_resident_kernel"

    def check_status(self, stream: torch.cuda.Stream | None = None) -> None:
        """SmcError(SMC_ERR_EXCHANGE_TIMEOUT) if a resident launch gave up on a partner slice since the
        last check (engine.check_sync_status)."""
        check_sync_status(self._sync, stream)

    @property
    def global_batch(self) -> int:
        return self.B * self.world_size

    def algorithmic_bytes_per_contract(self) -> int:
        rows = self.T if self.store_mode == _lib.STORE_ALL else 1
        return self.A * rows * self.P * 4 + self.A * self.P * 4 + self.N * 8 + self.dim * 8

    def set_position(self, sobol_index: int, ordinal: int) -> None:
        self.cursor.copy_(torch.tensor([sobol_index, ordinal], dtype=torch.int64), non_blocking=False)

    def make_slot(self) -> StepBuffers:
        """Another set of step outputs (see TrainingEngine.make_slot)."""
        b = self.buffers
        return StepBuffers(contracts=torch.empty_like(b.contracts), real_in=torch.empty_like(b.real_in),
                           imag_in=b.imag_in, targets=torch.empty_like(b.targets))

    def enqueue_step(self, out: StepBuffers | None = None) -> StepBuffers:
        b = out if out is not None else self.buffers
        offset = self.rank * self.B
        draw_device(self.tables, self.dim, self.cursor[0:1], offset, self.B, self.lower, self.upper, b.contracts,
                    b.real_in if self._f32_in else None)
        if not self._f32_in:
            b.real_in.copy_(b.contracts)
        self.launch_targets(_lib.stream_handle(), _lib.ptr(self.cursor[1:2]), offset, b)
        self.cursor.add_(self.global_batch)
        return b

    def launch_targets(self, stream: int | None, ordinal_ptr: int | None, ordinal0: int,
                       b: StepBuffers | None = None) -> None:
        b = b if b is not None else self.buffers
        _lib.check(_lib.lib().smc_basket_train_targets(
            _lib.ptr(b.contracts), self.B, self.A, self.T, self.N, self.M, self.cfg.mc_seed, ordinal_ptr, ordinal0,
            self._math, 1 if self.cfg.normalize else 0, self.store_mode, _lib.ptr(self._paths_buf), self.pitch,
            self.chunk, _lib.ptr(self.terminal_sum), _lib.ptr(b.targets), _lib.ptr(self._sync), self._sync_bytes,
            stream))


def use_basket_engine(pricer, cfg: BasketConfig, *, store_paths: bool = True) -> None:
    """Make ``pricer`` train on basket contracts: its training sessions build a ``BasketEngine``
    instead of the single-asset engine.  The pricer's CVNN must take ``cfg.dim`` inputs."""
    def factory(p, batch_size: int, device: torch.device, rank: int, world_size: int) -> BasketEngine:
        return BasketEngine(cfg, batch_size, device=device, sobol_skip=0, model_dtype=p._dtype.to_torch(), rank=rank,
                            world_size=world_size, store_paths=store_paths)

    pricer.mc_engine_factory = factory


__all__ = ["BasketConfig", "BasketEngine", "basket_fields", "basket_targets", "default_basket_bounds",
           "use_basket_engine", "MAX_ASSETS"]
