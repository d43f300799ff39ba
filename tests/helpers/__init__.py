"""Test helpers with the same names the reference's tests import from ``tests.helpers``
(reference tests/helpers/factories.py, result_utils.py, constants.py) — written for this
package so ``tests/test_e2e/test_full_stack_cvnn_pricer.py`` runs unchanged."""

from __future__ import annotations

import random
from typing import TypeVar

import numpy as np
import torch

from spectralmc.cvnn_factory import ActivationCfg, ActivationKind, ExplicitWidth, LinearCfg, build_cvnn_config, build_model
from spectralmc.effects import ForwardNormalization, PathScheme
from spectralmc.gbm import (
    BlackScholes,
    BlackScholesConfig,
    SimulationParams,
    ThreadsPerBlock,
    build_black_scholes_config,
    build_simulation_params,
)
from spectralmc.gbm_trainer import GbmCVNNPricerConfig, TrainingConfig, build_training_config
from spectralmc.models.numerical import Precision
from spectralmc.models.torch import AdamOptimizerState, Device, FullPrecisionDType
from spectralmc.result import Failure, Result, Success
from spectralmc.sobol_sampler import DomainBounds, build_bound_spec, build_domain_bounds
from spectralmc.validation import validate_model

T = TypeVar("T")
E = TypeVar("E")

DEFAULT_TIMESTEPS = 100
DEFAULT_NETWORK_SIZE = 1024
DEFAULT_BATCHES_PER_RUN = 8
DEFAULT_THREADS_PER_BLOCK: ThreadsPerBlock = 256
DEFAULT_MC_SEED = 42
DEFAULT_BUFFER_SIZE = 10_000
RTOL_FLOAT32, ATOL_FLOAT32 = 1e-5, 1e-6
RTOL_FLOAT64, ATOL_FLOAT64 = 1e-10, 1e-12


def expect_success(result: Result[T, E]) -> T:
    if isinstance(result, Failure):
        raise AssertionError(f"expected Success, got Failure: {result.error!r}")
    return result.value


def expect_failure(result: Result[T, E]) -> E:
    if isinstance(result, Success):
        raise AssertionError(f"expected Failure, got Success: {result.value!r}")
    return result.error


def seed_all_rngs(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def make_test_cvnn(*, n_inputs: int, n_outputs: int, seed: int, dtype: torch.dtype,
                   device: torch.device | str = Device.cuda.to_torch(), hidden_width: int = 32,
                   add_output_layer: bool = True, hidden_layers: int = 1):
    layers = [LinearCfg(width=ExplicitWidth(value=hidden_width),
                        activation=ActivationCfg(kind=ActivationKind.MOD_RELU)) for _ in range(hidden_layers)]
    if add_output_layer:
        layers.append(LinearCfg(width=ExplicitWidth(value=n_outputs)))
    cfg = expect_success(build_cvnn_config(dtype=expect_success(FullPrecisionDType.from_torch(dtype)),
                                           layers=layers, seed=seed))
    model = expect_success(build_model(n_inputs=n_inputs, n_outputs=n_outputs, cfg=cfg))
    return model.to(device, dtype)


def make_domain_bounds(*, x0=(0.001, 10_000.0), k=(0.001, 20_000.0), t=(0.0, 10.0), r=(-0.20, 0.20),
                       d=(-0.20, 0.20), v=(0.0, 2.0)) -> DomainBounds[BlackScholes.Inputs]:
    spec = {name: expect_success(build_bound_spec(lo, hi))
            for name, (lo, hi) in (("X0", x0), ("K", k), ("T", t), ("r", r), ("d", d), ("v", v))}
    return expect_success(build_domain_bounds(BlackScholes.Inputs, spec))


def make_simulation_params(timesteps: int = DEFAULT_TIMESTEPS, network_size: int = DEFAULT_NETWORK_SIZE,
                           batches_per_mc_run: int = DEFAULT_BATCHES_PER_RUN,
                           threads_per_block: ThreadsPerBlock = DEFAULT_THREADS_PER_BLOCK,
                           mc_seed: int = DEFAULT_MC_SEED, buffer_size: int = DEFAULT_BUFFER_SIZE, skip: int = 0,
                           dtype: Precision = Precision.float32) -> SimulationParams:
    return expect_success(build_simulation_params(timesteps=timesteps, network_size=network_size,
                                                  batches_per_mc_run=batches_per_mc_run,
                                                  threads_per_block=threads_per_block, mc_seed=mc_seed,
                                                  buffer_size=buffer_size, skip=skip, dtype=dtype))


def make_black_scholes_config(sim_params: SimulationParams | None = None,
                              path_scheme: PathScheme = PathScheme.LOG_EULER,
                              normalization: ForwardNormalization = ForwardNormalization.NORMALIZE
                              ) -> BlackScholesConfig:
    return expect_success(build_black_scholes_config(sim_params=sim_params or make_simulation_params(),
                                                     path_scheme=path_scheme, normalization=normalization))


def make_gbm_cvnn_config(model, global_step: int = 0, sim_params: SimulationParams | None = None,
                         bs_config: BlackScholesConfig | None = None,
                         domain_bounds: DomainBounds[BlackScholes.Inputs] | None = None, sobol_skip: int = 0,
                         optimizer_state: AdamOptimizerState | None = None) -> GbmCVNNPricerConfig:
    sp = sim_params or make_simulation_params()
    cpu_rng = torch.get_rng_state().numpy().tobytes()
    gpu_rngs = ([torch.cuda.get_rng_state(device=i).numpy().tobytes() for i in range(torch.cuda.device_count())]
                if torch.cuda.is_available() else [])
    return expect_success(validate_model(
        GbmCVNNPricerConfig, cfg=bs_config or make_black_scholes_config(sim_params=sp),
        domain_bounds=domain_bounds or make_domain_bounds(), cvnn=model, optimizer_state=optimizer_state,
        global_step=global_step, sobol_skip=sobol_skip, torch_cpu_rng_state=cpu_rng,
        torch_cuda_rng_states=gpu_rngs))


def make_training_config(*, num_batches: int, batch_size: int, learning_rate: float = 1.0e-2) -> TrainingConfig:
    return expect_success(build_training_config(num_batches=num_batches, batch_size=batch_size,
                                                learning_rate=learning_rate))


def max_param_diff(a, b) -> float:
    return max((float((pa - pb).abs().max()) for pa, pb in zip(a.parameters(), b.parameters(), strict=True)),
               default=0.0)


__all__ = ["expect_success", "expect_failure", "seed_all_rngs", "make_test_cvnn", "make_domain_bounds",
           "make_simulation_params", "make_black_scholes_config", "make_gbm_cvnn_config", "make_training_config",
           "max_param_diff", "ThreadsPerBlock", "DEFAULT_TIMESTEPS", "DEFAULT_NETWORK_SIZE",
           "DEFAULT_BATCHES_PER_RUN", "DEFAULT_THREADS_PER_BLOCK", "DEFAULT_MC_SEED", "DEFAULT_BUFFER_SIZE",
           "RTOL_FLOAT32", "ATOL_FLOAT32", "RTOL_FLOAT64", "ATOL_FLOAT64"]


def poisoned(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """An output buffer for a kernel under test, pre-filled with NaN (floating / complex) or a sentinel
    (integers) instead of ``torch.empty``: the caching allocator often hands a test the block a previous,
    correct call just filled, so an element a kernel never writes would otherwise pass unseen."""
    t = torch.empty(shape, dtype=dtype, device=device)
    if dtype.is_floating_point or dtype.is_complex:
        return t.fill_(float("nan"))
    return t.fill_(-0x5A5A5A5A if dtype in (torch.int32, torch.int64) else 0x5A)


def poisoned_like(x: torch.Tensor) -> torch.Tensor:
    return poisoned(x.shape, x.dtype, x.device)


def assert_rows_equal(got, want, err_msg: str = "", chunk: int | None = None) -> None:
    """``np.testing.assert_array_equal`` whose failure names the rows (the first axis: contracts, points) that
    differ, with (row within its launch) mod 8: the XCD the dispatcher deals workgroup w of a launch to when
    contract b runs on workgroup b (paths_kernel, cf_kernel, contract_kernel; ``chunk`` = contracts per
    launch of a chunked step).  A recurrence of a one-XCD fault (DESIGN.md section 3.2b') then carries its
    location."""
    got, want = np.asarray(got), np.asarray(want)
    if got.shape != want.shape or got.ndim == 0:
        np.testing.assert_array_equal(got, want, err_msg=err_msg)
        return
    g, w = got.reshape(got.shape[0], -1), want.reshape(want.shape[0], -1)
    same = (g == w) | (np.isnan(g) & np.isnan(w)) if np.issubdtype(g.dtype, np.inexact) else (g == w)
    bad = np.flatnonzero(~same.all(axis=1))
    if bad.size == 0:
        return
    local = bad % chunk if chunk else bad
    xcd = np.bincount(local % 8, minlength=8)
    cnt = (~same[bad]).sum(axis=1)
    unwritten = int(np.isnan(g[bad]).all(axis=1).sum()) if np.issubdtype(g.dtype, np.inexact) else 0
    raise AssertionError(
        f"{err_msg}: {bad.size} of {g.shape[0]} rows differ ({int(cnt.sum())} values, {unwritten} rows all NaN:"
        f" never written); rows {bad[:24].tolist()}"
        f"{' ...' if bad.size > 24 else ''}; row-in-launch mod 8 histogram {xcd.tolist()}"
        + (f" (chunk {chunk})" if chunk else "") + f"; first row {int(bad[0])}: got {g[bad[0]][:4]} want {w[bad[0]][:4]}")
