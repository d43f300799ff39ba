"""GBM Monte-Carlo engine API (reference ``src/spectralmc/gbm.py``), backed by the HIP engine.

Public names and semantics follow the reference: ``SimulationParams`` /
``BlackScholesConfig`` + their ``build_*`` validators, and the single-GPU engine
``BlackScholes`` with ``_simulate`` -> ``price`` -> ``price_to_host`` and ``snapshot``.

What changed underneath:
* the normal matrix of contract m is not materialised: ``smc_gbm_simulate`` draws it in
  registers from the counter stream (mc_seed, m, path);
* ``SimulateBlackScholes`` (Numba, gbm.py:224-257) is the HIP path kernel, which also
  returns the per-row sums, so forward normalisation (gbm.py:435-438) is one in-place
  scaling pass (``smc_gbm_normalize``) instead of a mean pass plus a scaling pass;
* ``threads_per_block`` is validated as before but the HIP kernels choose their own
  geometry (wave64, 512-thread workgroups);
* device arrays are torch tensors on the process's GPU, all work on the current stream.
"""

from __future__ import annotations

from math import exp
from typing import Annotated, Literal, TypeAlias

import numpy as np
import torch
from pydantic import BaseModel, ConfigDict, Field

from . import _lib
from .effects import ForwardNormalization, PathScheme
from .errors.async_normals import InvalidShape
from .errors.gbm import (
    GPUMemoryLimitExceeded,
    InvalidBlackScholesConfig,
    InvalidSimulationParams,
    NormalsGenerationFailed,
    NormalsUnavailable,
)
from .models.numerical import Precision
from .result import Failure, Result, Success
from .validation import validate_model

PosFloat = Annotated[float, Field(gt=0)]
NonNegFloat = Annotated[float, Field(ge=0)]
ThreadsPerBlock: TypeAlias = Literal[32, 64, 128, 256, 512, 1024]
NormalsError: TypeAlias = NormalsUnavailable | NormalsGenerationFailed

FIELDS: tuple[str, ...] = ("X0", "K", "T", "r", "d", "v")


class SimulationParams(BaseModel):
    """Immutable run-time parameters of one engine instance (reference gbm.py:77-103)."""

    timesteps: int = Field(..., gt=0)
    network_size: int = Field(..., gt=0)
    batches_per_mc_run: int = Field(..., gt=0)
    threads_per_block: ThreadsPerBlock
    mc_seed: int = Field(..., gt=0)
    buffer_size: int = Field(..., gt=0)
    skip: int = Field(0, ge=0)
    dtype: Precision

    model_config = ConfigDict(frozen=True, extra="forbid")

    def total_paths(self) -> int:
        return self.network_size * self.batches_per_mc_run

    def total_blocks(self) -> int:
        return (self.total_paths() + self.threads_per_block - 1) // self.threads_per_block


def validate_simulation_params_memory(params: SimulationParams) -> Result[SimulationParams, GPUMemoryLimitExceeded]:
    """Soft path-count guard (reference gbm.py:106-137)."""
    total = params.network_size * params.batches_per_mc_run
    limit = 1_000_000_000 if params.dtype == Precision.float32 else 500_000_000
    if total > limit:
        return Failure(GPUMemoryLimitExceeded(total_paths=total, max_paths=limit, network_size=params.network_size,
                                              batches_per_mc_run=params.batches_per_mc_run))
    return Success(params)


class BlackScholesConfig(BaseModel):
    sim_params: SimulationParams
    path_scheme: PathScheme = PathScheme.LOG_EULER
    normalization: ForwardNormalization = ForwardNormalization.NORMALIZE

    model_config = ConfigDict(frozen=True, extra="forbid")


def build_simulation_params(*, timesteps: int, network_size: int, batches_per_mc_run: int,
                            threads_per_block: ThreadsPerBlock, mc_seed: int, buffer_size: int, dtype: Precision,
                            skip: int = 0) -> Result[SimulationParams, InvalidSimulationParams | GPUMemoryLimitExceeded]:
    res = validate_model(SimulationParams, timesteps=timesteps, network_size=network_size,
                         batches_per_mc_run=batches_per_mc_run, threads_per_block=threads_per_block,
                         mc_seed=mc_seed, buffer_size=buffer_size, skip=skip, dtype=dtype)
    if isinstance(res, Failure):
        return Failure(InvalidSimulationParams(error=res.error))
    return validate_simulation_params_memory(res.value)


def build_black_scholes_config(*, sim_params: SimulationParams, path_scheme: PathScheme = PathScheme.LOG_EULER,
                               normalization: ForwardNormalization = ForwardNormalization.NORMALIZE
                               ) -> Result[BlackScholesConfig, InvalidBlackScholesConfig]:
    res = validate_model(BlackScholesConfig, sim_params=sim_params, path_scheme=path_scheme,
                         normalization=normalization)
    if isinstance(res, Failure):
        return Failure(InvalidBlackScholesConfig(error=res.error))
    return res


def scheme_code(scheme: PathScheme) -> int:
    return _lib.SCHEME_LOG_EULER if scheme is PathScheme.LOG_EULER else _lib.SCHEME_SIMPLE_EULER


def normalization_code(norm: ForwardNormalization) -> int:
    return _lib.NORM_NORMALIZE if norm is ForwardNormalization.NORMALIZE else _lib.NORM_RAW


def dtype_code(p: Precision) -> int:
    if p == Precision.float32:
        return _lib.DTYPE_F32
    if p == Precision.float64:
        return _lib.DTYPE_F64
    raise ValueError(f"simulation dtype must be float32 or float64, got {p}")


def time_grid(maturity: float, timesteps: int) -> np.ndarray:
    """``cp.linspace(dt, T, timesteps)`` evaluated in f64 (gbm.py:429), last point exact."""
    return np.linspace(maturity / timesteps, maturity, timesteps, dtype=np.float64)


class BlackScholes:
    """Single-GPU Monte-Carlo pricing engine (one process = one GPU)."""

    class Inputs(BaseModel):
        """One European option contract (reference gbm.py:267-277)."""

        X0: PosFloat
        K: PosFloat
        T: NonNegFloat
        r: float
        d: float
        v: NonNegFloat

        model_config = ConfigDict(frozen=True, extra="forbid")

    class SimResults(BaseModel):
        model_config = ConfigDict(arbitrary_types_allowed=True, extra="forbid")
        times: torch.Tensor
        sims: torch.Tensor
        forwards: torch.Tensor
        df: torch.Tensor

    class PricingResults(BaseModel):
        model_config = ConfigDict(arbitrary_types_allowed=True, extra="forbid")
        put_price_intrinsic: torch.Tensor
        call_price_intrinsic: torch.Tensor
        underlying: torch.Tensor
        put_price: torch.Tensor
        call_price: torch.Tensor

    class HostPricingResults(BaseModel):
        put_price_intrinsic: float
        call_price_intrinsic: float
        underlying: float
        put_convexity: float
        call_convexity: float
        put_price: float
        call_price: float

        model_config = ConfigDict(frozen=True, extra="forbid")

    def __init__(self, cfg: BlackScholesConfig) -> None:
        self._cfg = cfg
        self._sp = cfg.sim_params
        self._torch_dtype = self._sp.dtype.to_torch()
        self._served = self._sp.skip  # normal matrices consumed so far (= next contract ordinal)
        # The reference validates the normal-buffer size against one matrix
        # (async_normals.py:112-125); an invalid size surfaces as NormalsUnavailable.
        sp = self._sp
        self._normals_error = (InvalidShape(rows=sp.timesteps, cols=sp.total_paths())
                               if sp.buffer_size > sp.timesteps * sp.total_paths() else None)

    # ------------------------------------------------------------------ state
    @property
    def config(self) -> BlackScholesConfig:
        return self._cfg

    @property
    def ordinal(self) -> int:
        """Ordinal of the next contract's normal stream (= matrices served)."""
        return self._served

    def advance(self, n: int) -> None:
        """Account for n contracts simulated by the fused trainer kernel."""
        self._served += n

    def snapshot(self) -> Result[BlackScholesConfig, NormalsUnavailable]:
        if self._normals_error is not None:
            return Failure(NormalsUnavailable(error=self._normals_error))
        sp = self._sp.model_copy(update={"skip": self._served}, deep=True)
        return Success(self._cfg.model_copy(update={"sim_params": sp}, deep=True))

    # ------------------------------------------------------------------ engine
    def _device(self) -> torch.device:
        _lib.require_device()
        return torch.device("cuda", torch.cuda.current_device())

    def _contract_tensor(self, inputs: "BlackScholes.Inputs", device: torch.device) -> torch.Tensor:
        row = [float(getattr(inputs, f)) for f in FIELDS]
        return torch.tensor([row], dtype=torch.float64, device=device)

    def _simulate(self, inputs: "BlackScholes.Inputs") -> Result["BlackScholes.SimResults", NormalsError]:
        if self._normals_error is not None:
            return Failure(NormalsUnavailable(error=self._normals_error))
        dev = self._device()
        sp = self._sp
        T, P = sp.timesteps, sp.total_paths()
        contract = self._contract_tensor(inputs, dev)
        sims = torch.empty((T, P), dtype=self._torch_dtype, device=dev)
        rowsum = torch.empty((1, T), dtype=torch.float64, device=dev)
        L = _lib.lib()
        stream = _lib.stream_handle()
        _lib.check(L.smc_gbm_simulate(_lib.ptr(contract), 1, T, P, sp.mc_seed, None, self._served,
                                      scheme_code(self._cfg.path_scheme), dtype_code(sp.dtype), _lib.ptr(sims),
                                      _lib.ptr(rowsum), stream))
        self._served += 1
        times = torch.tensor(time_grid(inputs.T, T), device=dev).to(self._torch_dtype)
        rate = torch.tensor(inputs.r - inputs.d, dtype=self._torch_dtype, device=dev)
        forwards = torch.tensor(inputs.X0, dtype=self._torch_dtype, device=dev) * torch.exp(rate * times)
        df = torch.exp(torch.tensor(-inputs.r, dtype=self._torch_dtype, device=dev) * times)
        if self._cfg.normalization is ForwardNormalization.NORMALIZE:
            _lib.check(L.smc_gbm_normalize(_lib.ptr(contract), 1, T, P, dtype_code(sp.dtype), _lib.ptr(sims),
                                           _lib.ptr(rowsum), stream))
        return Success(self.SimResults(times=times, sims=sims, forwards=forwards, df=df))

    def price(self, *, inputs: "BlackScholes.Inputs",
              sr_result: "Result[BlackScholes.SimResults, NormalsError] | None" = None
              ) -> Result["BlackScholes.PricingResults", NormalsError]:
        sim = sr_result or self._simulate(inputs)
        if isinstance(sim, Failure):
            return sim
        sr = sim.value
        F, df_last = sr.forwards[-1], sr.df[-1]
        K = torch.tensor(inputs.K, dtype=self._torch_dtype, device=sr.sims.device)
        terminal = sr.sims[-1]
        zero = torch.zeros((), dtype=self._torch_dtype, device=sr.sims.device)
        return Success(self.PricingResults(
            put_price_intrinsic=df_last * torch.maximum(K - F, zero),
            call_price_intrinsic=df_last * torch.maximum(F - K, zero),
            underlying=terminal,
            put_price=df_last * torch.maximum(K - terminal, zero),
            call_price=df_last * torch.maximum(terminal - K, zero),
        ))

    def get_host_price(self, pr: "BlackScholes.PricingResults") -> "BlackScholes.HostPricingResults":
        put_intr = float(pr.put_price_intrinsic.item())
        call_intr = float(pr.call_price_intrinsic.item())
        put = float(pr.put_price.mean().item())
        call = float(pr.call_price.mean().item())
        return self.HostPricingResults(put_price_intrinsic=put_intr, call_price_intrinsic=call_intr,
                                       underlying=float(pr.underlying.mean().item()),
                                       put_convexity=put - put_intr, call_convexity=call - call_intr,
                                       put_price=put, call_price=call)

    def price_to_host(self, inputs: "BlackScholes.Inputs") -> Result["BlackScholes.HostPricingResults", NormalsError]:
        res = self.price(inputs=inputs)
        if isinstance(res, Failure):
            return res
        return Success(self.get_host_price(res.value))


def intrinsic_values(contract: "BlackScholes.Inputs") -> tuple[float, float, float]:
    """(discount, forward, strike) used by ``predict_price`` (gbm_trainer.py:1746-1749)."""
    return exp(-contract.r * contract.T), contract.X0 * exp((contract.r - contract.d) * contract.T), contract.K


__all__ = ("BlackScholes", "BlackScholesConfig", "SimulationParams", "ThreadsPerBlock",
           "build_black_scholes_config", "build_simulation_params", "validate_simulation_params_memory")
