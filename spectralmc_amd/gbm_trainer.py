"""GbmCVNNPricer: Sobol contracts -> GBM Monte-Carlo -> CF targets -> CVNN + Adam
(reference ``src/spectralmc/gbm_trainer.py``).

Same public API and step semantics as the reference trainer; the execution model is
MI355X-first:

* one HIP stream, no host synchronisation inside a step: the Monte-Carlo side is two
  launches (engine.py), the CVNN side is torch on hipBLASLt/rocBLAS;
* after ``warmup_steps`` eager steps the whole step (contracts, targets, forward, MSE,
  backward, Adam, grad norm, cursor advance) is captured once as a hipGraph and replayed
  (``torch.cuda.CUDAGraph`` is HIP graphs on ROCm);
* gradients live in one flat buffer, so data-parallel training (one process per GPU,
  ``torch.distributed`` "nccl" = RCCL) needs exactly one all-reduce per step (spectralmc_amd/dp.py);
* loss / grad-norm stay on the device; the host reads them once, after the last step.

Step semantics restated from the reference (``_run_batch`` 1532-1597, ``_torch_step`` 819-835):
    contracts = Sobol(seed=mc_seed)[sobol_skip : sobol_skip + B]  (scaled into the domain bounds)
    targets[b] = mean_m FFT_N(put payoff of contract b's normalised paths, batch m)
    loss = mse(Re pred, Re targets) + mse(Im pred, Im targets);  backward;  Adam.step()
    grad_norm = || all grads ||_2 (clip_grad_norm_(params, inf) after the step)
    sobol_skip += B; normal ordinal += B; global_step += 1
"""

from __future__ import annotations

import asyncio
import math
import time
import weakref
import warnings
from dataclasses import dataclass
from typing import Callable, Iterable, Literal, Protocol, Sequence, runtime_checkable

import numpy as np
import torch
from pydantic import BaseModel, ConfigDict, PositiveInt, ValidationError

from . import _lib
from .cvnn import ComplexLinear
from .engine import WHOLE_CONTRACT_KERNELS, StepBuffers, TrainingEngine
from .errors.gbm import EngineFailure, NormalsUnavailable
from .errors.sampler import SamplerValidationFailed, SequenceExhausted
from .errors.trainer import (
    InvalidTrainerConfig,
    InvalidTrainingConfig,
    OptimizerStateSerializationFailed,
    PredictionFailed,
    SamplerInitFailed,
    TrainerError,
)
from .gbm import FIELDS, BlackScholes, BlackScholesConfig, SimulationParams
from .models.cpu_gpu_transfer import module_state_device_dtype
from .models.numerical import Precision
from .models.torch import AdamOptimizerState, AnyDType, Device, FullPrecisionDType, build_adam_optimizer_state
from .result import Failure, Result, Success
from .sobol_sampler import MAX_POINTS, DomainBounds, SobolSampler, build_sobol_config
from .validation import validate_model

nn = torch.nn
optim = torch.optim

LOGGER_NAME = __name__


# ============================================================================ commit plans
@dataclass(frozen=True)
class NoCommit:
    kind: Literal["NoCommit"] = "NoCommit"


@dataclass(frozen=True)
class FinalCommit:
    kind: Literal["FinalCommit"] = "FinalCommit"
    commit_message_template: str = "Training checkpoint at step {step}"


@dataclass(frozen=True)
class IntervalCommit:
    interval: PositiveInt
    kind: Literal["IntervalCommit"] = "IntervalCommit"
    commit_message_template: str = "Training checkpoint at step {step}"


@dataclass(frozen=True)
class FinalAndIntervalCommit:
    interval: PositiveInt
    kind: Literal["FinalAndIntervalCommit"] = "FinalAndIntervalCommit"
    commit_message_template: str = "Training checkpoint at step {step}"


CommitPlan = NoCommit | FinalCommit | IntervalCommit | FinalAndIntervalCommit


# ============================================================================ protocol & configs
@runtime_checkable
class ComplexValuedModel(Protocol):
    """``(real, imag) -> (real, imag)`` network plus the nn.Module subset the trainer uses."""

    def __call__(self, __real: torch.Tensor, __imag: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]: ...
    def parameters(self) -> Iterable[nn.Parameter]: ...
    def named_parameters(self) -> Iterable[tuple[str, nn.Parameter]]: ...
    def state_dict(self, destination=None, prefix: str = "", keep_vars: bool = False) -> dict[str, torch.Tensor]: ...
    def load_state_dict(self, state_dict: dict[str, torch.Tensor], strict: bool = True) -> None: ...
    def to(self, device: torch.device, dtype: torch.dtype) -> nn.Module: ...
    def train(self, mode: bool = True) -> None: ...
    def eval(self) -> None: ...


@dataclass(frozen=True)
class TrainingConfig:
    """num_batches steps of batch_size contracts per rank (per GPU) at learning_rate."""

    num_batches: int
    batch_size: int
    learning_rate: float


def build_training_config(*, num_batches: int, batch_size: int, learning_rate: float
                          ) -> Result[TrainingConfig, InvalidTrainingConfig]:
    def bad(msg: str) -> Failure[InvalidTrainingConfig]:
        return Failure(InvalidTrainingConfig(num_batches=num_batches, batch_size=batch_size,
                                             learning_rate=learning_rate, message=msg))

    if num_batches <= 0:
        return bad("num_batches must be > 0")
    if batch_size <= 0:
        return bad("batch_size must be > 0")
    if not (0.0 < learning_rate < 1.0):
        return bad("learning_rate must be in (0, 1)")
    return Success(TrainingConfig(num_batches=num_batches, batch_size=batch_size, learning_rate=learning_rate))


class GbmCVNNPricerConfig(BaseModel):
    """Frozen, resumable trainer snapshot (reference gbm_trainer.py:301-313)."""

    cfg: BlackScholesConfig
    domain_bounds: DomainBounds[BlackScholes.Inputs]
    cvnn: ComplexValuedModel
    optimizer_state: AdamOptimizerState | None = None
    global_step: int = 0
    sobol_skip: int = 0
    torch_cpu_rng_state: bytes | None = None
    torch_cuda_rng_states: list[bytes] | None = None

    model_config = ConfigDict(arbitrary_types_allowed=True, frozen=True, extra="forbid")


def build_gbm_cvnn_pricer_config(**kwargs: object) -> Result[GbmCVNNPricerConfig, ValidationError]:
    return validate_model(GbmCVNNPricerConfig, **kwargs)


@dataclass(frozen=True)
class StepMetrics:
    step: int
    batch_time: float
    loss: float
    grad_norm: float
    lr: float
    optimizer: optim.Optimizer
    model: ComplexValuedModel


StepLogger = Callable[[StepMetrics], None]


@dataclass(frozen=True)
class TrainingResult:
    updated_config: GbmCVNNPricerConfig
    final_loss: float
    total_batches: int
    final_grad_norm: float


@dataclass(frozen=True)
class _BatchState:
    sobol_skip: int
    global_step: int
    loss: float
    grad_norm: float


# ============================================================================ creation errors
@dataclass(frozen=True)
class DeviceDTypeError:
    kind: Literal["DeviceDTypeError"] = "DeviceDTypeError"
    message: str = ""
    underlying_error: object | None = None


@dataclass(frozen=True)
class DeviceNotCUDA:
    kind: Literal["DeviceNotCUDA"] = "DeviceNotCUDA"
    device: Device = Device.cpu
    message: str = "GbmCVNNPricer requires a GPU (ROCm) device"


@dataclass(frozen=True)
class CudaUnavailableForRNGRestore:
    kind: Literal["CudaUnavailableForRNGRestore"] = "CudaUnavailableForRNGRestore"
    message: str = "Cannot restore GPU RNG state: no GPU available but the checkpoint carries one"


GbmPricerError = DeviceDTypeError | DeviceNotCUDA | CudaUnavailableForRNGRestore


def _gpu_count() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def _split_inputs(inputs: Sequence[BlackScholes.Inputs], *, dtype: torch.dtype, device: torch.device
                  ) -> tuple[torch.Tensor, torch.Tensor]:
    """Pydantic contracts -> (real, imag=0) CVNN input rows (gbm_trainer.py:1775-1783)."""
    rows = [[float(getattr(c, f)) for f in FIELDS] for c in inputs]
    real = torch.tensor(rows, dtype=dtype, device=device)
    return real, torch.zeros_like(real)


# ============================================================================ the step
class _StepProgram:
    """The per-step device program, split into a Monte-Carlo part and a network part so that
    the two can run on separate HIP streams (see TrainingSession):

        mc(k)      Sobol draw + fused paths/targets launch into step slot k (+ cursor)
        handoff(k) engines that cannot write a slot: copy their buffers into slot k
        fwd_bwd(k) CVNN forward, spectral MSE, backward into the flat [grads..., loss] buffer
        reduce()   data-parallel mean of the flat buffer (one RCCL all-reduce)
        update()   Adam + post-step grad norm

    Each part runs eagerly or is recorded once into a hipGraph and replayed."""

    SLOTS = 4

    def __init__(self, pricer: "GbmCVNNPricer", engine: TrainingEngine, adam: optim.Optimizer,
                 params: list[nn.Parameter], dp) -> None:
        self.pricer = pricer
        self.engine = engine
        self.adam = adam
        self.params = params
        self.dp = dp
        dev = params[0].device
        numel = sum(p.numel() for p in params)
        # flat [grads..., loss] buffer: one all-reduce carries both in data-parallel runs
        self.flat = torch.zeros(numel + 1, dtype=params[0].dtype, device=dev)
        off = 0
        for p in params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.loss_slot = self.flat[numel:]
        self.loss = torch.zeros((), dtype=params[0].dtype, device=dev)
        self.grad_norm = torch.zeros((), dtype=params[0].dtype, device=dev)
        eb = engine.buffers
        # SLOTS step slots: step s's MC part writes slot s % SLOTS directly while the network parts
        # of earlier steps may still read theirs (no hand-off copy between MC launches).  A network
        # part cannot run beside the path kernel (which holds every CU's registers), so its kernels
        # run in the gaps between path kernels and one network part completes two path kernels
        # after its own: with 4 slots the MC part never waits for a network part that just finished
        self.direct = hasattr(engine, "make_slot")
        self.slots = ([engine.make_slot() for _ in range(self.SLOTS)] if self.direct else
                      [StepBuffers(contracts=torch.empty_like(eb.contracts), real_in=torch.empty_like(eb.real_in),
                                   imag_in=eb.imag_in, targets=torch.empty_like(eb.targets))
                       for _ in range(self.SLOTS)])
        self.real_in = [b.real_in for b in self.slots]
        self.imag_in = eb.imag_in  # constant zeros
        self.targets = [b.targets for b in self.slots]
        self.mc_graphs: list[torch.cuda.CUDAGraph] = []  # per slot
        #: when a list: HIP events recorded around each data-parallel all-reduce on the stream that runs it
        #: (bench.py reports the all-reduce time per step)
        self.ar_events: list[tuple[torch.cuda.Event, torch.cuda.Event]] | None = None
        self.step_graphs: list[torch.cuda.CUDAGraph] = []  # per slot: MC + network (one stream)
        self.nn_graphs: list[list[torch.cuda.CUDAGraph]] = []  # per slot
        # network half on the fused HIP kernels when the architecture allows (net.py)
        self.fused = None
        if getattr(pricer, "fused_network", False):
            from .net import FusedNetworkStep, UnsupportedNetwork

            compute = getattr(pricer, "network_compute", "auto")
            try:
                self.fused = FusedNetworkStep(pricer._cvnn, adam, params, self.flat, self.loss, self.grad_norm,
                                              batch=eb.real_in.shape[0], fuse_adam=dp is None, compute=compute)
            except UnsupportedNetwork:
                if compute in ("mfma", "bf16"):  # an explicit kernel request never degrades silently
                    raise
                self.fused = None

    # -- pieces -------------------------------------------------------------------------
    def mc(self, slot: int, stream: int | None = None) -> None:
        """stream: the hipStream_t to launch on (None: the current stream)."""
        out = self.slots[slot] if self.direct else None
        lanes = getattr(self.engine, "lanes", 1)
        if lanes > 1:
            # slot k's step runs on lane k % lanes; steps take the lanes in turn because lanes divides
            # SLOTS (GbmCVNNPricer.open_session rejects other values)
            if self.SLOTS % lanes:
                raise ValueError(f"{lanes} MC lanes do not divide the {self.SLOTS} step slots")
            self.engine.enqueue_step(out, lane=slot, **({} if stream is None else {"stream": stream}))
        else:
            self.engine.enqueue_step(out, **({} if stream is None else {"stream": stream}))

    def handoff(self, slot: int) -> None:
        if self.direct:
            return
        eb = self.engine.buffers
        self.real_in[slot].copy_(eb.real_in)
        self.targets[slot].copy_(eb.targets)

    def fwd_bwd(self, slot: int, stream: int | None = None) -> None:
        if self.fused is not None:
            self.fused.fwd_bwd(self.real_in[slot], self.imag_in, self.targets[slot], stream=stream)
            return
        self.flat.zero_()
        targets = self.targets[slot]
        pred_r, pred_i = self.pricer._cvnn(self.real_in[slot], self.imag_in)
        loss = nn.functional.mse_loss(pred_r, torch.real(targets)) + nn.functional.mse_loss(
            pred_i, torch.imag(targets))
        loss.backward()
        self.loss_slot.copy_(loss.detach().reshape(1))

    def update(self, stream: int | None = None) -> None:
        if self.fused is not None:
            if not self.fused.fuse_adam:  # data-parallel: Adam after the all-reduce
                self.fused.adam(stream=stream)
            return
        self.adam.step()
        grads = [p.grad for p in self.params]
        self.grad_norm.copy_(torch.linalg.vector_norm(torch.stack(torch._foreach_norm(grads, 2.0)), 2.0))
        self.loss.copy_(self.loss_slot[0])

    def reduce(self) -> None:
        if self.dp is None:
            return
        if self.ar_events is None:
            self.dp.all_reduce_mean(self.flat)
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.dp.all_reduce_mean(self.flat)
        e1.record()
        self.ar_events.append((e0, e1))

    # -- eager / graph execution ------------------------------------------------------------
    @property
    def captured(self) -> bool:
        return bool(self.mc_graphs or self.step_graphs)

    def capture(self, mc_stream: torch.cuda.Stream, nn_stream: torch.cuda.Stream) -> None:
        """Record the MC part per slot (own memory pool: it may replay concurrently with the
        network graphs) and the network part per slot (two graphs around the all-reduce when
        data-parallel).  On one stream without data parallelism the whole step (MC part, network
        part, Adam) is one graph per slot.  Capturing launches nothing, so the device cursor does
        not move."""
        if mc_stream is nn_stream and self.dp is None:
            pool = torch.cuda.graph_pool_handle()
            self.step_graphs = []
            for slot in range(self.SLOTS):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, stream=mc_stream):
                    self.mc(slot)
                    self.handoff(slot)
                    self.fwd_bwd(slot)
                    self.update()
                self.step_graphs.append(g)
            return
        graphs = []
        mc_pool = torch.cuda.graph_pool_handle()
        for slot in range(self.SLOTS):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=mc_pool, stream=mc_stream):
                self.mc(slot)
            graphs.append(g)
        pool = torch.cuda.graph_pool_handle()
        self.nn_graphs = []
        upd = None
        for slot in range(self.SLOTS):
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, pool=pool, stream=nn_stream):
                self.fwd_bwd(slot)
                if self.dp is None:
                    self.update()
            if self.dp is None:
                self.nn_graphs.append([g1])
                continue
            if upd is None:
                upd = torch.cuda.CUDAGraph()
                with torch.cuda.graph(upd, pool=pool, stream=nn_stream):
                    self.update()
            self.nn_graphs.append([g1, upd])
        self.mc_graphs = graphs

    def run_step(self, slot: int) -> None:
        """The whole step on the current stream (one graph when captured on one stream)."""
        if self.step_graphs:
            self.step_graphs[slot].replay()
            return
        self.run_mc(slot)
        self.handoff(slot)
        self.run_nn(slot)

    def run_mc(self, slot: int, stream: int | None = None) -> None:
        """stream: eager launches on this hipStream_t (replays use the current stream)."""
        if self.mc_graphs:
            self.mc_graphs[slot].replay()
        else:
            self.mc(slot, stream)

    @property
    def explicit_streams(self) -> bool:
        """The eager step takes explicit stream handles (no torch op in it: direct slots, the one-call
        smc_train_step MC part, fused network, no all-reduce), so it needs no torch stream contexts (their host
        cost bounds short steps)."""
        return (self.direct and getattr(self.engine, "_uses_train_step", False) and self.fused is not None and
                self.dp is None and not self.captured)

    def run_nn(self, slot: int, stream: int | None = None) -> None:
        if not self.nn_graphs:
            self.fwd_bwd(slot, stream)
            self.reduce()
            self.update(stream)
            return
        graphs = self.nn_graphs[slot]
        graphs[0].replay()
        if len(graphs) == 2:
            self.reduce()
            graphs[1].replay()


# ============================================================================ trainer
GRAPH_MIN_PATH_STEPS = 1 << 27  # GbmCVNNPricer.graph_min_path_steps


class GbmCVNNPricer:
    """Coordinates the MC engine, the CF targets and CVNN optimisation on one GPU (per process)."""

    #: eager steps before the step is captured as a hipGraph (0 disables capture)
    warmup_steps: int = 2
    #: capture only steps of at least this many path-steps (contracts x paths x timesteps): below it every
    #: hipGraph launch cost the GPU more than the eager launches it replaces (the reference's e2e shape, 33.6 M
    #: path-steps: 0.092 ms/step replayed against 0.079-0.082 eager; the lock-step shape, 268 M, equal;
    #: profiles/r05/ab_graphs_short.txt)
    graph_min_path_steps: int = GRAPH_MIN_PATH_STEPS
    #: materialise the full [B][T][P] path matrix each step (the reference kernel's output contract)
    store_paths: bool = True
    #: "hw": hardware f32 transcendentals in the path kernel (throughput mode; parity with the
    #: CPU path at the stated fp32 tolerance); "portable": IEEE-only polynomial transcendentals,
    #: bit-identical to the oracle's kernel mode (CPU-reproducible paths and targets); "reference":
    #: the reference kernel's own typing (gbm.py:224-257 under Numba: f64 state and step of the f32
    #: normals, f32 stores), float32 simulations only (rows_ref_kernel + cf_kernel); "reference_hw": that step
    #: on the hardware-transcendental f32 normals (within the "hw" tolerance of "reference", 1.4x faster)
    math_mode: str = "hw"
    #: run step s+1's Monte-Carlo part on its own stream, concurrently with step s's network part
    overlap_mc: bool = True
    #: which of the two streams (overlap_mc) gets the high hardware-queue priority: "network",
    #: "mc" or "none"
    high_priority_stream: str = "network"
    #: with overlap_mc: MC launches of consecutive steps alternate over this many streams (engine
    #: lanes: own cursor, sync area and path scratch each, every contract from the launch's queue), so
    #: step s + 1's path kernel starts on the CUs step s's frees in its tail.  Taken only where the
    #: engine allows it (one whole-contract resident launch per step); with the network on its own
    #: CUs (network_cus) C2 runs 3.08 -> 2.98 ms/step
    mc_lanes: int = 2
    #: ... and this many when the fused network is narrow (every layer input < 128 complex features: the
    #: fb_kernel path on network_cus CUs) and one path launch does at least mc_lanes_long_path_steps
    #: path-steps.  Round 5, three boxes: C2 2.69-2.79 / 2.94-2.95 / 2.69-2.79 ms/step with 4 lanes against
    #: 2.95-3.00 with 2 (profiles/r05/ab_c2_lanes4.txt; round 4 had measured one box better, one equal): four
    #: launches in flight keep more write streams open.  Not taken at the lock-step and e2e shapes (slower
    #: there, profiles/r04/mc_lanes.txt) nor beside the wide C2/H=256 network (3.03 -> 3.07)
    mc_lanes_long: int = 4
    mc_lanes_long_path_steps: int = 1 << 30
    #: ... and this many for launches below network_cu_min_path_steps path-steps, where the network chain, not the
    #: path launch, sets the step time and a second launch in flight only slows it (the reference's e2e shape:
    #: one lane 0.095-0.097 against two 0.100-0.101 ms/step; profiles/r05/netcus_short_shapes.txt)
    mc_lanes_short: int = 1
    #: with engine lanes: CUs reserved for the network part (CU-masked HIP streams, the path kernels on
    #: the rest; 0: none) and their choice of CU ids ("low": the lowest logical ids, which measured
    #: best; "spread": evenly over the id range)
    network_cus: int = 32
    #: the same for a wide fused network (a layer input of >= 256 real features: the layered MFMA GEMMs,
    #: C2/H=256 ~0.26 ms of whole-chip work): more CUs, so the network still hides under the path kernel
    network_cus_wide: int = 64
    network_cu_pattern: str = "low"
    #: ... when one path launch does at least this many path-steps (contracts x paths x T): beside a
    #: shorter launch a 32-CU network outlasts it (the reference's e2e shape, 3.4e7 path-steps: 0.222
    #: ms/step on 32 masked CUs against 0.114 unmasked; the lock-step shape, 2.7e8: 0.308 masked against
    #: 0.329; profiles/r04/netcus_small_shapes.jsonl)
    network_cu_min_path_steps: int = 1 << 27
    #: ... and below it this many (0: no masks): beside a short launch half the chip for the network
    #: (e2e shape: 0.110 ms/step unmasked, 0.141 on 64 CUs, 0.101 on 128, 0.111 on 160;
    #: profiles/r04/e2e_network_cus.txt)
    network_cus_small: int = 128
    #: overlap_mc for the rows_kernel / rows_ref_kernel + cf_kernel shapes (f64, the reference typing): True puts
    #: step s's network part beside step s+1's rows launch (a network workgroup fits beside the persistent
    #: workgroups at the f64 register budget); False runs those shapes on one stream;
    #: None (default): overlapped for f64's rows_kernel (box-dependent: 8.35 against 8.43-8.47 ms/step on one
    #: box, 8.64 against 8.50-8.52 on another, profiles/r06/r06_f64_overlap*.txt), one stream for the reference
    #: typing's rows_ref_kernel, whose launch the network's workgroups stretch by more than the network takes
    #: (6.64-6.66 against 7.03-7.10, reference_hw 4.44-4.47 against 4.71-4.72, r06_ref_overlap*.txt)
    overlap_rows: bool | None = None
    #: launches whose workgroups wait for each other (the sliced resident kernel, C3; the resident
    #: basket kernel, C5) need every workgroup of a group co-resident.  A collective that spins on a
    #: few CUs while it waits for a slow peer (RCCL in data-parallel runs) could hold CUs past the
    #: exchange's poll budget; since round 6 a data-parallel session keeps the network part and the
    #: all-reduce (issued on the network stream: dp.RcclComm) on CU-masked CUs of their own and sizes the
    #: exchanging launch to the other CUs, so the launch runs beside the collective as it does on one GPU.
    #: True: enqueue an exchanging launch only after the previous step's network part (and all-reduce) has
    #: completed (round 4-5's data-parallel default); None / False: beside it
    exchange_after_network: bool | None = None
    #: CU masks for the exchanging launches (C3 sliced, C5 basket) with a fused network: None = in data-parallel
    #: runs (the collective on the network's CUs) and, on one GPU, for the sliced resident
    #: kernel (C3: the network on 32 CUs beside the launch, 48.06-48.11 against 48.51-48.64 ms/step; the W = 32
    #: basket launch loses a whole group per XCD to the mask: 51.1 against 46.5, profiles/r06/r06_xmasks.txt);
    #: True = always; False = never
    exchanging_masks: bool | None = None
    #: network forward/backward/Adam on the fused HIP kernels (csrc/cvnn.hip) when the CVNN is a
    #: ComplexLinear + modReLU/zReLU chain; False (or other architectures): torch-ROCm modules
    fused_network: bool = True
    #: fused network kernels (net.FusedNetworkStep): "auto" (f32 on MFMA when the widths fit, else
    #: VALU), "valu", "mfma", or "bf16" (bf16 MFMA operands, f32 master weights / Adam: the
    #: BASELINE configs[2] extension; the reference asserts full precision, gbm_trainer.py:679-686)
    network_compute: str = "auto"

    @staticmethod
    def create(cfg: GbmCVNNPricerConfig) -> Result["GbmCVNNPricer", GbmPricerError]:
        dd = module_state_device_dtype(cfg.cvnn.state_dict())
        if isinstance(dd, Failure):
            return Failure(DeviceDTypeError(message=f"Failed to get device/dtype from CVNN: {dd.error}",
                                            underlying_error=dd.error))
        device, dtype = dd.value
        if device is not Device.cuda:
            return Failure(DeviceNotCUDA(device=device, message=f"Model on {device}, but a GPU is required"))
        if cfg.torch_cuda_rng_states is not None and _gpu_count() == 0:
            return Failure(CudaUnavailableForRNGRestore())
        pricer = GbmCVNNPricer.__new__(GbmCVNNPricer)
        pricer._initialize(cfg, device, dtype)
        return Success(pricer)

    def _initialize(self, cfg: GbmCVNNPricerConfig, device: Device, dtype: AnyDType) -> None:
        self._cfg = cfg.cfg
        self._sim_params: SimulationParams = cfg.cfg.sim_params
        self._cvnn: ComplexValuedModel = cfg.cvnn
        self._domain_bounds = cfg.domain_bounds
        self._optimizer_state = cfg.optimizer_state
        self._global_step = cfg.global_step
        self._sobol_skip = cfg.sobol_skip
        self._device = device
        self._torch_device = next(iter(cfg.cvnn.parameters())).device
        assert isinstance(dtype, FullPrecisionDType), f"CVNN must use a full-precision dtype, got {dtype}"
        self._dtype: FullPrecisionDType = dtype
        assert self._dtype.to_precision() == self._sim_params.dtype, (
            f"Error: gbm sim dtype {self._sim_params.dtype} does not match cvnn dtype {self._dtype}")
        self._complex_dtype: Precision = self._dtype.to_precision().to_complex().unwrap()
        self._mc_engine = BlackScholes(cfg.cfg)
        self._sampler_result = SobolSampler.create(
            BlackScholes.Inputs, self._domain_bounds,
            config=build_sobol_config(seed=self._sim_params.mc_seed, skip=self._sobol_skip).unwrap())
        if cfg.torch_cpu_rng_state is not None:
            torch.set_rng_state(torch.from_numpy(np.frombuffer(cfg.torch_cpu_rng_state, dtype=np.uint8).copy()))
        if cfg.torch_cuda_rng_states is not None:
            count = _gpu_count()
            assert count == len(cfg.torch_cuda_rng_states), (
                f"GPU RNG state count ({len(cfg.torch_cuda_rng_states)}) does not match device count ({count})")
            torch.cuda.set_rng_state_all([torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy())
                                          for s in cfg.torch_cuda_rng_states])

    # ------------------------------------------------------------------ checkpointing
    @property
    def mc_engine(self) -> BlackScholes:
        return self._mc_engine

    def snapshot(self) -> Result[GbmCVNNPricerConfig, NormalsUnavailable]:
        cpu_rng = torch.get_rng_state().cpu().numpy().tobytes()
        cuda_rng = [s.cpu().numpy().tobytes() for s in torch.cuda.get_rng_state_all()] if _gpu_count() else None
        if cuda_rng is None:
            from .errors.gbm import CudaRNGUnavailable

            return Failure(NormalsUnavailable(error=CudaRNGUnavailable(reason="cuda_unavailable")))
        eng = self._mc_engine.snapshot()
        if isinstance(eng, Failure):
            return eng
        res = build_gbm_cvnn_pricer_config(cfg=eng.value, domain_bounds=self._domain_bounds, cvnn=self._cvnn,
                                           optimizer_state=self._optimizer_state, global_step=self._global_step,
                                           sobol_skip=self._sobol_skip, torch_cpu_rng_state=cpu_rng,
                                           torch_cuda_rng_states=cuda_rng)
        if isinstance(res, Failure):
            raise AssertionError(f"GbmCVNNPricerConfig validation failed: {res.error}")
        return res

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _validate_commit_plan(plan: CommitPlan) -> Result[CommitPlan, InvalidTrainerConfig]:
        if isinstance(plan, (IntervalCommit, FinalAndIntervalCommit)) and plan.interval <= 0:
            return Failure(InvalidTrainerConfig(message="commit interval must be positive for blockchain commit plan"))
        return Success(plan)

    @staticmethod
    def _should_commit_now(store, plan: CommitPlan, global_step: int) -> tuple[bool, str]:
        if isinstance(plan, (IntervalCommit, FinalAndIntervalCommit)):
            return store is not None and global_step % plan.interval == 0, plan.commit_message_template
        return False, ""

    @staticmethod
    def _should_commit_final(store, plan: CommitPlan) -> tuple[bool, str]:
        if isinstance(plan, (FinalCommit, FinalAndIntervalCommit)):
            return store is not None, plan.commit_message_template
        return False, ""

    def _torch_step(self, real_in: torch.Tensor, imag_in: torch.Tensor, targets: torch.Tensor,
                    optimizer: optim.Optimizer) -> tuple[torch.Tensor, float]:
        """One eager forward/backward/Adam step (reference semantics, host-synchronising)."""
        pred_r, pred_i = self._cvnn(real_in, imag_in)
        loss = nn.functional.mse_loss(pred_r, torch.real(targets)) + nn.functional.mse_loss(
            pred_i, torch.imag(targets))
        optimizer.zero_grad(set_to_none=True)
        loss.backward()
        optimizer.step()
        grad_norm = float(torch.nn.utils.clip_grad_norm_(self._cvnn.parameters(), float("inf")))
        return loss, grad_norm

    def _make_adam(self, lr: float) -> Result[optim.Optimizer, OptimizerStateSerializationFailed]:
        params = list(self._cvnn.parameters())
        adam = optim.Adam(params, lr=lr, foreach=True, capturable=True)
        if self._optimizer_state is not None:
            sd = self._optimizer_state.to_torch()
            if isinstance(sd, Failure):
                return Failure(OptimizerStateSerializationFailed(
                    message=f"Failed to deserialize optimizer state: {sd.error}"))
            adam.load_state_dict(sd.value)
            for group in adam.param_groups:
                group["capturable"] = True
                group["foreach"] = True
            for p in params:
                st = adam.state.get(p)
                if st and "step" in st:
                    step = st["step"]
                    st["step"] = (step if isinstance(step, torch.Tensor) else torch.tensor(float(step))).to(
                        device=p.device, dtype=torch.float32)
        return Success(adam)

    def _adam_snapshot(self, adam: optim.Optimizer) -> Result[AdamOptimizerState, OptimizerStateSerializationFailed]:
        sd = adam.state_dict()
        sd["state"] = {pid: {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in st.items()}
                       for pid, st in sd["state"].items()}
        res = AdamOptimizerState.from_torch(sd)
        if isinstance(res, Failure):
            return Failure(OptimizerStateSerializationFailed(message=f"Failed to capture optimizer snapshot: {res.error}"))
        return res

    # ------------------------------------------------------------------ training
    def open_session(self, config: TrainingConfig) -> Result["TrainingSession", TrainerError]:
        """Set up a device training session (engine buffers, Adam, step program) for ``config``."""
        if isinstance(self._sampler_result, Failure):
            return Failure(SamplerInitFailed(error=self._sampler_result.error))
        for name in ("mc_lanes", "mc_lanes_long", "mc_lanes_short"):
            lanes = getattr(self, name) if self.overlap_mc else 1
            if not isinstance(lanes, int) or lanes < 1 or _StepProgram.SLOTS % lanes:
                # a lane's device cursor assumes it runs every lanes-th step; the step slots (whose graphs
                # bind a lane) cycle mod SLOTS, so lanes must divide SLOTS
                return Failure(InvalidTrainerConfig(
                    message=f"{name} must divide {_StepProgram.SLOTS} (1, 2 or 4), got {lanes!r}"))
        adam_res = self._make_adam(config.learning_rate)
        if isinstance(adam_res, Failure):
            return adam_res
        from . import dp as _dp

        try:
            return Success(TrainingSession(self, config, self._sampler_result.value, adam_res.value, _dp.current()))
        except _lib.SmcError as exc:
            return Failure(EngineFailure(code=exc.code, message=exc.message))

    def train(self, config: TrainingConfig, *, logger: StepLogger | None = None, blockchain_store=None,
              commit_plan: CommitPlan = NoCommit()) -> Result[TrainingResult, TrainerError]:
        plan = self._validate_commit_plan(commit_plan)
        if isinstance(plan, Failure):
            return plan
        if not isinstance(commit_plan, NoCommit) and blockchain_store is None:
            return Failure(InvalidTrainerConfig(message="commit_plan requires blockchain_store to be provided"))
        if isinstance(self._sampler_result, Failure):
            return Failure(SamplerInitFailed(error=self._sampler_result.error))
        sampler = self._sampler_result.value
        lo, _hi = sampler.bounds
        if not _bounds_always_valid(lo):
            # Rows could violate BlackScholes.Inputs: keep the reference's error by validating
            # every batch on the host (slow path; never taken with positive bounds).
            return self._train_checked(config, sampler, logger, blockchain_store, commit_plan)
        opened = self.open_session(config)
        if isinstance(opened, Failure):
            return opened
        session = opened.value
        try:
            t_prev = time.perf_counter()
            for i in range(config.num_batches):
                stepped = session.step(prefetch_next=i + 1 < config.num_batches)
                if isinstance(stepped, Failure):
                    return stepped
                if logger is not None:
                    # read_metrics synchronises, so with a logger every step ends on the host:
                    # batch_time is the wall time of this step (enqueue -> network done)
                    loss, gn = session.read_metrics()
                    now = time.perf_counter()
                    logger(StepMetrics(step=session.global_step, batch_time=now - t_prev, loss=loss, grad_norm=gn,
                                       lr=config.learning_rate, optimizer=session.adam, model=self._cvnn))
                    t_prev = now
                do_commit, template = self._should_commit_now(blockchain_store, commit_plan, session.global_step)
                if do_commit:
                    session.sync()
                    self._global_step, self._sobol_skip = session.global_step, session.sobol_skip
                    loss, _ = session.read_metrics()
                    self._commit_to_blockchain(blockchain_store, session.adam, template, loss,
                                               batch=session.global_step)
            final_state = session.close()
        except _lib.SmcError as exc:
            if not session._closed:
                session.close_quietly()
            return Failure(EngineFailure(code=exc.code, message=exc.message))
        return self._finish(session.adam, final_state, config, blockchain_store, commit_plan)

    def _train_checked(self, config: TrainingConfig, sampler: SobolSampler, logger, blockchain_store,
                       commit_plan: CommitPlan) -> Result[TrainingResult, TrainerError]:
        """Host-validated variant for domains that admit invalid contracts (e.g. X0 lower <= 0)."""
        adam_res = self._make_adam(config.learning_rate)
        if isinstance(adam_res, Failure):
            return adam_res
        adam = adam_res.value
        self._cvnn.train()
        start = self._sobol_skip
        sobol_skip, global_step = self._sobol_skip, self._global_step
        loss_v, gn = 0.0, 0.0
        try:
            engine = TrainingEngine(self._cfg, sampler, config.batch_size, model_dtype=self._dtype.to_torch(),
                                    device=self._torch_device, store_paths=self.store_paths, math=self.math_mode)
        except _lib.SmcError as exc:
            return Failure(EngineFailure(code=exc.code, message=exc.message))
        engine.set_position(sobol_skip, self._mc_engine.ordinal)
        for _ in range(config.num_batches):
            if sobol_skip + config.batch_size > MAX_POINTS:  # the device draw indexes 30 bits
                sampler.skip(sobol_skip - start)
                return Failure(SamplerInitFailed(error=SequenceExhausted(requested_end=sobol_skip + config.batch_size)))
            t0 = time.perf_counter()
            buf = engine.enqueue_step()
            host = buf.contracts.cpu().numpy()
            for row in host:
                res = validate_model(BlackScholes.Inputs, **{f: float(row[i]) for i, f in enumerate(FIELDS)})
                if isinstance(res, Failure):
                    sampler.skip(sobol_skip - start)
                    return Failure(SamplerInitFailed(error=SamplerValidationFailed(error=res.error)))
            loss, gn = self._torch_step(buf.real_in, buf.imag_in, buf.targets, adam)
            loss_v = float(loss.item())
            sobol_skip += config.batch_size
            global_step += 1
            self._mc_engine.advance(config.batch_size)
            # the same per-step hooks as train(): logger, interval commits (reference _run_batch)
            self._global_step, self._sobol_skip = global_step, sobol_skip
            if logger is not None:
                logger(StepMetrics(step=global_step, batch_time=time.perf_counter() - t0, loss=loss_v, grad_norm=gn,
                                   lr=config.learning_rate, optimizer=adam, model=self._cvnn))
            do_commit, template = self._should_commit_now(blockchain_store, commit_plan, global_step)
            if do_commit:
                self._commit_to_blockchain(blockchain_store, adam, template, loss_v, batch=global_step)
        sampler.skip(sobol_skip - start)
        return self._finish(adam, _BatchState(sobol_skip, global_step, loss_v, gn), config, blockchain_store,
                            commit_plan)

    def _finish(self, adam: optim.Optimizer, st: _BatchState, config: TrainingConfig, blockchain_store,
                commit_plan: CommitPlan) -> Result[TrainingResult, TrainerError]:
        opt = self._adam_snapshot(adam)
        if isinstance(opt, Failure):
            return opt
        self._optimizer_state = opt.value
        self._global_step = st.global_step
        self._sobol_skip = st.sobol_skip
        do_commit, template = self._should_commit_final(blockchain_store, commit_plan)
        if do_commit:
            self._commit_to_blockchain(blockchain_store, adam, template, st.loss, batch=config.num_batches)
        snap = self.snapshot()
        if isinstance(snap, Failure):
            return snap
        return Success(TrainingResult(updated_config=snap.value, final_loss=st.loss, total_batches=config.num_batches,
                                      final_grad_norm=st.grad_norm))

    async def train_via_effects(self, config: TrainingConfig, *, logger: StepLogger | None = None,
                                blockchain_store=None, commit_plan: CommitPlan = NoCommit()
                                ) -> Result[TrainingResult, TrainerError]:
        return self.train(config, logger=logger, blockchain_store=blockchain_store, commit_plan=commit_plan)

    def _commit_to_blockchain(self, store, adam: optim.Optimizer, template: str, loss: float, batch: int) -> None:
        """Synchronous commit of the current snapshot; failures are logged, training continues."""
        import logging

        log = logging.getLogger(LOGGER_NAME)
        try:
            opt = self._adam_snapshot(adam)
            if isinstance(opt, Failure):
                log.error("Skipping commit at step %s: %s", self._global_step, opt.error)
                return
            self._optimizer_state = opt.value
            snap = self.snapshot()
            if isinstance(snap, Failure):
                log.error("Skipping commit at step %s: %s", self._global_step, snap.error)
                return
            message = template.format(step=self._global_step, loss=loss, batch=batch)
            from .storage import commit_snapshot

            try:
                asyncio.get_running_loop()
                log.warning("Skipping commit at step %s: called from a running event loop", self._global_step)
                return
            except RuntimeError:
                pass
            asyncio.run(commit_snapshot(store, snap.value, message))
        except Exception as exc:  # storage failures never stop training (reference 1296-1302)
            log.error("Failed to commit at step %s: %s", self._global_step, exc)

    # ------------------------------------------------------------------ inference
    def predict_price(self, inputs: Sequence[BlackScholes.Inputs]
                      ) -> Result[list[BlackScholes.HostPricingResults], TrainerError]:
        """CVNN spectrum -> mean of the IFFT = DC/N -> put; call by put-call parity
        (reference gbm_trainer.py:1709-1767)."""
        if len(inputs) == 0:
            return Success([])
        self._cvnn.eval()
        try:
            real_in, imag_in = _split_inputs(inputs, dtype=self._dtype.to_torch(), device=self._torch_device)
            with torch.no_grad():
                pred_r, pred_i = self._cvnn(real_in, imag_in)
                spectrum = torch.complex(pred_r, pred_i)
                coeffs = torch.fft.ifft(spectrum, dim=1).mean(dim=1).cpu()
            out: list[BlackScholes.HostPricingResults] = []
            for coeff, c in zip(coeffs, inputs, strict=True):
                re, im = float(coeff.real), float(coeff.imag)
                if abs(im) > 1.0e-6:
                    warnings.warn(f"IFFT imaginary component {im:.3e} exceeds tolerance.", RuntimeWarning)
                disc = math.exp(-c.r * c.T)
                fwd = c.X0 * math.exp((c.r - c.d) * c.T)
                put = re
                call = put + fwd - c.K * disc
                put_i = disc * max(c.K - fwd, 0.0)
                call_i = disc * max(fwd - c.K, 0.0)
                res = validate_model(BlackScholes.HostPricingResults, underlying=fwd, put_price=put, call_price=call,
                                     put_price_intrinsic=put_i, call_price_intrinsic=call_i,
                                     put_convexity=put - put_i, call_convexity=call - call_i)
                if isinstance(res, Failure):
                    raise AssertionError(f"HostPricingResults validation failed: {res.error}")
                out.append(res.value)
            return Success(out)
        except Exception as exc:
            return Failure(PredictionFailed(message=str(exc)))


class TrainingSession:
    """A live training run on the device: ``step()`` enqueues one full training step
    (eager for the first ``warmup_steps``, then one captured hipGraph replay); ``close()``
    synchronises once and returns the final counters / metrics."""

    def __init__(self, pricer: GbmCVNNPricer, config: TrainingConfig, sampler: SobolSampler,
                 adam: optim.Optimizer, ctx) -> None:
        self.pricer = pricer
        self.config = config
        self.sampler = sampler
        self.adam = adam
        self.ctx = ctx
        world, rank = (ctx.world_size, ctx.rank) if ctx is not None else (1, 0)
        self.global_batch = config.batch_size * world
        pricer._cvnn.train()
        dev = pricer._torch_device
        factory = getattr(pricer, "mc_engine_factory", None)  # e.g. basket.use_basket_engine
        if factory is not None:
            self.engine = factory(pricer, config.batch_size, dev, rank, world)
        else:
            lanes = pricer.mc_lanes if pricer.overlap_mc else 1
            sp = pricer._cfg.sim_params
            widest_in = max((m.in_features for m in pricer._cvnn.modules() if isinstance(m, ComplexLinear)), default=0)
            path_steps = config.batch_size * sp.total_paths() * sp.timesteps
            if (lanes > 1 and pricer.fused_network and 0 < widest_in < 128
                    and path_steps >= pricer.mc_lanes_long_path_steps):
                lanes = pricer.mc_lanes_long
            if lanes > 1 and path_steps < pricer.network_cu_min_path_steps:
                lanes = pricer.mc_lanes_short
            self.engine = TrainingEngine(pricer._cfg, sampler, config.batch_size, model_dtype=pricer._dtype.to_torch(),
                                         device=dev, rank=rank, world_size=world, store_paths=pricer.store_paths,
                                         math=pricer.math_mode, lanes=lanes)
        self.params = list(pricer._cvnn.parameters())
        self.program = _StepProgram(pricer, self.engine, adam, self.params, ctx)
        self.sobol_skip0 = pricer._sobol_skip
        self.sobol_skip = pricer._sobol_skip
        self.global_step = pricer._global_step
        self.steps = 0
        self.engine.set_position(self.sobol_skip, pricer._mc_engine.ordinal)
        cur = torch.cuda.current_stream(dev)
        self._hip_streams: list[int] = []  # CU-masked streams this session created (destroyed at close)
        self.network_cus_used = 0  # CUs of the network's CU-masked stream (0: no masks)
        # rows_kernel (f64, the f32 shapes no resident launch takes) is persistent.  At round 3's 8 waves
        # per SIMD it left no registers for a concurrent network part, which only stretched it (C2 in f64:
        # 10.55 ms/step overlapped, 10.35 sequential); at the f64 register budget (two workgroups per CU,
        # 4 waves per SIMD) a network workgroup fits beside it and the latency-bound f64 network hides
        # under the VALU-bound path launch (round 4: 8.64-8.71 against 8.81-8.89 ms/step,
        # profiles/r04/ab_f64_overlap_rows.txt).  Round 6: for f64 a box-dependent wash (+-1.5 %); for the
        # reference typing's rows_ref_kernel one stream is 4-6 % faster (pricer.overlap_rows = None).
        kname = getattr(self.engine, "kernel_name", "")
        rows_overlap = pricer.overlap_rows if pricer.overlap_rows is not None else not kname.startswith("rows_ref")
        overlap = pricer.overlap_mc and (rows_overlap or not kname.startswith("rows_"))
        if overlap:
            # the network part is a few short launches: a high-priority queue lets its workgroups
            # take CU slots as the long MC kernel frees them instead of queueing behind it
            hi = pricer.high_priority_stream
            lanes = getattr(self.engine, "lanes", 1)
            fused = self.program.fused
            narrow = fused is not None and max(t.in_features for t in fused.table) < 128
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            net_cus = pricer.network_cus if narrow else (pricer.network_cus_wide if fused is not None else 0)
            eng = self.engine
            path_steps = min(getattr(eng, "chunk", 0), getattr(eng, "B", 0)) * getattr(eng, "P", 0) * \
                getattr(eng, "T", 0)
            if path_steps < pricer.network_cu_min_path_steps and fused is not None:
                # (a torch-module network keeps the whole chip: network_cus_small was measured with the fused
                # network only, profiles/r04/e2e_network_cus.txt)
                net_cus = pricer.network_cus_small
            # data-parallel runs of the exchanging launches (C3 sliced, C5 basket) take the masks too: the step's
            # all-reduce runs on the network stream (dp.RcclComm), so RCCL's kernels stay on the network's CUs and
            # cannot keep a partner workgroup of the exchanging launch off a CU while they wait for a slow peer
            want = pricer.exchanging_masks if pricer.exchanging_masks is not None else (
                ctx is not None or getattr(eng, "kernel_name", "") == "resident_kernel(sliced)")
            exchanging_dp = want and getattr(eng, "exchanges", False) and fused is not None
            if (net_cus > 0 and (getattr(eng, "kernel_name", "") in WHOLE_CONTRACT_KERNELS or exchanging_dp)
                    and cus >= 2 * net_cus):
                # the network on its own CUs beside the path kernels (CU-masked HIP streams); the path
                # kernel sizes its persistent grid to its stream's CUs (gbm.hip resident_grid).  Only for
                # the whole-contract resident launch (C2, the lock-step shape) and a fused network: a
                # narrow one (fb_kernel path, ~70 us of whole-chip work at C2) on network_cus, a wide one
                # (C2/H=256: 0.26 ms) on network_cus_wide (on 32 CUs it outlasted the path kernel: 3.39
                # vs 3.30 ms/step)
                self.network_cus_used = net_cus
                net_mask, mc_mask = _cu_masks(dev, net_cus, pricer.network_cu_pattern)
                self.stream = _masked_stream(dev, net_mask, self._hip_streams)
                self.mc_streams = [_masked_stream(dev, mc_mask, self._hip_streams) for _ in range(lanes)]
            else:
                self.stream = torch.cuda.Stream(device=dev, priority=-1 if hi == "network" else 0)
                # one MC stream per engine lane: step s + 1's path launch may start on the CUs step s's
                # launch frees in its tail (TrainingEngine lanes)
                self.mc_streams = [torch.cuda.Stream(device=dev, priority=-1 if hi == "mc" else 0)
                                   for _ in range(lanes)]
        else:
            self.stream = torch.cuda.Stream(device=dev)
            self.mc_streams = [self.stream]
        self.mc_stream = self.mc_streams[0]
        self.stream.wait_stream(cur)
        for ms in self.mc_streams:
            ms.wait_stream(cur)
        K = _StepProgram.SLOTS
        self._mc_done = [torch.cuda.Event() for _ in range(K)]  # step slot k written by the MC part
        self._nn_done = [torch.cuda.Event() for _ in range(K)]  # network finished reading slot k
        self._slot_used = [False] * K
        self._mc_pending = False             # the MC part of the next step is already enqueued
        eng = self.engine
        self.capture_graphs = (getattr(eng, "B", 0) * getattr(eng, "P", 0) * getattr(eng, "T", 0) >=
                               pricer.graph_min_path_steps)
        self.mc_events: list[tuple[torch.cuda.Event, torch.cuda.Event]] | None = None
        #: timing-event pairs the live MC timing takes before creating new ones (created and recorded once
        #: beforehand, so a timed loop pays no event creation)
        self.mc_event_pool: list[tuple[torch.cuda.Event, torch.cuda.Event]] = []
        self._closed = False
        # exchanging path launches wait for the previous step's network part only on request
        # (pricer.exchange_after_network; data-parallel runs keep the collective on masked CUs instead)
        self._mc_after_nn = bool(getattr(self.engine, "exchanges", False) and pricer.exchange_after_network)
        # a session that is never closed still destroys its masked streams (after a device sync: the
        # streams may hold queued work when the session is collected)
        self._finalizer = weakref.finalize(self, _finalize_streams, self._hip_streams, dev)

    def step(self, prefetch_next: bool = True) -> Result[int, TrainerError]:
        """Enqueue one training step.  With ``prefetch_next`` (and ``pricer.overlap_mc``) the MC
        part of the following step is enqueued on the MC stream right behind this step's
        hand-off, so it runs concurrently with this step's network part.  Bit-identical to the
        sequential order: the MC part reads only the device cursor, the network part only its
        own buffers."""
        if self.sobol_skip + self.global_batch > MAX_POINTS:
            return Failure(SamplerInitFailed(error=SequenceExhausted(requested_end=self.sobol_skip + self.global_batch)))
        prog = self.program
        warm = self.pricer.warmup_steps
        if warm > 0 and self.steps >= warm and not prog.captured and self.capture_graphs:
            if self._mc_pending:  # the pending eager MC launch must finish before capture
                for ms in self.mc_streams:
                    ms.synchronize()
            prog.capture(self.mc_stream, self.stream)
        K = _StepProgram.SLOTS
        slot = self.steps % K
        if self.stream is self.mc_stream and self.ctx is None:
            with torch.cuda.stream(self.stream):  # sequential: one stream, one graph per step
                prog.run_step(slot)
            self.steps += 1
            self.sobol_skip += self.global_batch
            self.global_step += 1
            self.pricer._mc_engine.advance(self.global_batch)
            return Success(self.global_step)
        if prog.explicit_streams:
            return self._step_explicit(slot, prefetch_next)
        ms = self._lane_stream(slot)
        with torch.cuda.stream(ms):
            if not self._mc_pending:
                self._enqueue_mc(slot)
            prog.handoff(slot)
            self._mc_done[slot].record(ms)
            self._mc_pending = False
        prefetch = prefetch_next and self.sobol_skip + 2 * self.global_batch <= MAX_POINTS
        nxt = (self.steps + 1) % K
        if prefetch and not self._mc_after_nn:
            with torch.cuda.stream(self._lane_stream(nxt)):
                self._enqueue_mc(nxt)
            self._mc_pending = True
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(self._mc_done[slot])
            prog.run_nn(slot)
            self._nn_done[slot].record(self.stream)
            self._slot_used[slot] = True
        if prefetch and self._mc_after_nn:
            # an exchanging launch never shares the chip with this step's all-reduce
            ns = self._lane_stream(nxt)
            with torch.cuda.stream(ns):
                ns.wait_event(self._nn_done[slot])
                self._enqueue_mc(nxt)
            self._mc_pending = True
        self.steps += 1
        self.sobol_skip += self.global_batch
        self.global_step += 1
        self.pricer._mc_engine.advance(self.global_batch)
        return Success(self.global_step)

    def _step_explicit(self, slot: int, prefetch_next: bool) -> Result[int, TrainerError]:
        """step() for an eager step of fused HIP launches only: the same launches and events in the same
        order, on explicit stream handles instead of inside torch stream contexts (e2e: 0.078 ms of host
        time per step, the bound of that shape, before; profiles/r05/)."""
        K = _StepProgram.SLOTS
        ms = self._lane_stream(slot)
        if not self._mc_pending:
            self._enqueue_mc(slot, explicit=True)
        self._mc_done[slot].record(ms)
        self._mc_pending = False
        prefetch = prefetch_next and self.sobol_skip + 2 * self.global_batch <= MAX_POINTS
        nxt = (self.steps + 1) % K
        if prefetch and not self._mc_after_nn:
            self._enqueue_mc(nxt, explicit=True)
            self._mc_pending = True
        self.stream.wait_event(self._mc_done[slot])
        self.program.run_nn(slot, self.stream.cuda_stream)
        self._nn_done[slot].record(self.stream)
        self._slot_used[slot] = True
        if prefetch and self._mc_after_nn:
            ns = self._lane_stream(nxt)
            ns.wait_event(self._nn_done[slot])
            self._enqueue_mc(nxt, explicit=True)
            self._mc_pending = True
        self.steps += 1
        self.sobol_skip += self.global_batch
        self.global_step += 1
        self.pricer._mc_engine.advance(self.global_batch)
        return Success(self.global_step)

    def _lane_stream(self, slot: int) -> torch.cuda.Stream:
        """The MC stream of step slot ``slot`` (slot k runs on engine lane k % lanes)."""
        return self.mc_streams[slot % len(self.mc_streams)]

    def _enqueue_mc(self, slot: int, explicit: bool = False) -> None:
        """MC part of a step into ``slot`` on its lane's MC stream, once the network part that last
        read the slot (SLOTS steps back) is done with it.  explicit: eager launches on the lane's stream
        handle (else the caller's current stream is the lane's)."""
        ms = self._lane_stream(slot)
        handle = ms.cuda_stream if explicit else None
        if self._slot_used[slot]:
            ms.wait_event(self._nn_done[slot])
        if self.mc_events is not None:  # live timing of the MC part on its own stream
            e0, e1 = (self.mc_event_pool.pop() if self.mc_event_pool else
                      (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
            e0.record(ms)
            self.program.run_mc(slot, handle)
            e1.record(ms)
            self.mc_events.append((e0, e1))
        else:
            self.program.run_mc(slot, handle)

    def sync(self) -> None:
        """Wait for the enqueued steps; raises SmcError (SMC_ERR_EXCHANGE_TIMEOUT) if an exchanging
        path launch gave up on a partner workgroup since the last check (its targets hold NaN)."""
        if self._closed:
            raise RuntimeError("session is closed")
        self.stream.synchronize()
        for ms in self.mc_streams:
            ms.synchronize()
        check = getattr(self.engine, "check_status", None)
        if check is not None:
            check(self.mc_stream)

    def read_metrics(self) -> tuple[float, float]:
        if self._closed:
            raise RuntimeError("session is closed")
        self.sync()
        return float(self.program.loss), float(self.program.grad_norm)

    def close(self) -> _BatchState:
        if self._closed:
            raise RuntimeError("session already closed")
        self._closed = True
        self.stream.synchronize()
        for ms in self.mc_streams:
            ms.synchronize()
        dev = self.pricer._torch_device
        if not self._hip_streams:  # (masked streams: synchronised above, destroyed below)
            torch.cuda.current_stream(dev).wait_stream(self.stream)
            for ms in self.mc_streams:
                torch.cuda.current_stream(dev).wait_stream(ms)
        loss, gn = (float(self.program.loss), float(self.program.grad_norm)) if self.steps else (0.0, 0.0)
        for p in self.params:  # detach the flat-buffer grad views from the parameters
            p.grad = p.grad.clone()
        self.sampler.skip(self.sobol_skip - self.sobol_skip0)
        check = getattr(self.engine, "check_status", None)
        try:
            if check is not None:  # after the bookkeeping: the session is closed either way
                check(torch.cuda.current_stream(dev))  # every stream of the session is idle by now
        finally:
            self._release_streams()
        return _BatchState(self.sobol_skip, self.global_step, loss, gn)

    def _release_streams(self) -> None:
        """Destroy the CU-masked streams and drop every reference to them (the torch wrappers)."""
        self._finalizer.detach()
        self.stream = self.mc_stream = None
        self.mc_streams = []
        _destroy_streams(self._hip_streams)


    def close_quietly(self) -> None:
        """Release the session after a failure: wait for the streams, leave the status unread."""
        if self._closed:
            return
        self._closed = True
        self.stream.synchronize()
        for ms in self.mc_streams:
            ms.synchronize()
        self._release_streams()
        for p in self.params:
            if p.grad is not None:
                p.grad = p.grad.clone()


def _cu_masks(dev: torch.device, n_net: int, pattern: str) -> tuple[list[int], list[int]]:
    """32-bit mask words (hipExtStreamCreateWithCUMask) of the network's n_net CUs and of the rest.
    Logical CU ids interleave the XCDs (ids 0..31 are 4 CUs of each of the 8 XCDs, one per shader
    engine: tools/xcc_probe.py), and the dispatcher deals a grid's workgroups round-robin over them,
    so "low" takes n_net / 32 CUs from every shader engine when n_net is a multiple of 32."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    if n_net % 32 or n_net >= cus:
        raise ValueError(f"network_cus must be a multiple of 32 below {cus} (one CU per shader engine each), "
                         f"got {n_net}")
    net = set(range(n_net)) if pattern == "low" else {(i * cus) // n_net for i in range(n_net)}
    words = (cus + 31) // 32
    nm, mm = [0] * words, [0] * words
    for c in range(cus):
        if c in net:
            nm[c // 32] |= 1 << (c % 32)
        else:
            mm[c // 32] |= 1 << (c % 32)
    return nm, mm


def _hip():
    import ctypes

    return ctypes.CDLL("libamdhip64.so")


def _masked_stream(dev: torch.device, mask: list[int], owned: list[int]) -> torch.cuda.ExternalStream:
    """A HIP stream restricted to the CUs in `mask` (hipExtStreamCreateWithCUMask), as a torch stream;
    its handle is appended to `owned` (the session destroys it at close)."""
    import ctypes

    handle = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(mask))(*mask)
    with torch.cuda.device(dev):
        if _hip().hipExtStreamCreateWithCUMask(ctypes.byref(handle), ctypes.c_uint32(len(mask)), arr) != 0:
            raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    owned.append(handle.value)
    return torch.cuda.ExternalStream(handle.value, device=dev)


def _finalize_streams(owned: list[int], dev: torch.device) -> None:
    if owned:
        torch.cuda.synchronize(dev)
        _destroy_streams(owned)


def _destroy_streams(owned: list[int]) -> None:
    import ctypes

    for h in owned:
        _hip().hipStreamDestroy(ctypes.c_void_p(h))
    owned.clear()


def _bounds_always_valid(lower: np.ndarray) -> bool:
    """x in [0,1) maps to [lower, upper): rows satisfy X0>0, K>0, T>=0, v>=0 if the lower bounds do."""
    X0, K, T, _r, _d, v = (float(x) for x in lower)
    return X0 > 0 and K > 0 and T >= 0 and v >= 0


__all__ = ("TrainingSession", "GbmCVNNPricerConfig", "StepMetrics", "TrainingResult", "GbmCVNNPricer", "TrainingConfig",
           "build_training_config", "ComplexValuedModel", "NoCommit", "FinalCommit", "IntervalCommit",
           "FinalAndIntervalCommit", "CommitPlan", "build_gbm_cvnn_pricer_config")
