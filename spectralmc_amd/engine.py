"""Device-resident Monte-Carlo side of one GbmCVNNPricer training step.

Replaces the reference's per-step host loop (gbm_trainer.py:1539-1561):

    sampler.sample(B)                      -> Sobol kernel writes contracts (B,6) f64 + CVNN input (B,6)
    [_simulate_fft(c) for c in contracts]  -> ONE fused launch (per chunk): paths, normalisation,
                                              put payoff, M-mean and the N-point DFT -> targets (B,N)
    cp.asarray + torch.from_dlpack         -> targets are written in place into a torch tensor
    _split_inputs (host list -> H2D)       -> already on the device

Everything is enqueued on the caller's (current) HIP stream with no host synchronisation.
The Sobol index and the normal-stream ordinal of the batch are read by the kernels from a
small device cursor that the step itself advances, so one recorded step can be replayed as
a hipGraph indefinitely (see GbmCVNNPricer.train).

Data-parallel layout (one process per GPU): rank r of W draws global contracts
[base + r*B, base + (r+1)*B) of the step's W*B, for both the Sobol index and the normal
ordinal, and the cursor advances by W*B per step — so W ranks with B contracts each see the
same contracts and normals as one rank with W*B.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import _lib
from .gbm import BlackScholesConfig, dtype_code, normalization_code, scheme_code
from .models.numerical import Precision
from .sobol_sampler import SobolSampler, draw_device

# path scratch budget (SMC_PATH_BUFFER_GB overrides): by default half of the device's HBM (144 GB of
# an MI355X's 288 GB).  C2 needs 17.4 GB (one launch); C3's 275 GB of paths per step run as 2 launches
# of 8192 contracts instead of 8 of 2048 (each launch ends in a tail of unevenly finishing workgroup
# groups: 47.1 vs 51.9 ms/step measured)
DEFAULT_PATH_BUFFER_BYTES: int | None = (int(float(os.environ["SMC_PATH_BUFFER_GB"]) * (1 << 30))
                                         if os.environ.get("SMC_PATH_BUFFER_GB") else None)


def path_buffer_budget(device: torch.device) -> int:
    """Bytes of path scratch an engine may allocate on ``device``."""
    if DEFAULT_PATH_BUFFER_BYTES is not None:
        return DEFAULT_PATH_BUFFER_BYTES
    return torch.cuda.get_device_properties(device).total_memory // 2


# persistent launches whose workgroups never wait for each other (whole contracts per workgroup or per
# wave): MC lanes and the CU-masked network streams apply to them
WHOLE_CONTRACT_KERNELS = ("resident_kernel", "wave_kernel", "packed_kernel")


@dataclass(frozen=True)
class StepBuffers:
    contracts: torch.Tensor   # (B, 6) f64, BlackScholes.Inputs field order
    real_in: torch.Tensor     # (B, 6) CVNN dtype
    imag_in: torch.Tensor     # (B, 6) zeros
    targets: torch.Tensor     # (B, N) complex


class TrainingEngine:
    """Owns the device buffers of the Monte-Carlo step and launches its kernels."""

    def __init__(self, cfg: BlackScholesConfig, sampler: SobolSampler, batch_size: int, *, model_dtype: torch.dtype,
                 device: torch.device, rank: int = 0, world_size: int = 1, store_paths: bool = True,
                 path_buffer_bytes: int | None = None, math: str = "portable",
                 sliced: bool = False, lanes: int = 1) -> None:
        sp = cfg.sim_params
        self.cfg = cfg
        self.B = batch_size
        self.T = sp.timesteps
        self.N = sp.network_size
        self.M = sp.batches_per_mc_run
        self.P = sp.total_paths()
        self.seed = sp.mc_seed
        self.rank = rank
        self.world_size = world_size
        self.device = device
        self.sim_dtype = sp.dtype
        self._dtype_code = dtype_code(sp.dtype)
        if math not in ("portable", "hw", "reference", "reference_hw"):
            raise ValueError(f"math must be 'portable', 'hw', 'reference' or 'reference_hw', got {math!r}")
        ref = math in ("reference", "reference_hw")
        if ref and sp.dtype != Precision.float32:
            raise ValueError(f"math={math!r} is the reference kernel's f32 typing (float32 simulations only)")
        if ref and sliced:
            # rows_ref_kernel runs whole contracts per workgroup: every sliced launch would fail INVALID_SHAPE
            raise ValueError(f"math={math!r} runs whole contracts per workgroup (rows_ref_kernel); sliced=True "
                             "is not supported")
        _lib.require_device()
        self.math = math
        # "hw": f32 hardware transcendentals in the path kernel (faster, ~1 ulp, not CPU-reproducible);
        # "reference": the reference kernel's typing (f64 state and step, f32 normals and stores: rows_ref_kernel);
        # "reference_hw": the same step on the hardware-transcendental f32 normals (SMC_MATH_REF | SMC_MATH_HW)
        self._scheme = scheme_code(cfg.path_scheme) | {"hw": _lib.MATH_HW, "reference": _lib.MATH_REF,
                                                       "reference_hw": _lib.MATH_REF | _lib.MATH_HW}.get(math, 0)
        self._norm = normalization_code(cfg.normalization)
        self.store_mode = _lib.STORE_ALL if store_paths else _lib.STORE_TERMINAL
        sim_torch = sp.dtype.to_torch()
        cplx = torch.complex64 if sp.dtype == Precision.float32 else torch.complex128

        self._sampler = sampler
        self.dim = len(sampler.fields)
        lo, hi = sampler.bounds
        self.tables = torch.from_numpy(sampler.engine.tables().view("int32")).to(device)
        self.lower = torch.from_numpy(lo).to(device)
        self.upper = torch.from_numpy(hi).to(device)

        B = batch_size
        contracts = torch.empty((B, self.dim), dtype=torch.float64, device=device)
        real_in = torch.empty((B, self.dim), dtype=model_dtype, device=device)
        self.buffers = StepBuffers(contracts=contracts, real_in=real_in,
                                   imag_in=torch.zeros_like(real_in),
                                   targets=torch.empty((B, self.N), dtype=cplx, device=device))
        # scratch rows at a padded pitch: a power-of-two row stride aliases in HBM
        # (math="reference": rows_ref_kernel keeps the terminal sum in the row padding, so the pitch must leave
        # room after column P even where P is itself an odd multiple of 4 KiB)
        self.pitch = int(_lib.lib().smc_path_pitch(self.P + (4 if ref else 0), self._dtype_code))
        per_contract = (self.T * self.pitch if store_paths else self.pitch) * torch.finfo(sim_torch).bits // 8
        budget = path_buffer_bytes if path_buffer_bytes is not None else path_buffer_budget(device)
        max_chunk = max(1, min(B, budget // per_contract))
        if max_chunk < B:
            # several launches: whole rounds of resident contract workgroups (2 per CU)
            slots = 2 * torch.cuda.get_device_properties(device).multi_processor_count
            if max_chunk >= slots:
                max_chunk -= max_chunk % slots
        launches = -(-B // max_chunk)
        self.chunk = -(-B // launches)  # equal launches: no small trailing launch
        # sliced=True: each contract runs as several workgroups (slice row sums + arrival counters
        # in a workspace); the default one-workgroup-per-contract launch takes the
        # contract_kernel
        ws = int(_lib.lib().smc_engine_workspace_bytes(self.chunk, self.T, self.P, 0)) if sliced else 0
        self._workspace = torch.zeros(max(ws, 8), dtype=torch.uint8, device=device) if ws else None
        self._workspace_bytes = ws
        self._f32_in = model_dtype == torch.float32
        # smc_train_step's sync area (arrival counters; the sliced resident kernel's exchanged sums),
        # zero-filled once; every step leaves its counters zeroed
        self._uses_train_step = self._f32_in and self.dim == 6 and self._workspace is None
        # the path/CF kernel the step runs for this shape (bench labels, rocprof cross-check)
        query = self._dtype_code | (_lib.QUERY_RAW if self._norm == _lib.NORM_RAW else 0) | \
            (_lib.MATH_REF if ref else 0)
        if self._uses_train_step:
            self.kernel_name = _lib.lib().smc_train_step_kernel(self.T, self.N, self.M, query, self.pitch).decode()
        else:
            self.kernel_name = _lib.lib().smc_train_targets_kernel(
                self.T, self.N, self.P, query, self.pitch, 1 if ws else 0).decode()
        # MC lanes: consecutive steps alternate over `lanes` sets of {cursor, sync area, path scratch}, so
        # a caller may run step s + 1's launch on another stream while step s's is still in its tail
        # (the next launch's workgroups take the CUs the last contracts free).
        # Lane k's cursor is the position of the next step that uses lane k; each launch advances it by
        # lanes * global_batch.  Only for one whole-contract resident launch per step (no exchange
        # between workgroups, which needs every workgroup of a group co-resident) within the budget.
        self.lanes = 1
        if (lanes > 1 and self._uses_train_step and self.kernel_name in WHOLE_CONTRACT_KERNELS and self.chunk >= B
                and lanes * per_contract * self.chunk <= budget):
            self.lanes = lanes
        self._next_lane = 0
        # per lane: [global Sobol index of the lane's next step's first contract, its global normal ordinal]
        self.cursors = torch.zeros((self.lanes, 2), dtype=torch.int64, device=device)
        self.cursor = self.cursors[0]
        shape = (self.chunk, self.T, self.pitch) if store_paths else (self.chunk, self.pitch)
        self._paths_bufs = [torch.empty(shape, dtype=sim_torch, device=device) for _ in range(self.lanes)]
        self._paths_buf = self._paths_bufs[0]
        self.paths = self._paths_buf[..., :self.P]  # (chunk, T, P) / (chunk, P) strided view (lane 0)
        self._syncs: list[torch.Tensor | None] = [None] * self.lanes
        self._sync_bytes = 0
        if self._uses_train_step:
            sync = int(_lib.lib().smc_train_step_sync_bytes(self.T, self.N, self.M, self._dtype_code, self.pitch))
            if sync < 0:
                raise RuntimeError("smc_train_step_sync_bytes: device query failed")
            self._syncs = [torch.zeros(max(sync, 8), dtype=torch.uint8, device=device) for _ in range(self.lanes)]
            self._sync_bytes = sync
        self._sync = self._syncs[0]

    @property
    def exchanges(self) -> bool:
        """The step's path launch has workgroups that wait for each other (sliced resident kernel)."""
        return self.kernel_name == "resident_kernel(sliced)"

    def check_status(self, stream: torch.cuda.Stream | None = None) -> None:
        """Raise SmcError(SMC_ERR_EXCHANGE_TIMEOUT) if a launch since the last check gave up waiting
        for a partner workgroup (its targets hold NaN); clears the sticky status word.  Waits for
        ``stream`` (default: the current stream)."""
        for sync in self._syncs:
            check_sync_status(sync, stream)

    @property
    def global_batch(self) -> int:
        return self.B * self.world_size

    def set_position(self, sobol_index: int, ordinal: int) -> None:
        """Host -> device cursors (outside any captured region): the next step runs on lane 0 at
        (sobol_index, ordinal), lane k's next step k global batches later."""
        gb = self.global_batch
        self.cursors.copy_(torch.tensor([[sobol_index + k * gb, ordinal + k * gb] for k in range(self.lanes)],
                                        dtype=torch.int64), non_blocking=False)
        self._next_lane = 0

    def make_slot(self) -> StepBuffers:
        """Another set of step outputs (contracts, CVNN input, targets) the step can write into
        directly; the training session rotates through a few so the network part of step s reads
        its own slot while steps s+1, s+2 are produced (no hand-off copy)."""
        b = self.buffers
        return StepBuffers(contracts=torch.empty_like(b.contracts), real_in=torch.empty_like(b.real_in),
                           imag_in=b.imag_in, targets=torch.empty_like(b.targets))

    def enqueue_step(self, out: StepBuffers | None = None, lane: int | None = None,
                     stream: int | None = None) -> StepBuffers:
        """Launch contracts + targets of the next step on the current stream (or the hipStream_t ``stream``)
        into ``out`` (default: the engine's own buffers), advance the cursor.  ``lane``: the lane of this step
        (default: the next in turn); steps must use the lanes in turn, 0, 1, ..., so a lane's cursor stays the
        position of its next step."""
        stream = stream if stream is not None else _lib.stream_handle()
        b = out if out is not None else self.buffers
        offset = self.rank * self.B
        k = self._next_lane if lane is None else lane % self.lanes
        self._next_lane = (k + 1) % self.lanes
        if self._uses_train_step:
            # draw + targets + cursor advance: one launch per chunk where the resident kernel takes the shape
            _lib.check(_lib.lib().smc_train_step(
                _lib.ptr(self.tables), self.dim, _lib.ptr(self.lower), _lib.ptr(self.upper),
                _lib.ptr(self.cursors[k]), offset, self.lanes * self.global_batch, _lib.ptr(b.contracts),
                _lib.ptr(b.real_in), self.B, self.T, self.N, self.M, self.seed,
                # lanes: a launch may start while the previous one holds CUs, so no static contract share
                self._scheme | (_lib.TRAIN_DYNAMIC if self.lanes > 1 else 0), self._norm,
                self._dtype_code, self.store_mode, _lib.ptr(self._paths_bufs[k]), self.pitch, self.chunk,
                _lib.ptr(b.targets), _lib.ptr(self._syncs[k]), self._sync_bytes, stream))
            return b
        draw_device(self.tables, self.dim, self.cursor[0:1], offset, self.B, self.lower, self.upper, b.contracts,
                    b.real_in if self._f32_in else None)
        if not self._f32_in:
            b.real_in.copy_(b.contracts)
        self.launch_targets(stream, _lib.ptr(self.cursor[1:2]), offset, b)
        self.cursor.add_(self.global_batch)
        return b

    def launch_targets(self, stream: int | None, ordinal_ptr: int | None, ordinal0: int,
                       b: StepBuffers | None = None) -> None:
        """The fused path/CF kernel(s) for the contracts in ``b`` (training needs only the
        terminal row sum, so no rowsum buffer)."""
        b = b if b is not None else self.buffers
        _lib.check(_lib.lib().smc_train_targets(
            _lib.ptr(b.contracts), self.B, self.T, self.N, self.M, self.seed, ordinal_ptr, ordinal0,
            self._scheme, self._norm, self._dtype_code, self.store_mode, _lib.ptr(self._paths_buf), self.pitch,
            self.chunk, None, _lib.ptr(b.targets), _lib.ptr(self._workspace), self._workspace_bytes, stream))


def check_sync_status(sync: torch.Tensor | None, stream: torch.cuda.Stream | None = None) -> None:
    """The sync area's status word (include/spectralmc_hip.h, smc_sync_status) as an exception."""
    if sync is None:
        return
    status = _lib.sync_status(sync, clear=True, stream=stream)
    if status & _lib.SYNC_EXCHANGE_TIMEOUT:
        raise _lib.SmcError(_lib.SMC_ERR_EXCHANGE_TIMEOUT,
                            "a workgroup exchange timed out: a partner workgroup never arrived, so the step's "
                            "targets hold NaN (were all workgroups of a group co-resident?)")


__all__ = ["TrainingEngine", "StepBuffers", "DEFAULT_PATH_BUFFER_BYTES", "WHOLE_CONTRACT_KERNELS", "check_sync_status",
           "path_buffer_budget"]
