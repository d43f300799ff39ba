"""Generate the golden vectors in tests/golden/golden.npz FROM THE REFERENCE CODE.

Run in the build container (where the read-only reference checkout exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference/src

What is taken from the reference, and how:
* Sobol contracts: the reference's own ``SobolSampler`` / ``build_domain_bounds`` /
  ``build_bound_spec`` / ``build_sobol_config`` (src/spectralmc/sobol_sampler.py), imported
  unmodified (it needs only scipy + pydantic, both installed).  The point model is a local
  Pydantic class with BlackScholes.Inputs' fields and constraints (gbm.py:267-277), because
  gbm.py itself imports CuPy/Numba, which this image lacks.
* CVNN: the reference's own layer classes (src/spectralmc/cvnn.py), imported unmodified except
  that ``spectralmc.runtime`` (the reference's CUDA-presence guard, runtime/torch_runtime.py:83-97)
  is replaced by a module whose ``get_torch_handle`` returns torch — no arithmetic is touched.
  ``cvnn_factory.build_model`` cannot be imported (its models.numerical imports CuPy), so its
  construction order (cvnn_factory.py:343-367: fork_rng, manual_seed(seed), layers in config
  order, output projection last, default dtype = config dtype, CPU) is restated here.
* Training step: ``_torch_step`` (gbm_trainer.py:819-835) restated on the reference modules
  (gbm_trainer.py itself needs aioboto3 / CUDA streams).

* GBM / CF targets (``gbm_golden.npz``): the reference's own ``spectralmc.gbm`` (BlackScholes
  engine, ``SimulateBlackScholes`` kernel body, normalisation, payoff; gbm.py:224-257,400-488)
  and ``async_normals`` pool, imported behind the CPU shims of ``ref_shim.py`` (cupy -> numpy,
  numba.cuda.jit -> serial grid emulator with Numba's f64-compute / dtype-store typing), fed
  with the BUILD's normal matrices through the shimmed ``default_rng(...).standard_normal``.
  ``_simulate_fft`` (gbm_trainer.py:814-817) is restated as its one line on the engine output.
  One full C1 training step pair comes from the reference ``cvnn_factory.build_model`` (now
  importable through the same shims) + ``_torch_step`` restated (gbm_trainer.py:819-835).

Nothing from the reference is copied into the repository: only the numbers it produced.
"""

from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REF = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "golden.npz")
OUT_GBM = os.path.join(HERE, "gbm_golden.npz")

# (name, timesteps, network_size, batches, dtype, scheme, normalization, mc_seed, ordinal0, contract rows)
# contract rows: a slice of the reference-sampler Sobol points (seed 7, skip 0) or explicit rows.
EDGE_ROWS = np.array([
    [100.0, 100.0, 0.0, 0.05, 0.01, 0.4],     # T = 0 maturity: every path stays X0
    [100.0, 110.0, 1.5, 0.03, 0.01, 0.0],     # v = 0: deterministic forward
    [100.0, 0.001, 2.0, 0.02, 0.00, 0.3],     # deep OTM put: all-zero targets
    [10.0, 20_000.0, 3.0, -0.1, 0.05, 1.5],   # deep ITM, high vol
    [0.001, 0.002, 10.0, 0.2, -0.2, 2.0],     # domain corner
])
GBM_CASES = (
    ("e2e", 16, 128, 4, "float32", "log_euler", "normalize", 7, 0, slice(0, 16)),
    ("c1", 16, 256, 4, "float32", "log_euler", "normalize", 7, 0, slice(0, 64)),
    ("raw", 16, 64, 4, "float32", "log_euler", "raw", 7, 5, slice(16, 24)),
    ("euler", 16, 64, 4, "float32", "simple_euler", "normalize", 7, 0, slice(24, 32)),
    ("f64", 16, 128, 4, "float64", "log_euler", "normalize", 7, 0, slice(0, 8)),
    ("f64euler", 5, 64, 4, "float64", "simple_euler", "raw", 31, 3, slice(8, 16)),
    ("edge", 16, 64, 4, "float32", "log_euler", "normalize", 7, 0, "edge"),
    ("edgef64", 16, 64, 4, "float64", "log_euler", "normalize", 7, 0, "edge"),
    ("t1", 1, 16, 64, "float32", "log_euler", "normalize", 9, 100, slice(32, 40)),
    ("t3", 3, 256, 4, "float32", "log_euler", "normalize", 7, 0, slice(40, 44)),
    ("n1", 4, 1, 64, "float32", "log_euler", "normalize", 7, 0, slice(44, 48)),
    ("n5", 4, 5, 16, "float32", "log_euler", "normalize", 7, 0, slice(48, 52)),
    ("n1025", 4, 1025, 2, "float32", "log_euler", "normalize", 7, 0, slice(52, 54)),
    ("c2shape", 16, 256, 256, "float32", "log_euler", "normalize", 7, 0, slice(0, 2)),
    ("c3shape", 16, 1024, 256, "float32", "log_euler", "normalize", 7, 0, slice(2, 3)),
    # resident-kernel shapes with T != 16 (rolled row loop): the reference's lock-step trainer shape
    # (tests/test_gbm_trainer.py:122-131: T = 1, N = 16, M = 4096), odd T with simple Euler, T > 16 RAW
    ("lockstep", 1, 16, 4096, "float32", "log_euler", "raw", 43, 0, slice(54, 56)),
    ("lockstepf64", 1, 16, 4096, "float64", "log_euler", "raw", 43, 0, slice(54, 56)),
    ("t5", 5, 64, 64, "float32", "simple_euler", "normalize", 11, 40, slice(56, 58)),
    ("t33", 33, 256, 16, "float32", "log_euler", "raw", 7, 2, slice(58, 60)),
)


from bn_archs import BN_ARCHS  # noqa: E402  (the same builders construct this build's modules in the tests)


def main() -> None:
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    guard = types.ModuleType("spectralmc.runtime")
    guard.get_torch_handle = lambda: torch  # CUDA-presence guard only
    sys.modules["spectralmc.runtime"] = guard

    from pydantic import BaseModel, ConfigDict, Field
    from typing import Annotated

    from spectralmc import cvnn as ref_cvnn
    from spectralmc.result import Success
    from spectralmc.sobol_sampler import SobolSampler, build_bound_spec, build_domain_bounds, build_sobol_config

    PosFloat = Annotated[float, Field(gt=0)]
    NonNegFloat = Annotated[float, Field(ge=0)]

    class Inputs(BaseModel):
        X0: PosFloat
        K: PosFloat
        T: NonNegFloat
        r: float
        d: float
        v: NonNegFloat
        model_config = ConfigDict(frozen=True, extra="forbid")

    fields = ("X0", "K", "T", "r", "d", "v")
    # tests/helpers/factories.py:108-161 defaults
    default_bounds = {"X0": (0.001, 10_000.0), "K": (0.001, 20_000.0), "T": (0.0, 10.0), "r": (-0.20, 0.20),
                      "d": (-0.20, 0.20), "v": (0.0, 2.0)}
    out: dict[str, np.ndarray] = {}
    out["bounds_lower"] = np.array([default_bounds[f][0] for f in fields])
    out["bounds_upper"] = np.array([default_bounds[f][1] for f in fields])
    bounds = build_domain_bounds(Inputs, {f: build_bound_spec(*default_bounds[f]).unwrap() for f in fields}).unwrap()

    for seed in (7, 31, 42, 123):
        for skip in (0, 8, 4096):
            sampler = SobolSampler.create(Inputs, bounds, config=build_sobol_config(seed=seed, skip=skip).unwrap())
            assert isinstance(sampler, Success)
            pts = sampler.value.sample(64)
            assert isinstance(pts, Success)
            out[f"sobol_s{seed}_k{skip}"] = np.array([[getattr(p, f) for f in fields] for p in pts.value])
            # a second draw continues the sequence (skip + 64 ...)
            pts2 = sampler.value.sample(32)
            out[f"sobol_s{seed}_k{skip}_next"] = np.array([[getattr(p, f) for f in fields] for p in pts2.value])

    def build(seed: int, widths: list[int], n_out: int, dtype: torch.dtype) -> torch.nn.Module:
        """cvnn_factory.build_model for [Linear(w, modReLU)...] + output projection."""
        with torch.random.fork_rng():
            saved = torch.get_default_dtype()
            torch.set_default_dtype(dtype)
            try:
                torch.manual_seed(seed)
                mods = []
                w = 6
                for hw in widths:
                    mods.append(ref_cvnn.ComplexSequential(ref_cvnn.ComplexLinear(w, hw), ref_cvnn.modReLU(hw)))
                    w = hw
                body = mods[0] if len(mods) == 1 else ref_cvnn.ComplexSequential(*mods)
                net = ref_cvnn.ComplexSequential(body, ref_cvnn.ComplexLinear(w, n_out)) if w != n_out else body
            finally:
                torch.set_default_dtype(saved)
        return net

    contracts = out["sobol_s7_k0"]
    rng = np.random.default_rng(2024)
    for name, seed, widths, n_out, dtype in (("e2e", 123, [32], 128, torch.float32),
                                             ("c1", 123, [32], 256, torch.float32),
                                             ("c2", 123, [32, 32], 256, torch.float32),
                                             ("c2f64", 123, [32, 32], 256, torch.float64),
                                             ("tmpl", 999, [32], 128, torch.float32)):
        net = build(seed, widths, n_out, dtype)
        for k, v in net.state_dict().items():
            out[f"cvnn_{name}__{k}"] = v.detach().numpy().copy()
        x_re = torch.tensor(contracts, dtype=dtype)
        x_im = torch.zeros_like(x_re)
        with torch.no_grad():
            yr, yi = net(x_re, x_im)
        out[f"cvnn_{name}_fwd_re"] = yr.numpy()
        out[f"cvnn_{name}_fwd_im"] = yi.numpy()
        # one _torch_step against fixed complex targets of the same magnitude as CF targets
        tgt = (rng.normal(size=(contracts.shape[0], n_out)) + 1j * rng.normal(size=(contracts.shape[0], n_out))) * 1e3
        out[f"cvnn_{name}_step_targets"] = tgt.astype(np.complex128 if dtype == torch.float64 else np.complex64)
        targets = torch.tensor(out[f"cvnn_{name}_step_targets"])
        adam = torch.optim.Adam(net.parameters(), lr=1e-2)
        pr, pi = net(x_re, x_im)
        loss = torch.nn.functional.mse_loss(pr, torch.real(targets)) + torch.nn.functional.mse_loss(
            pi, torch.imag(targets))
        adam.zero_grad(set_to_none=True)
        loss.backward()
        adam.step()
        gn = float(torch.nn.utils.clip_grad_norm_(net.parameters(), float("inf")))
        out[f"cvnn_{name}_step_loss"] = np.array(float(loss.item()))
        out[f"cvnn_{name}_step_gradnorm"] = np.array(gn)
        for k, v in net.state_dict().items():
            out[f"cvnn_{name}_after__{k}"] = v.detach().numpy().copy()

    # batch-norm / residual architectures (cvnn.py:213-480): train-mode forward, one _torch_step
    # (batch statistics, running-stat updates, Adam) and the eval-mode forward after it
    for name, make in BN_ARCHS.items():
        with torch.random.fork_rng():
            torch.manual_seed(321)
            net = make(ref_cvnn)
        for k, v in net.state_dict().items():
            out[f"bn_{name}__{k}"] = v.detach().numpy().copy()
        x_re = torch.tensor(contracts / contracts.max(axis=0), dtype=torch.float32)
        x_im = torch.tensor(np.roll(contracts, 1, axis=1) / contracts.max(axis=0), dtype=torch.float32)
        net.train()
        with torch.no_grad():
            yr, yi = net(x_re, x_im)
        out[f"bn_{name}_fwd_re"], out[f"bn_{name}_fwd_im"] = yr.numpy(), yi.numpy()
        n_out = yr.shape[1]
        tgt = rng.normal(size=(contracts.shape[0], n_out)) + 1j * rng.normal(size=(contracts.shape[0], n_out))
        out[f"bn_{name}_step_targets"] = tgt.astype(np.complex64)
        targets = torch.tensor(out[f"bn_{name}_step_targets"])
        adam = torch.optim.Adam(net.parameters(), lr=1e-2)
        pr, pi = net(x_re, x_im)
        loss = torch.nn.functional.mse_loss(pr, torch.real(targets)) + torch.nn.functional.mse_loss(
            pi, torch.imag(targets))
        adam.zero_grad(set_to_none=True)
        loss.backward()
        adam.step()
        out[f"bn_{name}_step_loss"] = np.array(float(loss.item()))
        out[f"bn_{name}_step_gradnorm"] = np.array(float(torch.nn.utils.clip_grad_norm_(net.parameters(), float("inf"))))
        for k, v in net.state_dict().items():
            out[f"bn_{name}_after__{k}"] = v.detach().numpy().copy()
        net.eval()
        with torch.no_grad():
            er, ei = net(x_re, x_im)
        out[f"bn_{name}_eval_re"], out[f"bn_{name}_eval_im"] = er.numpy(), ei.numpy()

    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


def main_gbm() -> None:
    """CF targets and a C1 training step pair from the reference's own gbm.py (shimmed)."""
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root: oracle (normals)
    sys.path.insert(0, HERE)
    import ref_shim

    ref_shim.install(REF)
    from spectralmc import gbm
    from spectralmc.cvnn_factory import ActivationCfg, ActivationKind, ExplicitWidth, LinearCfg, build_cvnn_config
    from spectralmc.cvnn_factory import build_model
    from spectralmc.effects import ForwardNormalization, PathScheme
    from spectralmc.models.numerical import Precision
    from spectralmc.models.torch import FullPrecisionDType
    from spectralmc.sobol_sampler import SobolSampler, build_bound_spec, build_domain_bounds, build_sobol_config

    fields = ("X0", "K", "T", "r", "d", "v")
    default_bounds = {"X0": (0.001, 10_000.0), "K": (0.001, 20_000.0), "T": (0.0, 10.0), "r": (-0.20, 0.20),
                      "d": (-0.20, 0.20), "v": (0.0, 2.0)}
    bounds = build_domain_bounds(gbm.BlackScholes.Inputs,
                                 {f: build_bound_spec(*default_bounds[f]).unwrap() for f in fields}).unwrap()
    sampler = SobolSampler.create(gbm.BlackScholes.Inputs, bounds,
                                  config=build_sobol_config(seed=7, skip=0).unwrap()).unwrap()
    step_contracts = [sampler.sample(64).unwrap() for _ in range(2)]  # the trainer's first two C1 batches
    sobol_rows = np.array([[getattr(p, f) for f in fields] for p in step_contracts[0]])

    def engine(T: int, N: int, M: int, dtype: str, scheme: str, norm: str, seed: int, ordinal0: int):
        ref_shim.SOURCE.seed, ref_shim.SOURCE.next_ordinal = seed, ordinal0
        sp = gbm.build_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                         mc_seed=seed, buffer_size=1, dtype=Precision(dtype)).unwrap()
        cfg = gbm.build_black_scholes_config(sim_params=sp, path_scheme=PathScheme(scheme),
                                             normalization=ForwardNormalization.NORMALIZE if norm == "normalize" else ForwardNormalization.RAW).unwrap()
        return gbm.BlackScholes(cfg)

    def simulate_fft(eng, row: np.ndarray, N: int, M: int) -> np.ndarray:
        """GbmCVNNPricer._simulate_fft (gbm_trainer.py:806-817) on the engine's price()."""
        pricing = eng.price(inputs=gbm.BlackScholes.Inputs(**dict(zip(fields, (float(x) for x in row))))).unwrap()
        mat = pricing.put_price.reshape(M, N)
        return np.mean(np.fft.fft(mat, axis=1), axis=0)

    out: dict[str, np.ndarray] = {}
    for name, T, N, M, dtype, scheme, norm, seed, ordinal0, rows in GBM_CASES:
        t0 = time.time()
        contracts = EDGE_ROWS if isinstance(rows, str) else sobol_rows[rows]
        eng = engine(T, N, M, dtype, scheme, norm, seed, ordinal0)
        targets = np.stack([simulate_fft(eng, row, N, M) for row in contracts])
        out[f"{name}_contracts"] = contracts
        out[f"{name}_targets"] = targets
        out[f"{name}_meta"] = np.array([T, N, M, int(dtype == "float64"), int(scheme == "simple_euler"),
                                        int(norm == "normalize"), seed, ordinal0], dtype=np.int64)
        print(f"  {name}: {contracts.shape[0]} contracts, targets {targets.dtype}, {time.time() - t0:.1f} s",
              flush=True)

    # one C1 training-step pair: T=16, N=256, M=4, B=64, mc_seed 7, e2e CVNN (6 -> 32 modReLU -> 256, seed 123)
    import torch

    T, N, M = 16, 256, 4
    eng = engine(T, N, M, "float32", "log_euler", "normalize", 7, 0)
    cfg = build_cvnn_config(dtype=FullPrecisionDType.float32,
                            layers=[LinearCfg(width=ExplicitWidth(value=32),
                                              activation=ActivationCfg(kind=ActivationKind.MOD_RELU)),
                                    LinearCfg(width=ExplicitWidth(value=N))], seed=123).unwrap()
    net = build_model(n_inputs=6, n_outputs=N, cfg=cfg).unwrap()
    for k, v in net.state_dict().items():
        out[f"step_init__{k}"] = v.detach().numpy().copy()
    adam = torch.optim.Adam(net.parameters(), lr=1e-2)
    for s, batch in enumerate(step_contracts):
        rows = np.array([[getattr(p, f) for f in fields] for p in batch])
        targets = np.stack([simulate_fft(eng, row, N, M) for row in rows])
        x = torch.tensor(rows, dtype=torch.float32)
        y = torch.from_numpy(targets)
        pr, pi = net(x, torch.zeros_like(x))
        loss = torch.nn.functional.mse_loss(pr, torch.real(y)) + torch.nn.functional.mse_loss(pi, torch.imag(y))
        adam.zero_grad(set_to_none=True)
        loss.backward()
        adam.step()
        gn = float(torch.nn.utils.clip_grad_norm_(net.parameters(), float("inf")))
        out[f"step{s}_contracts"] = rows
        out[f"step{s}_targets"] = targets
        out[f"step{s}_loss"] = np.array(float(loss.item()))
        out[f"step{s}_gradnorm"] = np.array(gn)
        for k, v in net.state_dict().items():
            out[f"step{s}_after__{k}"] = v.detach().numpy().copy()
        print(f"  C1 step {s}: loss {float(loss):.6e} grad-norm {gn:.6e}", flush=True)

    np.savez_compressed(OUT_GBM, **out)
    print(f"wrote {OUT_GBM}: {len(out)} arrays, {os.path.getsize(OUT_GBM)} bytes")


if __name__ == "__main__":
    if "--gbm-only" not in sys.argv:
        main()
    if "--no-gbm" not in sys.argv:
        main_gbm()
