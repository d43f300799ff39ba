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

Nothing from the reference is copied into the repository: only the numbers it produced.
"""

from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz")


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

    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
