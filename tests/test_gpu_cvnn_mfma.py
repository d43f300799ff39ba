"""The network step on the matrix cores (csrc/cvnn_mfma.hip) against the oracle's explicit-precision
restatement (oracle/cvnn_mixed.py, itself equal to torch autograd of _torch_step in f32,
tests/test_cvnn_mixed_oracle.py):

* SMC_CVNN_MFMA_F32: loss within 1e-5 rel, gradients within 1e-5 norm-relative (f32 summation
  order is the only difference);
* SMC_CVNN_MFMA_BF16: the same bf16 roundings as the restatement; a GPU f32 accumulation that lands
  an intermediate on the other side of a bf16 rounding boundary moves that element by one bf16 ulp,
  so loss within 1e-4 rel and gradients within 2e-3 norm-relative;
* shapes: the C2 network (6 -> 32 -> 32 -> 256) and its H = 256 variant, the C3 network
  (6 -> 32 -> 32 -> 1024), zReLU and a last-layer activation, ragged batches (row padding);
* bit-identical reruns; the trainer's C3 session on the bf16 kernels.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle.cvnn_mixed import cvnn_step
from spectralmc_amd import _lib
from spectralmc_amd.cvnn import ComplexLinear, ComplexSequential, modReLU, zReLU
from spectralmc_amd.net import FusedNetworkStep
from tests.helpers import make_test_cvnn

pytestmark = pytest.mark.gpu

DEV = "cuda"


def table_of(step: FusedNetworkStep) -> list[tuple[int, ...]]:
    return [(t.in_features, t.out_features, t.activation, t.w_re, t.w_im, t.b_re, t.b_im, t.act_bias)
            for t in step.table]


def build(arch: str, n_out: int) -> torch.nn.Module:
    if arch == "zrelu":
        torch.manual_seed(5)
        return ComplexSequential(ComplexLinear(6, 24), zReLU(), ComplexLinear(24, 40), modReLU(40),
                                 ComplexLinear(40, n_out)).to(DEV)
    if arch == "lastact":
        torch.manual_seed(6)
        return ComplexSequential(ComplexLinear(6, 32), modReLU(32), ComplexLinear(32, n_out), modReLU(n_out)).to(DEV)
    if arch == "widelast":  # wide (layered GEMM path), a width that is not a multiple of the 128 tile
        torch.manual_seed(7)
        return ComplexSequential(ComplexLinear(6, 160), modReLU(160), ComplexLinear(160, n_out), modReLU(n_out)).to(DEV)
    if arch == "widez":
        torch.manual_seed(8)
        return ComplexSequential(ComplexLinear(6, 128), zReLU(), ComplexLinear(128, 144), modReLU(144),
                                 ComplexLinear(144, n_out)).to(DEV)
    width = {"h256": 256, "h128": 128}.get(arch, 32)
    return make_test_cvnn(n_inputs=6, n_outputs=n_out, seed=123, dtype=torch.float32, device=DEV,
                          hidden_layers=2, hidden_width=width)


def data(B: int, n_out: int, seed: int = 11) -> tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    # contract-like inputs (positive, up to ~1e4 on the first features) and CF-magnitude targets
    scale = torch.tensor([1e4, 2e4, 10.0, 0.2, 0.2, 2.0])
    x = torch.rand((B, 6), generator=g) * scale
    t = torch.complex(torch.randn((B, n_out), generator=g), torch.randn((B, n_out), generator=g)) * 1e3
    return x, t


def gpu_grads(model, compute: str, x: torch.Tensor, t: torch.Tensor) -> tuple[FusedNetworkStep, torch.Tensor]:
    params = list(model.parameters())
    adam = torch.optim.Adam(params, lr=1e-3)
    n = sum(p.numel() for p in params)
    flat = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
    loss = torch.zeros((), dtype=torch.float32, device=DEV)
    gn = torch.zeros((), dtype=torch.float32, device=DEV)
    step = FusedNetworkStep(model, adam, params, flat, loss, gn, x.shape[0], fuse_adam=False, compute=compute)
    xd = x.to(DEV)
    step.fwd_bwd(xd, torch.zeros_like(xd), t.to(DEV))
    torch.cuda.synchronize()
    return step, flat.cpu()


# h256 / h128 / widelast / widez take the layered GEMM launches (2 H >= 256, csrc/cvnn_mfma.hip lgemm_kernel)
CASES = [("c2", 256, 4096), ("c2", 256, 1000), ("c3", 1024, 2048), ("h256", 256, 4096), ("zrelu", 64, 21),
         ("lastact", 96, 333), ("h256", 256, 1000), ("h128", 64, 777), ("widelast", 200, 333), ("widez", 64, 500)]


@pytest.mark.parametrize("compute", ["mfma", "bf16"])
@pytest.mark.parametrize("arch,n_out,B", CASES)
def test_mfma_step_matches_oracle(compute, arch, n_out, B) -> None:
    model = build(arch, n_out)
    x, t = data(B, n_out)
    params0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    step, flat = gpu_grads(model, compute, x, t)
    assert step.kernels == ("mfma_bf16" if compute == "bf16" else "mfma_f32")
    operand = "bf16" if compute == "bf16" else "f32"
    loss, g = cvnn_step(table_of(step), params0, x.numpy(), None, t.numpy(), operand=operand)
    got = flat[:-1].double().numpy()
    rel = np.linalg.norm(got - g) / np.linalg.norm(g)
    loss_rel = abs(float(flat[-1]) - loss) / loss
    tol_g, tol_l = (2e-3, 1e-4) if compute == "bf16" else (1e-5, 1e-5)
    assert loss_rel < tol_l, (loss_rel, rel)
    assert rel < tol_g, (loss_rel, rel)
    # every parameter group is resolved, not only the largest
    off = 0
    for p in model.parameters():
        k = p.numel()
        sl = slice(off, off + k)
        gn = np.linalg.norm(g[sl])
        if gn > 1e-3 * np.linalg.norm(g):
            assert np.linalg.norm(got[sl] - g[sl]) / gn < 10 * tol_g
        off += k


@pytest.mark.parametrize("compute,arch", [("mfma", "c3"), ("bf16", "c3"), ("mfma", "h256")])
def test_mfma_step_bit_reproducible(compute, arch) -> None:
    n_out = 1024 if arch == "c3" else 256
    model = build(arch, n_out)
    x, t = data(4096, n_out, seed=3)
    _, a = gpu_grads(model, compute, x, t)
    _, b = gpu_grads(model, compute, x, t)
    assert torch.equal(a, b)


@pytest.mark.parametrize("compute,arch,n_out,B", [("mfma", "c2", 256, 1000), ("bf16", "zrelu", 64, 333),
                                                  ("mfma", "lastact", 96, 4096), ("mfma", "h128", 64, 500)])
@pytest.mark.parametrize("dp", [False, True])
def test_adam_written_packed_weights_equal_the_pack_launch(compute, arch, n_out, B, dp) -> None:
    """Adam writes the MFMA operand copies of the weights it updates (smc_cvnn_pack), so every fwd_bwd after
    the first skips pack_kernel (SMC_CVNN_MFMA_PACKED): four steps equal, bit for bit (parameters, Adam
    moments, loss, grad norm), four steps that run the pack launch every time; fused Adam and the separate
    data-parallel update alike; the layered GEMM path (h128) keeps its own pack launch."""
    runs = []
    for packed in (True, False):
        model = build(arch, n_out)
        params = list(model.parameters())
        adam = torch.optim.Adam(params, lr=1e-2)
        n = sum(p.numel() for p in params)
        flat = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
        loss = torch.zeros((), dtype=torch.float32, device=DEV)
        gn = torch.zeros((), dtype=torch.float32, device=DEV)
        step = FusedNetworkStep(model, adam, params, flat, loss, gn, B, fuse_adam=not dp, compute=compute)
        assert (step._pack is not None) == (arch != "h128")
        if not packed:
            step._pack = None
            step.adam_args.pack = None
        losses = []
        for k in range(4):
            x, t = data(B, n_out, seed=20 + k)
            xd = x.to(DEV)
            step.fwd_bwd(xd, torch.zeros_like(xd), t.to(DEV))
            if dp:
                step.adam()
            losses.append((float(loss), float(gn)))
        torch.cuda.synchronize()
        assert step._packed == (packed and arch != "h128")
        runs.append((step.params_flat.cpu(), step.exp_avg.cpu(), step.exp_avg_sq.cpu(), losses))
    (pa, ma, va, la), (pb, mb, vb, lb) = runs
    assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)
    assert la == lb


def test_auto_uses_mfma_for_f32_and_valu_for_f64() -> None:
    m32 = build("c2", 256)
    s32, _ = gpu_grads(m32, "auto", *data(64, 256))
    assert s32.kernels == "mfma_f32"
    m64 = make_test_cvnn(n_inputs=6, n_outputs=64, seed=1, dtype=torch.float64, device=DEV, hidden_layers=1)
    params = list(m64.parameters())
    n = sum(p.numel() for p in params)
    z = torch.zeros((), dtype=torch.float64, device=DEV)
    s64 = FusedNetworkStep(m64, torch.optim.Adam(params), params, torch.zeros(n + 1, dtype=torch.float64, device=DEV),
                           z, z.clone(), 16, fuse_adam=True, compute="auto")
    assert s64.kernels == "valu"


def test_c3_training_session_on_bf16_kernels(oracle) -> None:
    """One step of the C3 shape (network 6 -> 32 -> 32 -> 1024 on bf16 MFMA, N = 1024) through the trainer
    with a small batch (B = 64, M = 4): the session uses the bf16 kernels, its targets equal the oracle's
    reference-mode targets within 1e-5 per contract, and its loss and gradients equal the explicit-precision
    bf16 restatement of the network step on those targets (loss 1e-4 rel, gradients 2e-3 norm-relative);
    two more (graph-replayed) steps stay finite.  The full-size C3 session: test_gpu_c3_c5_sessions.py."""
    from spectralmc_amd.gbm_trainer import GbmCVNNPricer
    from spectralmc_amd.models.numerical import Precision
    from tests.helpers import (expect_success, make_black_scholes_config, make_domain_bounds, make_gbm_cvnn_config,
                               make_simulation_params, make_training_config)
    from tests.test_reference_fixtures import per_contract_rel

    B, T, N, M = 64, 16, 1024, 4
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                mc_seed=7, buffer_size=4, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device=DEV, hidden_layers=2)
    params0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.network_compute = "bf16"
    session = expect_success(pricer.open_session(make_training_config(num_batches=1, batch_size=B,
                                                                      learning_rate=1e-2)))
    prog = session.program
    assert prog.fused is not None and prog.fused.kernels == "mfma_bf16"
    for s in prog.slots:
        s.targets.fill_(complex("nan"))
    expect_success(session.step(prefetch_next=False))
    final = session.close()
    contracts = prog.slots[0].contracts.cpu().numpy()
    targets = prog.slots[0].targets.cpu().numpy()
    real_in = prog.slots[0].real_in.cpu().numpy()
    lo, hi = make_domain_bounds().arrays()
    np.testing.assert_array_equal(contracts, oracle.sobol_contracts(7, 0, B, lo, hi))
    want = oracle.training_targets(contracts, T, N, M, seed=7, ordinal0=0)
    assert per_contract_rel(targets, want).max() < 1e-5
    loss, g = cvnn_step(table_of(prog.fused), params0, real_in, None, targets, operand="bf16")
    got = prog.flat[:-1].double().cpu().numpy()
    assert final.loss == pytest.approx(loss, rel=1e-4)
    assert np.linalg.norm(got - g) / np.linalg.norm(g) < 2e-3
    res = expect_success(pricer.train(make_training_config(num_batches=2, batch_size=B, learning_rate=1e-2)))
    assert np.isfinite(res.final_loss)


def test_invalidate_pack_after_an_in_place_parameter_write() -> None:
    """The packed MFMA weight copies are written by Adam only: parameters written in place mid-session (here
    halved through the model's views) followed by invalidate_pack() give the step a pack launch every time
    gives, bit for bit; without invalidate_pack the next step would read the stale copies."""
    B = 1000
    runs = {}
    for mode in ("packed", "always_pack", "stale"):
        model = build("c2", 256)
        params = list(model.parameters())
        adam = torch.optim.Adam(params, lr=1e-2)
        n = sum(p.numel() for p in params)
        flat = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
        loss = torch.zeros((), dtype=torch.float32, device=DEV)
        gn = torch.zeros((), dtype=torch.float32, device=DEV)
        step = FusedNetworkStep(model, adam, params, flat, loss, gn, B, fuse_adam=True, compute="mfma")
        if mode == "always_pack":
            step._pack = None
            step.adam_args.pack = None
        for k in range(4):
            if k == 2:
                with torch.no_grad():
                    for p in params:
                        p.mul_(0.5)
                if mode != "stale":
                    step.invalidate_pack()
            x, t = data(B, 256, seed=40 + k)
            xd = x.to(DEV)
            step.fwd_bwd(xd, torch.zeros_like(xd), t.to(DEV))
        torch.cuda.synchronize()
        runs[mode] = (step.params_flat.cpu(), float(loss), float(gn))
    assert torch.equal(runs["packed"][0], runs["always_pack"][0])
    assert runs["packed"][1:] == runs["always_pack"][1:]
    assert not torch.equal(runs["stale"][0], runs["always_pack"][0])
