"""The timed C3 and C5 sessions end to end (BASELINE configs[2] and configs[4] per GPU), as
tests/test_gpu_c2_session.py does for C2: ``GbmCVNNPricer`` built and configured exactly as ``bench.py``
builds it for ``--config c3`` / ``--config c5`` (``bench.make_pricer(bench.parse(["--config", ...]))``).

* C3: 16,384 contracts x 262,144 paths (N = 1024, M = 256), T = 16, hw math, full path store: two
  8192-contract ``resident_kernel(sliced)`` launches per step (W = 4 workgroups per contract, the dynamic
  exchange tail) through half the HBM of path scratch, the 6 -> 32 -> 32 -> 1024 network on the bf16 MFMA
  kernels, per-slot hipGraphs after 2 eager steps, the next step's MC part beside the network part;
* C5: 8192 contracts x 131,072 paths (N = 256, M = 512) of 4 correlated assets, three 2731-contract
  ``basket_resident_kernel`` launches (W = 32) per step, the 16 -> 32 -> 32 -> 256 f32 MFMA network.

For each:
* three steps (the third a graph replay) bit-identical to the same pricer with ``--overlap off`` (one
  stream, one graph per step): contracts, targets, parameters, loss, grad norm;
* every target of every step written (slots NaN-filled first) and finite; the targets of a strided
  sample of 64 contracts per step against the oracle -- C3: ``oracle.training_targets`` (the reference
  arithmetic: f64 recursion, f32 stores, numpy FFT per batch row then mean; reference gbm.py:224-257,
  428-474, gbm_trainer.py:806-817) within 1e-5 per contract; C5: ``oracle.basket_kernel`` in the launch's
  reduction order (portable math) within the hw tolerance, 1e-4 of the row scale;
* the network half of step 1 on the session's own inputs and targets: C3's bf16 step against
  ``oracle/cvnn_mixed.py`` (operand "bf16": loss within 1e-4 rel, gradients within 2e-3 norm-relative);
  C5's f32 step against ``oracle.torch_step`` (torch-cpu ``_torch_step``, gbm_trainer.py:819-835: loss within
  1e-4 rel, grad norm 1e-3, post-Adam parameters 1e-4 where the gradient is resolved).
Reference anchor for the step: gbm_trainer.py:1532-1597.
"""

from __future__ import annotations

import copy
import os
import sys

import numpy as np
import pytest
import torch

from tests.test_reference_fixtures import per_contract_rel

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

STEPS = 3
SAMPLE = 64


def _session(config: str, overlap: bool, steps: int) -> dict:
    """Train `steps` steps with the bench's pricer for `config`; CPU copies of every step slot, the
    model after the steps, the flat [grads..., loss] buffer of the last step and the session facts."""
    import bench
    from tests.helpers import expect_success, make_training_config

    args = bench.parse(["--config", config] + ([] if overlap else ["--overlap", "off"]))
    assert (args.math, args.store) == ("hw", "all")
    B = bench.CONFIGS[config][0]
    pricer, model = bench.make_pricer(args, torch.device("cuda", 0))
    params0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    session = expect_success(pricer.open_session(make_training_config(num_batches=steps, batch_size=B,
                                                                      learning_rate=1e-2)))
    prog = session.program
    for s in prog.slots:  # an unwritten target, contract or CVNN input shows as NaN
        s.targets.fill_(complex("nan"))
        s.contracts.fill_(float("nan"))
        s.real_in.fill_(float("nan"))
    for i in range(steps):
        expect_success(session.step(prefetch_next=i + 1 < steps))
    eng = session.engine
    facts = {"kernel": eng.kernel_name, "chunk": eng.chunk, "launches": -(-eng.B // eng.chunk),
             "streams": len(session.mc_streams), "overlapped": session.stream is not session.mc_stream,
             "network_cus": session.network_cus_used,
             "captured": prog.captured, "network": prog.fused.kernels if prog.fused is not None else None,
             "table": ([(t.in_features, t.out_features, t.activation, t.w_re, t.w_im, t.b_re, t.b_im, t.act_bias)
                        for t in prog.fused.table] if prog.fused is not None else None)}
    final = session.close()
    slots = [(prog.slots[k].contracts.cpu().numpy().copy(), prog.slots[k].targets.cpu().numpy().copy(),
              prog.slots[k].real_in.cpu().numpy().copy()) for k in range(steps)]
    out = {"model": copy.deepcopy(model).cpu(), "params0": params0, "slots": slots, "loss": final.loss,
           "grad_norm": final.grad_norm, "flat": prog.flat.cpu().clone(), "facts": facts}
    del session, prog, pricer, model
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


_CACHE: dict[tuple[str, bool, int], dict] = {}


def session(config: str, overlap: bool = True, steps: int = STEPS) -> dict:
    """One run per (config, overlap, steps) per test process: each C3 pricer holds half the HBM of path
    scratch, so runs never overlap in time and their results are kept on the host."""
    key = (config, overlap, steps)
    if key not in _CACHE:
        _CACHE[key] = _session(config, overlap, steps)
    return _CACHE[key]


@pytest.fixture(scope="module", autouse=True)
def _free_cache():
    yield
    _CACHE.clear()


EXPECT = {"c3": ("resident_kernel(sliced)", 8192, 2, "mfma_bf16", 32),
          "c5": ("basket_resident_kernel", 2731, 3, "mfma_f32", 0)}


@pytest.mark.parametrize("config", ["c3", "c5"])
def test_session_uses_the_bench_policy(config) -> None:
    f = session(config)["facts"]
    kernel, chunk, launches, network, net_cus = EXPECT[config]
    assert (f["kernel"], f["chunk"], f["launches"], f["network"]) == (kernel, chunk, launches, network)
    # exchanging launches: one MC stream, the network on its own stream beside it (C3: on 32 CU-masked CUs, the
    # sliced launch sized to the rest; C5: unmasked), graphs replayed
    assert f["streams"] == 1 and f["overlapped"] and f["captured"]
    assert f["network_cus"] == net_cus


@pytest.mark.parametrize("config", ["c3", "c5"])
def test_session_equals_one_stream_run(config) -> None:
    """Overlapped MC/network streams + per-slot graphs + prefetch == the sequential single-stream program,
    bit for bit, over three steps."""
    a, b = session(config), session(config, overlap=False)
    assert not b["facts"]["overlapped"] and b["facts"]["streams"] == 1
    for step, (sa, sb) in enumerate(zip(a["slots"], b["slots"], strict=True)):
        for name, xa, xb in zip(("contracts", "targets", "real_in"), sa, sb):
            np.testing.assert_array_equal(xa, xb, err_msg=f"{config} step {step} {name}")
    for (name, pa), pb in zip(a["model"].named_parameters(), b["model"].parameters(), strict=True):
        assert torch.equal(pa, pb), name
    assert a["loss"] == b["loss"] and a["grad_norm"] == b["grad_norm"]


def _sample(step: int, B: int) -> np.ndarray:
    return np.arange(step % (B // SAMPLE), B, B // SAMPLE)


def _bad(rel: np.ndarray, idx: np.ndarray, tol: float) -> str:
    """Failing contracts with their index and (index mod 8): the XCD a whole-contract launch put them on."""
    bad = [(int(i), int(i) % 8, float(r)) for i, r in zip(idx, rel) if not r < tol]
    return f"{len(bad)} contracts above {tol}: (index, index mod 8, rel) {bad[:16]}"


def test_c3_session_targets_match_oracle(oracle) -> None:
    import bench
    from tests.helpers import make_domain_bounds

    B, T, N, M = bench.CONFIGS["c3"][:4]
    lo, hi = make_domain_bounds().arrays()
    for step, (contracts, targets, real_in) in enumerate(session("c3")["slots"]):
        np.testing.assert_array_equal(contracts, oracle.sobol_contracts(7, step * B, B, lo, hi))
        np.testing.assert_array_equal(real_in, contracts.astype(np.float32))
        finite = np.isfinite(targets).all(axis=1)
        assert finite.all(), f"step {step}: unwritten targets at {np.flatnonzero(~finite)[:16]}"
        idx = _sample(step, B)
        want = np.concatenate([oracle.training_targets(contracts[i:i + 1], T, N, M, seed=7, ordinal0=step * B + int(i))
                               for i in idx])
        rel = per_contract_rel(targets[idx], want)
        assert rel.max() < 1e-5, f"step {step}: " + _bad(rel, idx, 1e-5)


def test_c5_session_targets_match_oracle(oracle) -> None:
    import bench
    from spectralmc_amd.basket import BasketConfig

    B, T, N, M = bench.CONFIGS["c5"][:4]
    A = bench.BASKET_ASSETS["c5"]
    lo, hi = BasketConfig(n_assets=A, timesteps=T, network_size=N, batches_per_mc_run=M).arrays()
    wg, W = oracle.basket_order(A, T, N, M)
    assert (wg, W) == (1024, 32)
    for step, (contracts, targets, real_in) in enumerate(session("c5")["slots"]):
        np.testing.assert_array_equal(contracts, oracle.sobol_contracts(7, step * B, B, lo, hi))
        np.testing.assert_array_equal(real_in, contracts.astype(np.float32))
        finite = np.isfinite(targets).all(axis=1)
        assert finite.all(), f"step {step}: unwritten targets at {np.flatnonzero(~finite)[:16]}"
        idx = _sample(step, B)
        want = np.concatenate([oracle.basket_kernel(contracts[i:i + 1], A, T, N, M, 7, ordinal0=step * B + int(i),
                                                    wg=wg, slices=W)[2] for i in idx])
        scale = np.abs(want).max(axis=1) + 1e-30
        rel = np.abs(targets[idx] - want).max(axis=1) / scale  # hw math: 1e-4 of the row scale
        assert rel.max() < 1e-4, f"step {step}: " + _bad(rel, idx, 1e-4)


def test_c3_session_network_step_matches_oracle() -> None:
    """Step 1's bf16 network half (forward, spectral MSE, backward) on the session's own CVNN inputs and
    targets against the explicit-precision restatement with the same bf16 roundings."""
    from oracle.cvnn_mixed import cvnn_step

    run = session("c3", steps=1)
    contracts, targets, real_in = run["slots"][0]
    assert np.isfinite(targets).all()
    loss, g = cvnn_step(run["facts"]["table"], run["params0"].numpy(), real_in, None, targets, operand="bf16")
    flat = run["flat"]
    got = flat[:-1].double().numpy()
    assert float(flat[-1]) == pytest.approx(loss, rel=1e-4)
    assert run["loss"] == pytest.approx(loss, rel=1e-4)
    assert np.linalg.norm(got - g) / np.linalg.norm(g) < 2e-3
    assert run["grad_norm"] == pytest.approx(float(np.linalg.norm(g.astype(np.float64))), rel=2e-3)


def test_c5_session_network_step_matches_oracle(oracle) -> None:
    """Step 1's f32 network step (MFMA forward/backward, fused Adam) on the session's own inputs and targets
    against torch-cpu's _torch_step on the same initial weights."""
    import bench
    from tests.helpers import make_test_cvnn

    run = session("c5", steps=1)
    contracts, targets, real_in = run["slots"][0]
    assert np.isfinite(targets).all()
    B, T, N, M, widths = bench.CONFIGS["c5"][:5]
    cpu_model = make_test_cvnn(n_inputs=contracts.shape[1], n_outputs=N, seed=123, dtype=torch.float32, device="cpu",
                               hidden_layers=len(widths), hidden_width=widths[0])
    p0 = torch.cat([p.detach().reshape(-1) for p in cpu_model.parameters()])
    assert torch.equal(p0, run["params0"])
    x = torch.from_numpy(real_in)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert run["loss"] == pytest.approx(ref.loss, rel=1e-4)
    assert run["grad_norm"] == pytest.approx(ref.grad_norm, rel=1e-3)
    for (name, pg), pc in zip(run["model"].named_parameters(), cpu_model.parameters(), strict=True):
        g = pc.grad.detach().double().reshape(-1)
        a, b = pg.detach().double().reshape(-1), pc.detach().double().reshape(-1)
        resolved = g.abs() > 1e-4 * float(g.abs().max())
        rel = float((a - b)[resolved].norm() / max(float(b[resolved].norm()), 1e-12))
        assert rel < 1e-4, (name, rel)
        assert int((~resolved & ((a - b).abs() > 1e-4)).sum()) <= max(2, b.numel() // 1000), name
