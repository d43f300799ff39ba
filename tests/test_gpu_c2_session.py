"""The timed C2 session end to end (BASELINE configs[1], north_star's own acceptance criterion):
``GbmCVNNPricer`` built and configured exactly as ``bench.py`` builds it for the driver's default run
(``bench.make_pricer(bench.parse([]))``: B = 4096 contracts x 65,536 paths, T = 16, N = M = 256,
6 -> 32 -> 32 -> 256 CVNN, hw math, full path store, 4 MC lanes (mc_lanes_long), the network on a 32-CU masked stream,
per-slot hipGraphs after 2 eager steps, next step's MC part prefetched beside the network part).

* three steps (the third a graph replay) bit-identical to the same pricer with
  ``overlap_mc = False`` (one stream, one graph per step);
* every step's targets (all 4096 contracts of step 1, a strided sample of steps 2 and 3, which ran on
  lane 1 and as a graph replay) within 1e-5 per contract of the reference-mode oracle
  (oracle.training_targets: f64 recursion, f32 stores, numpy-order FFT per batch then mean,
  reference gbm.py:224-257, 428-474 and gbm_trainer.py:806-817), every target written (slots NaN-filled
  before the session runs);
* step 1's spectral loss within 1e-4 rel, grad norm within 1e-3 rel and post-Adam parameters within
  1e-4 (norm-relative, over the elements whose gradient is resolved) of the oracle's full C2 step:
  oracle.training_targets on all 4096 contracts + oracle.torch_step (torch-cpu _torch_step,
  reference gbm_trainer.py:1532-1597, 819-835).
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

B, T, N, M = 4096, 16, 256, 256


def _session(overlap: bool, steps: int):
    """Train `steps` steps with the bench's pricer; returns (model, per-step slot copies, loss, grad norm,
    session facts)."""
    import bench
    from tests.helpers import expect_success, make_training_config

    args = bench.parse([] if overlap else ["--overlap", "off"])
    assert (args.config, args.lanes, args.net_cus, args.math, args.store) == ("c2", 2, 32, "hw", "all")
    pricer, model = bench.make_pricer(args, torch.device("cuda", 0))
    session = expect_success(pricer.open_session(make_training_config(num_batches=steps, batch_size=B,
                                                                      learning_rate=1e-2)))
    prog = session.program
    for s in prog.slots:  # an unwritten target or contract shows as NaN
        s.targets.fill_(complex("nan"))
        s.contracts.fill_(float("nan"))
    for i in range(steps):
        expect_success(session.step(prefetch_next=i + 1 < steps))
    facts = {"lanes": session.engine.lanes, "network_cus": session.network_cus_used, "captured": prog.captured,
             "kernel": session.engine.kernel_name, "streams": len(session.mc_streams)}
    final = session.close()
    slots = [(prog.slots[k].contracts.cpu().numpy().copy(), prog.slots[k].targets.cpu().numpy().copy())
             for k in range(steps)]
    out = (copy.deepcopy(model).cpu(), slots, final.loss, final.grad_norm, facts)
    del session, prog, pricer, model
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


@pytest.fixture(scope="module")
def overlapped():
    return _session(True, 3)


def test_c2_session_uses_the_bench_policy(overlapped) -> None:
    facts = overlapped[4]
    assert facts["kernel"] == "resident_kernel"
    assert facts["lanes"] == 4 and facts["network_cus"] == 32 and facts["captured"]


def test_c2_session_equals_one_stream_run(overlapped) -> None:
    """MC lanes + masked network stream + per-slot graphs + prefetch == the sequential single-stream
    program, bit for bit, over three steps."""
    m_a, slots_a, loss_a, gn_a, _ = overlapped
    m_b, slots_b, loss_b, gn_b, facts_b = _session(False, 3)
    assert facts_b["lanes"] == 1 and facts_b["network_cus"] == 0 and facts_b["streams"] == 1
    for (ca, ta), (cb, tb) in zip(slots_a, slots_b, strict=True):
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(ta, tb)
    for (name, pa), pb in zip(m_a.named_parameters(), m_b.parameters(), strict=True):
        assert torch.equal(pa, pb), name
    assert loss_a == loss_b and gn_a == gn_b


def test_c2_session_targets_match_oracle(oracle, overlapped) -> None:
    from tests.helpers import make_domain_bounds

    slots = overlapped[1]
    lo, hi = make_domain_bounds().arrays()
    for step, (contracts, targets) in enumerate(slots):
        np.testing.assert_array_equal(contracts, oracle.sobol_contracts(7, step * B, B, lo, hi))
        assert np.isfinite(targets).all(), f"step {step}: unwritten targets"
        if step == 0:
            continue  # all 4096 of step 1: test_c2_session_step_matches_oracle
        idx = np.arange(step, B, B // 64)
        want = np.stack([oracle.training_targets(contracts[i:i + 1], T, N, M, seed=7, ordinal0=step * B + int(i))[0]
                         for i in idx])
        assert per_contract_rel(targets[idx], want).max() < 1e-5, step


def test_c2_session_step_matches_oracle(oracle) -> None:
    """Step 1 of the timed session against the oracle's full C2 step (all 4096 contracts)."""
    import bench
    from tests.helpers import make_domain_bounds, make_test_cvnn

    model_gpu, slots, loss, gn, _ = _session(True, 1)
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    np.testing.assert_array_equal(slots[0][0], contracts)
    want = oracle.training_targets(contracts, T, N, M, seed=7, ordinal0=0)
    got = slots[0][1]
    assert np.isfinite(got).all()
    assert per_contract_rel(got, want).max() < 1e-5
    widths = bench.CONFIGS["c2"][4]
    cpu_model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device="cpu",
                               hidden_layers=len(widths), hidden_width=widths[0])
    x = torch.tensor(contracts, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(want),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert loss == pytest.approx(ref.loss, rel=1e-4)  # north_star: spectral-loss match within 1e-4 rel
    assert gn == pytest.approx(ref.grad_norm, rel=1e-3)
    # Adam's first step is ~ lr * sign(g): compare where the gradient is resolved above the f32 noise of
    # a B = 4096 reduction (an element with |g| ~ 0 may step either way on either device)
    for (name, pg), pc in zip(model_gpu.named_parameters(), cpu_model.parameters(), strict=True):
        g = pc.grad.detach().double().reshape(-1)
        a, b = pg.detach().double().reshape(-1), pc.detach().double().reshape(-1)
        resolved = g.abs() > 1e-4 * float(g.abs().max())
        rel = float((a - b)[resolved].norm() / max(float(b[resolved].norm()), 1e-12))
        assert rel < 1e-4, (name, rel)
        assert int((~resolved & ((a - b).abs() > 1e-4)).sum()) <= max(2, b.numel() // 1000), name
