"""Exchanging path launches beside a spinning collective.

The sliced resident kernel (C3: W = 4 workgroups per contract) and the resident basket kernel (C5:
W = 32) need every workgroup of a group co-resident: partners poll a bounded time (~1 s) and then give
up with NaN targets and SMC_ERR_EXCHANGE_TIMEOUT.  In a data-parallel run the step's RCCL all-reduce is
a kernel that can spin on a few CUs while it waits for a slow peer (e.g. rank 0 committing a
checkpoint, reference gbm_trainer.py:1296-1302: training must not die on a slow commit); a resident
workgroup needs a whole CU, so a launch dispatched beside it may not fit.  Since round 6 a data-parallel
session keeps the network part and the all-reduce (issued on the network stream, dp.RcclComm) on CU-masked
CUs of their own and sizes the exchanging launch to the others, so the launch runs beside the collective
(DESIGN.md section 5); GbmCVNNPricer.exchange_after_network = True still orders it after the previous step's
network part, all-reduce included (round 4-5's data-parallel default).

Here the all-reduce is replaced by a kernel that spins ~2 s on the network stream (a stand-in for a
stalled peer), and training at the C3 and C5 per-contract shapes must finish bit-identical to the
run without it, with the sync area's status word clear, in both orders.
"""

from __future__ import annotations

import time

import pytest
import torch

from spectralmc.gbm_trainer import GbmCVNNPricer
from spectralmc.models.numerical import Precision
from spectralmc_amd import dp as dp_mod
from spectralmc_amd.basket import BasketConfig, use_basket_engine
from tests.helpers import (
    expect_success,
    make_black_scholes_config,
    make_domain_bounds,
    make_gbm_cvnn_config,
    make_simulation_params,
    make_test_cvnn,
    make_training_config,
    max_param_diff,
)

pytestmark = pytest.mark.gpu


class SpinningCollective:
    """A one-rank data-parallel context whose all-reduce is a ~`seconds` spin kernel on the current
    (network) stream: what a collective waiting for a stalled peer looks like to the chip."""

    world_size = 1
    rank = 0

    def __init__(self, cycles: int) -> None:
        self.cycles = cycles
        self.calls = 0

    def all_reduce_mean(self, flat: torch.Tensor) -> None:
        self.calls += 1
        if self.cycles:
            torch.cuda._sleep(self.cycles)


def _spin_cycles(seconds: float) -> int:
    """torch.cuda._sleep cycles that spin for about `seconds` on this device (measured)."""
    probe = 20_000_000
    torch.cuda._sleep(probe)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(probe)
    e1.record()
    e1.synchronize()
    per_ms = probe / max(e0.elapsed_time(e1), 1e-3)
    return int(per_ms * seconds * 1e3)


def _pricer(shape: str):
    T = 16
    if shape == "c3":  # C3 per-contract shape: P = 262,144 -> resident_kernel(sliced), W = 4
        N, M, n_in, basket = 1024, 256, 6, None
    else:              # C5 per-contract shape: 4 assets, P = 131,072 -> basket_resident_kernel, W = 32
        N, M, basket = 256, 512, BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=512,
                                              mc_seed=7, math="hw")
        n_in = basket.dim
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                mc_seed=7, buffer_size=512, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=n_in, n_outputs=N, seed=11, dtype=torch.float32)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    p = expect_success(GbmCVNNPricer.create(cfg))
    p.math_mode = "hw"
    if basket is not None:
        use_basket_engine(p, basket)
    return p, model


@pytest.mark.parametrize("order", [None, True], ids=["beside_on_masked_cus", "after_network"])
@pytest.mark.parametrize("shape,batch", [("c3", 64), ("c5", 16)])
def test_exchanging_launch_beside_a_spinning_collective(monkeypatch, shape: str, batch: int, order) -> None:
    steps = 3
    cycles = _spin_cycles(2.0)

    def run(spin: int):
        ctx = SpinningCollective(spin)
        monkeypatch.setattr(dp_mod, "current", lambda: ctx)
        p, model = _pricer(shape)
        p.exchange_after_network = order
        sess = expect_success(p.open_session(make_training_config(num_batches=steps, batch_size=batch)))
        assert sess.engine.exchanges and sess._mc_after_nn == bool(order)
        assert sess.network_cus_used > 0  # the collective's stream and the exchanging launch's: disjoint CUs
        t0 = time.perf_counter()
        for i in range(steps):
            expect_success(sess.step(prefetch_next=i + 1 < steps))
        st = sess.close()  # raises SmcError(SMC_ERR_EXCHANGE_TIMEOUT) if any exchange gave up
        return st, model, ctx.calls, time.perf_counter() - t0

    ref, m_ref, _, _ = run(0)
    st, m_spin, calls, wall = run(cycles)
    assert calls == steps and wall > 1.5 * steps  # every step's all-reduce spun ~2 s
    assert st.loss == ref.loss and st.grad_norm == ref.grad_norm
    assert max_param_diff(m_ref, m_spin) == 0.0
    assert torch.isfinite(torch.tensor(st.loss))
