"""End-to-end workflow of the reference's guided full-stack test
(reference tests/test_e2e/test_full_stack_cvnn_pricer.py): configs -> GPU training ->
checkpoint commit -> reload into a differently seeded template -> inference, driven only
through the reference API names (``spectralmc.*`` resolves to this build)."""

from __future__ import annotations

import math

import pytest
import torch

from spectralmc.gbm import BlackScholes
from spectralmc.gbm_trainer import GbmCVNNPricer
from spectralmc.models.numerical import Precision
from spectralmc.storage import AsyncBlockchainModelStore, commit_snapshot, load_snapshot_from_checkpoint
from tests.helpers import (
    expect_success,
    make_black_scholes_config,
    make_domain_bounds,
    make_gbm_cvnn_config,
    make_simulation_params,
    make_test_cvnn,
    make_training_config,
    max_param_diff,
    seed_all_rngs,
)

pytestmark = pytest.mark.gpu


def _config(model, sp):
    return make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                domain_bounds=make_domain_bounds())


async def test_train_commit_reload_predict(async_store: AsyncBlockchainModelStore) -> None:
    seed_all_rngs(123)
    sp = make_simulation_params(timesteps=16, network_size=128, batches_per_mc_run=4, threads_per_block=256,
                                mc_seed=7, buffer_size=512, skip=0, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=6, n_outputs=sp.network_size, seed=123, dtype=torch.float32)
    pricer = expect_success(GbmCVNNPricer.create(_config(model, sp)))
    result = expect_success(pricer.train(make_training_config(num_batches=4, batch_size=8, learning_rate=1e-2)))
    assert result.total_batches == 4 and math.isfinite(result.final_loss)

    snapshot = result.updated_config
    version = await commit_snapshot(async_store, snapshot, "full-stack demo checkpoint")
    assert version.counter == 0 and version.commit_message == "full-stack demo checkpoint"

    template = make_test_cvnn(n_inputs=6, n_outputs=sp.network_size, seed=999, dtype=torch.float32)
    assert max_param_diff(template, snapshot.cvnn) > 0
    reloaded = expect_success(await load_snapshot_from_checkpoint(async_store, version, template, snapshot))
    assert max_param_diff(reloaded.cvnn, snapshot.cvnn) == 0.0
    assert reloaded.global_step == snapshot.global_step == 4
    assert reloaded.optimizer_state is not None

    loaded = expect_success(GbmCVNNPricer.create(reloaded))
    contracts = [BlackScholes.Inputs(X0=100.0, K=95.0, T=0.5, r=0.03, d=0.01, v=0.25),
                 BlackScholes.Inputs(X0=120.0, K=105.0, T=1.0, r=0.02, d=0.00, v=0.30)]
    prices = expect_success(loaded.predict_price(contracts))
    assert len(prices) == 2
    for p in prices:
        assert all(math.isfinite(v) for v in p.model_dump(mode="python").values())
    again = expect_success(pricer.predict_price(contracts))
    assert [p.put_price for p in prices] == [p.put_price for p in again]  # same weights, same prices


async def test_resume_from_checkpoint_continues_training(async_store: AsyncBlockchainModelStore) -> None:
    """A reloaded snapshot (weights + Adam state from the checkpoint) trains on identically."""
    sp = make_simulation_params(timesteps=8, network_size=64, batches_per_mc_run=4, mc_seed=11, buffer_size=1,
                                dtype=Precision.float32)
    m_a = make_test_cvnn(n_inputs=6, n_outputs=64, seed=5, dtype=torch.float32)
    a = expect_success(GbmCVNNPricer.create(_config(m_a, sp)))
    r1 = expect_success(a.train(make_training_config(num_batches=2, batch_size=8)))
    v = await commit_snapshot(async_store, r1.updated_config, "mid-run")
    tmpl = make_test_cvnn(n_inputs=6, n_outputs=64, seed=6, dtype=torch.float32)
    snap = expect_success(await load_snapshot_from_checkpoint(async_store, v, tmpl, r1.updated_config))
    b = expect_success(GbmCVNNPricer.create(snap))
    expect_success(a.train(make_training_config(num_batches=2, batch_size=8)))
    expect_success(b.train(make_training_config(num_batches=2, batch_size=8)))
    assert max_param_diff(m_a, tmpl) == 0.0
