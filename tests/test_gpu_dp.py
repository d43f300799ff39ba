"""Data-parallel GbmCVNNPricer on the GPU code path: 2 ranks (gloo process group, both on
cuda:0 — a 1-GPU box cannot host two RCCL ranks) vs one process with the global batch.
Exercises the engine's rank sharding, the fused network step with the separate Adam launch,
and the graphs around the eager all-reduce."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, N, M, B_LOCAL, STEPS = 16, 64, 4, 8, 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _train(batch: int, outfile: str, basket: int = 0) -> None:
    from spectralmc_amd.gbm_trainer import GbmCVNNPricer
    from spectralmc_amd.models.numerical import Precision
    from tests.helpers import (
        expect_success,
        make_black_scholes_config,
        make_domain_bounds,
        make_gbm_cvnn_config,
        make_simulation_params,
        make_test_cvnn,
        make_training_config,
    )

    m = 32 if basket else M  # the basket engine takes N*M in multiples of 2048
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=m, mc_seed=7, buffer_size=1,
                                dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=3 * basket + 4 if basket else 6, n_outputs=N, seed=123, dtype=torch.float32, device="cuda:0",
                           hidden_layers=2)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    if basket:
        from spectralmc_amd.basket import BasketConfig, use_basket_engine

        use_basket_engine(pricer, BasketConfig(n_assets=basket, timesteps=T, network_size=N, batches_per_mc_run=m))
    res = expect_success(pricer.train(make_training_config(num_batches=STEPS, batch_size=batch)))
    snap = res.updated_config
    np.savez(outfile, loss=res.final_loss, grad_norm=res.final_grad_norm, sobol_skip=snap.sobol_skip,
             **{f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(model.parameters())})


def _rank(rank: int, world: int, port: int, outdir: str, basket: int) -> None:
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _train(B_LOCAL, os.path.join(outdir, f"rank{rank}.npz"), basket)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("basket", [0, 4], ids=["single_asset", "basket4"])
def test_two_ranks_match_one_process_with_the_global_batch(tmp_path, basket) -> None:
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(tmp_path), basket)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    single = tmp_path / "single.npz"
    _train(2 * B_LOCAL, str(single), basket)
    r0, r1, s = np.load(tmp_path / "rank0.npz"), np.load(tmp_path / "rank1.npz"), np.load(single)
    for k in r0.files:
        np.testing.assert_array_equal(r0[k], r1[k])  # replicas stay bit-identical
    assert int(r0["sobol_skip"]) == int(s["sobol_skip"]) == STEPS * 2 * B_LOCAL
    np.testing.assert_allclose(r0["loss"], s["loss"], rtol=1e-4)
    for k in r0.files:
        if k.startswith("p"):
            np.testing.assert_allclose(r0[k], s[k], rtol=1e-4, atol=3e-4)
