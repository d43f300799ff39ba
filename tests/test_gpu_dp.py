"""Data-parallel GbmCVNNPricer on the GPU code path: 2 ranks (gloo process group, both on
cuda:0 — a 1-GPU box cannot host two RCCL ranks) vs one process with the global batch.
Exercises the engine's rank sharding, the fused network step with the separate Adam launch,
and the graphs around the eager all-reduce."""

from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, N, M, B_LOCAL, STEPS = 16, 64, 4, 8, 4


def _rdzv(outdir: str) -> str:
    """A file rendezvous in the test's own directory: no TCP port to race other processes for (a port
    picked free and released can be taken again before the ranks bind it)."""
    return "file://" + os.path.join(outdir, "rdzv")


# BASELINE configs[2] / configs[4] per-rank contract shapes (batches kept small): C3's P = 262,144 runs the
# sliced resident kernel (W = 4 co-resident workgroups per contract), C5's 4-asset P = 131,072 the resident
# basket kernel (W = 32); both exchange sums between workgroups
SHAPES = {"c3": (1024, 256, 0), "c5": (256, 512, 4)}


def _train(batch: int, outfile: str, basket: int | str = 0) -> None:
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

    # basket > 0: the basket engine (N*M in multiples of 2048); basket < 0: P = 4096, the shape the
    # whole-contract resident kernel takes (MC lanes, the network on CU-masked streams); "c3" / "c5": SHAPES
    n = N
    if isinstance(basket, str):
        n, m, basket = SHAPES[basket]
    else:
        m = 32 if basket > 0 else 64 if basket < 0 else M
    sp = make_simulation_params(timesteps=T, network_size=n, batches_per_mc_run=m, mc_seed=7, buffer_size=1,
                                dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=3 * basket + 4 if basket > 0 else 6, n_outputs=n, seed=123, dtype=torch.float32,
                           device="cuda:0", hidden_layers=2)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    if basket < 0:
        pricer.mc_lanes_short = 2  # keep two MC lanes at this short launch (the policy would run one)
    if basket > 0:
        from spectralmc_amd.basket import BasketConfig, use_basket_engine

        use_basket_engine(pricer, BasketConfig(n_assets=basket, timesteps=T, network_size=n, batches_per_mc_run=m))
    from spectralmc_amd import dp

    if dp.current() is not None and m >= 256:  # the exchanging shapes: the session's own policy, recorded
        sess = expect_success(pricer.open_session(make_training_config(num_batches=1, batch_size=batch)))
        facts = (sess.engine.exchanges, sess._mc_after_nn, sess.network_cus_used)
        sess.close()
        assert facts[0] and not facts[1] and facts[2] > 0, facts  # beside the collective, on masked CUs
    res = expect_success(pricer.train(make_training_config(num_batches=STEPS, batch_size=batch)))  # raises on a
    snap = res.updated_config  # timed-out exchange (the sync area's status word), so a pass means it stayed clear
    np.savez(outfile, loss=res.final_loss, grad_norm=res.final_grad_norm, sobol_skip=snap.sobol_skip,
             **{f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(model.parameters())})


def _rank(rank: int, world: int, outdir: str, basket: int) -> None:
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=_rdzv(outdir), rank=rank, world_size=world)
    try:
        _train(B_LOCAL, os.path.join(outdir, f"rank{rank}.npz"), basket)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("basket", [0, 4, -1, "c3", "c5"], ids=["single_asset", "basket4", "resident_lanes", "c3_sliced",
                                                                "c5_basket_resident"])
def test_two_ranks_match_one_process_with_the_global_batch(tmp_path, basket) -> None:
    """Two gloo ranks on the GPU code path (both on cuda:0) against one process with both ranks' contracts.
    c3 / c5: the exchanging launches of BASELINE configs[2] / configs[4] per rank, prefetched beside the
    previous step's network part and all-reduce (no serialisation since round 6: the network stream and the
    collective on CU-masked CUs, the exchanging launch sized to the rest); the sync area's status word stays
    clear (train() fails on a timed-out exchange).  Unmeasured at 8 GPUs (no node in this pool)."""
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, 2, str(tmp_path), basket)) for r in range(2)]
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


def _rccl_single_rank(outdir: str, outfile: str, shape: int = 0) -> None:
    """One RCCL rank driving the data-parallel step program: the network half as the two
    captured graphs around the eager RCCL all-reduce on the network stream, Adam as its own
    launch (fuse_adam off) — the path an 8-GPU node takes, minus the other ranks."""
    import torch.distributed as dist

    import spectralmc_amd.dp as dp
    import spectralmc_amd.gbm_trainer  # noqa: F401

    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=_rdzv(outdir), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        flat = torch.arange(7, dtype=torch.float32, device="cuda")
        dp.DataParallel(world_size=1, rank=0).all_reduce_mean(flat)  # torch.distributed's collective
        torch.testing.assert_close(flat.cpu(), torch.arange(7, dtype=torch.float32))
        comm = dp.RcclComm(0, 1)  # the step's own communicator: ncclAllReduce on the caller's stream
        ctx = dp.DataParallel(world_size=1, rank=0, comm=comm)
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            flat2 = torch.arange(9, dtype=torch.float32, device="cuda") * 2
            ctx.all_reduce_mean(flat2)
        side.synchronize()
        torch.testing.assert_close(flat2.cpu(), torch.arange(9, dtype=torch.float32) * 2)
        dp.current = lambda: ctx  # a 1-rank RCCL group: world_size 1 normally means "no DP"
        _train(2 * B_LOCAL, outfile, shape)
        comm.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shape", [0, -1, "c3"], ids=["p256", "resident_lanes", "c3_sliced"])
def test_rccl_step_program_single_rank_equals_plain_run(tmp_path, shape) -> None:
    """The RCCL (backend "nccl") code path on one GPU: init with a device id, the eager
    all-reduce between the fwd/bwd graph and the Adam graph.  A 1-rank all-reduce is the
    identity, so the run must equal the non-DP run up to the separate Adam launch (adam_kernel)
    standing in for the update fused into the gradient reduction: the same formula in two
    compilation units, equal to f32 rounding (measured: 32 of 192 weights 1 ulp apart after 4
    steps), and the grad norm's partial sums grouped differently."""
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rccl_single_rank, args=(str(tmp_path), str(tmp_path / "rccl.npz"), shape))
    p.start()
    p.join(timeout=600)
    assert p.exitcode == 0, f"RCCL rank exited with {p.exitcode}"
    plain = tmp_path / "plain.npz"
    _train(2 * B_LOCAL, str(plain), shape)
    a, b = np.load(tmp_path / "rccl.npz"), np.load(plain)
    assert int(a["sobol_skip"]) == int(b["sobol_skip"])
    for k in a.files:
        if k != "sobol_skip":
            np.testing.assert_allclose(a[k], b[k], rtol=1e-5, atol=1e-7)
