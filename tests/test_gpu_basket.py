"""Correlated multi-asset (basket) engine through the C ABI vs the oracle's kernel-mode
restatement (oracle_basket_kernel, in the reduction order of the launch: oracle.basket_order):
bit-exact in portable math for basket_kernel (+ basket_cf_kernel) and basket_resident_kernel (W = 1
... 32 workgroups per contract, the C5 shape included); HW math within the stated north-star
tolerance; statistics of the correlated drivers; training through GbmCVNNPricer."""

from __future__ import annotations

import copy

import numpy as np
import pytest
import torch

from spectralmc_amd import _lib
from spectralmc_amd.basket import BasketConfig, BasketEngine, basket_targets, use_basket_engine
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
    poisoned,
)

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _contracts(oracle, cfg: BasketConfig, n: int, skip: int = 0) -> np.ndarray:
    lo, hi = cfg.arrays()
    return oracle.sobol_contracts(cfg.mc_seed, skip, n, lo, hi)


@pytest.mark.parametrize("A", [1, 3, 4, 8])
@pytest.mark.parametrize("T", [16, 5])
@pytest.mark.parametrize("resident", [True, False])
def test_portable_bit_exact_vs_oracle(oracle, A, T, resident) -> None:
    """T = 16 with a sync area runs basket_resident_kernel (P = 4096: W = 1), else basket_kernel."""
    cfg = BasketConfig(n_assets=A, timesteps=T, network_size=64, batches_per_mc_run=64, math="portable")
    B = 6
    c = _contracts(oracle, cfg, B)
    wg, W = oracle.basket_order(A, T, 64, 64, resident)
    assert (wg == 1024) == (resident and T == 16 and A <= 6)  # A > 6: the LDS plan does not fit
    want_paths, want_sum, want_t = oracle.basket_kernel(c, A, T, 64, 64, cfg.mc_seed, ordinal0=3, want_paths=True,
                                                        wg=wg, slices=W)
    cd = torch.from_numpy(c).to(DEV)
    paths = poisoned((B, A, T, cfg.total_paths), torch.float32, DEV)
    tsum = poisoned((B, A), torch.float64, DEV)
    got = basket_targets(cd, cfg, ordinal0=3, paths=paths, terminal_sum=tsum, resident=resident)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(paths.cpu().numpy(), want_paths)
    np.testing.assert_array_equal(tsum.cpu().numpy(), want_sum)
    np.testing.assert_array_equal(got.cpu().numpy(), want_t)


@pytest.mark.parametrize("A,N,M,B", [(4, 256, 512, 11), (4, 256, 64, 150), (2, 1024, 16, 40), (1, 4, 2048, 5),
                                     (6, 256, 32, 9), (3, 2048, 6, 17), (4, 256, 512, 40), (2, 256, 64, 260)])
def test_resident_sliced_bit_exact(oracle, A, N, M, B) -> None:
    """basket_resident_kernel with W = N*M/4096 workgroups per contract: C5's shape (W = 32, 8 groups,
    B = 11: some groups run two contracts, some one), several rounds per group (B = 150, W = 4), N = 4
    and N = 2048 (the extremes of the column mapping), A = 6 (the largest whose LDS plan fits), a non-power-of-two W (3);
    B = 40 at C5 (5 contracts per group) and B = 260 at W = 4: the dynamic tail (contracts of the last quarter of
    the rounds taken from the queue)."""
    cfg = BasketConfig(n_assets=A, timesteps=16, network_size=N, batches_per_mc_run=M, math="portable")
    wg, W = oracle.basket_order(A, 16, N, M)
    assert wg == 1024 and W == N * M // 4096
    c = _contracts(oracle, cfg, B, skip=3)
    _, want_sum, want = oracle.basket_kernel(c, A, 16, N, M, cfg.mc_seed, ordinal0=5, wg=wg, slices=W)
    cd = torch.from_numpy(c).to(DEV)
    tsum = poisoned((B, A), torch.float64, DEV)
    got = basket_targets(cd, cfg, ordinal0=5, terminal_sum=tsum)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tsum.cpu().numpy(), want_sum)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    # the full path matrix at the padded pitch: same targets, stored rows equal the oracle's
    if B <= 11:
        pitch = int(_lib.lib().smc_path_pitch(cfg.total_paths, 0))
        paths = poisoned((B, A, 16, pitch), torch.float32, DEV)
        again = basket_targets(cd, cfg, ordinal0=5, paths=paths, pitch=pitch)
        np.testing.assert_array_equal(again.cpu().numpy(), want)
        want_paths, _, _ = oracle.basket_kernel(c[:2], A, 16, N, M, cfg.mc_seed, ordinal0=5, want_paths=True,
                                                wg=wg, slices=W)
        np.testing.assert_array_equal(paths[:2, ..., :cfg.total_paths].cpu().numpy(), want_paths)


def test_resident_sync_area_left_zeroed_and_reusable(oracle) -> None:
    """Every launch leaves the sync area's counters zeroed, so back-to-back launches (and chunks)
    reuse it; the exchanged sums are rewritten before they are read."""
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=128, math="hw")
    eng = BasketEngine(cfg, 40, device=torch.device(DEV))
    assert eng.kernel_name == "basket_resident_kernel" and eng._sync is not None
    eng.set_position(0, 0)
    outs = []
    for _ in range(3):
        eng.set_position(0, 0)
        eng.enqueue_step()
        outs.append(eng.buffers.targets.clone())
    torch.cuda.synchronize()
    W = cfg.total_paths // 4096
    groups = torch.cuda.get_device_properties(0).multi_processor_count // W
    assert int(eng._sync[:128 + 128 * groups].count_nonzero()) == 0  # done counter + one line per group
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_resident_hw_close_to_split_pair(oracle) -> None:
    """HW math, C5 shape: the resident kernel and the split pair differ only in f64 summation order."""
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=512, math="hw")
    B = 24
    c = torch.from_numpy(_contracts(oracle, cfg, B, skip=9)).to(DEV)
    t1 = poisoned((B, 4), torch.float64, DEV)
    t2 = poisoned((B, 4), torch.float64, DEV)
    res = basket_targets(c, cfg, terminal_sum=t1).cpu().numpy()
    split = basket_targets(c, cfg, terminal_sum=t2, resident=False).cpu().numpy()
    np.testing.assert_allclose(t1.cpu().numpy(), t2.cpu().numpy(), rtol=1e-12)
    scale = np.abs(split).max(axis=1, keepdims=True) + 1e-30
    assert float((np.abs(res - split) / scale).max()) < 1e-6


@pytest.mark.parametrize("A,N,M,B", [(2, 64, 32, 1100), (4, 2048, 2, 530), (3, 12, 512, 9)])
def test_multi_round_and_general_shapes_bit_exact(oracle, A, N, M, B) -> None:
    """B above the resident grid (512 workgroups): several rounds of contract workgroups; N = 2048
    (4-column quads over the whole workgroup) and N = 12 (not a divisor of the chunk)."""
    cfg = BasketConfig(n_assets=A, timesteps=4, network_size=N, batches_per_mc_run=M, math="portable")
    c = _contracts(oracle, cfg, B, skip=5)
    _, want_sum, want = oracle.basket_kernel(c, A, 4, N, M, cfg.mc_seed, ordinal0=11)
    cd = torch.from_numpy(c).to(DEV)
    tsum = poisoned((B, A), torch.float64, DEV)
    got = basket_targets(cd, cfg, ordinal0=11, terminal_sum=tsum)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tsum.cpu().numpy(), want_sum)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    if B > 600:  # full path matrix, padded pitch
        pitch = int(_lib.lib().smc_path_pitch(cfg.total_paths, 0))
        paths = poisoned((B, A, 4, pitch), torch.float32, DEV)
        again = basket_targets(cd, cfg, ordinal0=11, paths=paths, pitch=pitch)
        np.testing.assert_array_equal(again.cpu().numpy(), want)


def test_terminal_store_and_padded_pitch_same_targets(oracle) -> None:
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=16, math="portable")
    B = 5
    c = _contracts(oracle, cfg, B, skip=64)
    wg, W = oracle.basket_order(4, 16, 256, 16)
    _, _, want = oracle.basket_kernel(c, 4, 16, 256, 16, cfg.mc_seed, wg=wg, slices=W)
    cd = torch.from_numpy(c).to(DEV)
    got_term = basket_targets(cd, cfg)
    pitch = int(_lib.lib().smc_path_pitch(cfg.total_paths, 0))
    paths = poisoned((B, 4, 16, pitch), torch.float32, DEV)
    got_all = basket_targets(cd, cfg, paths=paths, pitch=pitch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got_term.cpu().numpy(), want)
    np.testing.assert_array_equal(got_all.cpu().numpy(), want)


def test_hw_math_within_tolerance(oracle) -> None:
    """HW transcendentals (~1 ulp per op): targets within 1e-4 of the oracle relative to the row scale."""
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=64, math="hw")
    B = 16
    c = _contracts(oracle, cfg, B)
    wg, W = oracle.basket_order(4, 16, 256, 64)
    assert W == 4
    _, want_sum, want = oracle.basket_kernel(c, 4, 16, 256, 64, cfg.mc_seed, wg=wg, slices=W)
    tsum = poisoned((B, 4), torch.float64, DEV)
    got = basket_targets(torch.from_numpy(c).to(DEV), cfg, terminal_sum=tsum).cpu().numpy()
    np.testing.assert_allclose(tsum.cpu().numpy(), want_sum, rtol=1e-4)
    scale = np.abs(want).max(axis=1, keepdims=True) + 1e-30
    assert float((np.abs(got - want) / scale).max()) < 1e-4


def test_correlation_and_forward_statistics(oracle) -> None:
    """Log-returns of the terminal values have correlation rho and per-asset mean/variance of GBM."""
    A, T = 3, 4
    cfg = BasketConfig(n_assets=A, timesteps=T, network_size=256, batches_per_mc_run=256, math="hw")
    rho, v, Tm, r = 0.6, np.array([0.2, 0.3, 0.4]), 1.0, 0.03
    d = np.array([0.0, 0.01, 0.02])
    X0 = np.array([100.0, 50.0, 10.0])
    row = np.concatenate([[100.0, Tm, r, rho], X0, d, v])
    c = torch.from_numpy(np.tile(row, (2, 1))).to(DEV)
    paths = poisoned((2, A, T, cfg.total_paths), torch.float32, DEV)
    basket_targets(c, cfg, paths=paths)
    lr = np.log(paths[0, :, -1, :].double().cpu().numpy() / X0[:, None])
    corr = np.corrcoef(lr)
    for i in range(A):
        for k in range(i):
            assert abs(corr[i, k] - rho) < 0.01, corr
        assert lr[i].std() == pytest.approx(v[i] * np.sqrt(Tm), rel=0.01)
        assert lr[i].mean() == pytest.approx((r - d[i] - 0.5 * v[i] ** 2) * Tm, abs=0.01)
    # different contract ordinals draw different streams
    assert not torch.equal(paths[0], paths[1])


@pytest.mark.parametrize("M", [32, 128])
def test_chunked_launches_match_single_launch(oracle, M) -> None:
    """M = 32 (P = 2048): the split pair; M = 128 (P = 8192): the resident kernel, W = 2."""
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=64, batches_per_mc_run=M, math="portable")
    B = 12
    per = 4 * 16 * int(_lib.lib().smc_path_pitch(cfg.total_paths, 0)) * 4
    big = BasketEngine(cfg, B, device=torch.device(DEV))
    small = BasketEngine(cfg, B, device=torch.device(DEV), path_buffer_bytes=5 * per)
    assert small.chunk == 4 and big.chunk == B
    wg, W = oracle.basket_order(4, 16, 64, M)
    assert big.kernel_name == ("basket_resident_kernel" if wg == 1024 else "basket_kernel+basket_cf_kernel")
    for e in (big, small):
        e.set_position(0, 0)
        e.enqueue_step()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(big.buffers.targets.cpu().numpy(), small.buffers.targets.cpu().numpy())
    c = _contracts(oracle, cfg, B)
    np.testing.assert_array_equal(big.buffers.contracts.cpu().numpy(), c)
    _, _, want = oracle.basket_kernel(c, 4, 16, 64, M, cfg.mc_seed, wg=wg, slices=W)
    np.testing.assert_array_equal(big.buffers.targets.cpu().numpy(), want)


def test_bad_shapes_fail_loudly() -> None:
    cfg = BasketConfig(n_assets=2, timesteps=4, network_size=64, batches_per_mc_run=32)
    c = torch.zeros((2, cfg.dim), dtype=torch.float64, device=DEV)
    t = poisoned((2, 64), torch.complex64, DEV)
    p = poisoned((2, 2, 2048), torch.float32, DEV)
    L = _lib.lib()
    st = L.smc_basket_train_targets(_lib.ptr(c), 2, 9, 4, 64, 32, 7, None, 0, 0, 1, _lib.STORE_TERMINAL,
                                    _lib.ptr(p), 0, 2, None, _lib.ptr(t), None, 0, None)
    assert st == 1
    st = L.smc_basket_train_targets(_lib.ptr(c), 2, 2, 4, 64, 30, 7, None, 0, 0, 1, _lib.STORE_TERMINAL,
                                    _lib.ptr(p), 0, 2, None, _lib.ptr(t), None, 0, None)
    assert st == 2
    assert b"2048" in L.smc_last_error_string()


@pytest.mark.parametrize("M", [16, 64])
def test_pricer_trains_on_baskets_and_matches_oracle_step(oracle, M) -> None:
    """One GbmCVNNPricer step on basket contracts (portable math) vs the oracle targets + torch-cpu step
    (M = 16: the split pair; M = 64: the resident kernel, W = 2)."""
    A, T, N, B = 4, 16, 128, 32
    bcfg = BasketConfig(n_assets=A, timesteps=T, network_size=N, batches_per_mc_run=M, mc_seed=7, math="portable")
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256, mc_seed=7,
                                buffer_size=512, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=bcfg.dim, n_outputs=N, seed=123, dtype=torch.float32)
    cpu_model = copy.deepcopy(model).cpu()
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.warmup_steps = 0
    use_basket_engine(pricer, bcfg)
    res = expect_success(pricer.train(make_training_config(num_batches=1, batch_size=B, learning_rate=1e-2)))

    c = _contracts(oracle, bcfg, B)
    wg, W = oracle.basket_order(A, T, N, M)
    _, _, targets = oracle.basket_kernel(c, A, T, N, M, 7, wg=wg, slices=W)
    x = torch.tensor(c, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert res.final_loss == pytest.approx(ref.loss, rel=1e-4)

    # and several graph-replayed steps stay finite
    pricer.warmup_steps = 2
    res = expect_success(pricer.train(make_training_config(num_batches=5, batch_size=B, learning_rate=1e-2)))
    assert np.isfinite(res.final_loss)


def test_resident_exchange_timeout_is_reported() -> None:
    """basket_resident_kernel with a withheld slice arrival (test hook): the launch completes, the
    contract's targets are NaN, and BasketEngine.check_status raises SMC_ERR_EXCHANGE_TIMEOUT instead of
    training on NaN silently; the next launch with the hook cleared matches a clean launch."""
    cfg = BasketConfig(n_assets=4, timesteps=16, network_size=256, batches_per_mc_run=128, math="portable")
    eng = BasketEngine(cfg, 12, device=torch.device(DEV))
    assert eng.kernel_name == "basket_resident_kernel"
    eng.set_position(0, 0)
    eng.enqueue_step()
    clean = eng.buffers.targets.clone()
    eng.check_status()
    L = _lib.lib()
    _lib.check(L.smc_test_exchange_fault(1, 20000))
    try:
        eng.set_position(0, 0)
        eng.enqueue_step()
        torch.cuda.synchronize()
    finally:
        _lib.check(L.smc_test_exchange_fault(0, 0))
    assert torch.isnan(eng.buffers.targets[0].real).all()
    with pytest.raises(_lib.SmcError) as exc:
        eng.check_status()
    assert exc.value.code == _lib.SMC_ERR_EXCHANGE_TIMEOUT
    eng.set_position(0, 0)
    eng.enqueue_step()
    eng.check_status()
    assert torch.equal(eng.buffers.targets, clean)
