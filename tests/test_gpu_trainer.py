"""GbmCVNNPricer on the HIP path vs the oracle step, plus the reference trainer's determinism
contracts (tests/test_gbm_trainer.py:170-320): lock-step bit-exactness, snapshot/resume,
Adam state round trip, predict_price."""

from __future__ import annotations

import copy
import math

import numpy as np
import pytest
import torch

from spectralmc.gbm import BlackScholes
from spectralmc.gbm_trainer import GbmCVNNPricer
from spectralmc.models.numerical import Precision
from spectralmc.result import Failure
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

T, N, M = 16, 128, 4


def _sim(dtype: Precision = Precision.float32, mc_seed: int = 7):
    return make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                  mc_seed=mc_seed, buffer_size=512, dtype=dtype)


def _pricer(seed: int = 123, dtype: torch.dtype = torch.float32, warmup: int | None = None, **cfg_kw):
    prec = Precision.float32 if dtype == torch.float32 else Precision.float64
    sp = _sim(prec)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=seed, dtype=dtype)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds(), **cfg_kw)
    p = expect_success(GbmCVNNPricer.create(cfg))
    if warmup is not None:
        p.warmup_steps = warmup
    return p, model


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_one_step_matches_oracle(oracle, dtype) -> None:
    B = 32
    pricer, model = _pricer(dtype=dtype, warmup=0)
    cpu_model = copy.deepcopy(model).cpu()
    res = expect_success(pricer.train(make_training_config(num_batches=1, batch_size=B, learning_rate=1e-2)))

    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    sdt = "float32" if dtype == torch.float32 else "float64"
    targets = oracle.training_targets(contracts, T, N, M, seed=7, ordinal0=0, dtype=sdt)
    adam = torch.optim.Adam(cpu_model.parameters(), lr=1e-2)
    x = torch.tensor(contracts, dtype=dtype)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets), adam)

    assert res.final_loss == pytest.approx(ref.loss, rel=1e-4)          # spectral-loss match, 1e-4 rel
    assert res.final_grad_norm == pytest.approx(ref.grad_norm, rel=1e-3)
    for (name, pg), pc in zip(model.named_parameters(), cpu_model.parameters(), strict=True):
        a, b = pg.detach().cpu().double(), pc.detach().double()
        rel = float((a - b).norm() / max(float(b.norm()), 1e-12))
        assert rel < 1e-4, (name, rel)


def test_portable_math_trainer_loss_within_tolerance(oracle) -> None:
    """The CPU-reproducible math mode through the whole trainer (default is "hw")."""
    B = 32
    pricer, model = _pricer(warmup=0)
    assert pricer.math_mode == "hw"
    pricer.math_mode = "portable"
    res = expect_success(pricer.train(make_training_config(num_batches=1, batch_size=B, learning_rate=1e-2)))
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    targets = oracle.training_targets(contracts, T, N, M, seed=7)
    cpu_model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device="cpu")
    x = torch.tensor(contracts, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert res.final_loss == pytest.approx(ref.loss, rel=1e-4)


def test_short_steps_run_eager_and_long_steps_capture(monkeypatch) -> None:
    """graph_min_path_steps (the product default, 2^27 path-steps): a step below it stays eager after the
    warm-up steps, one at or above it is captured (here by lowering the threshold to the step's own size)."""
    from spectralmc_amd.gbm_trainer import GRAPH_MIN_PATH_STEPS

    monkeypatch.setattr(GbmCVNNPricer, "graph_min_path_steps", GRAPH_MIN_PATH_STEPS)
    B = 16
    for threshold, captured in ((GRAPH_MIN_PATH_STEPS, False), (B * N * M * T, True)):
        p, _ = _pricer(warmup=1)
        p.graph_min_path_steps = threshold
        session = expect_success(p.open_session(make_training_config(num_batches=3, batch_size=B)))
        for _ in range(3):
            expect_success(session.step())
        assert session.program.captured is captured
        session.close()


def test_graph_replay_matches_eager() -> None:
    eager, m_e = _pricer(warmup=0)
    graph, m_g = _pricer(warmup=1)
    cfg = make_training_config(num_batches=5, batch_size=16)
    r_e = expect_success(eager.train(cfg))
    r_g = expect_success(graph.train(cfg))
    assert max_param_diff(m_e, m_g) == 0.0
    assert r_e.final_loss == r_g.final_loss


PRECISIONS = [torch.float32, torch.float64]  # reference tests/helpers/fixtures.py:19-107


@pytest.mark.parametrize("dtype", PRECISIONS)
def test_lockstep_training_is_bit_exact(dtype) -> None:
    """Reference tests/test_gbm_trainer.py:182-193 (both precisions)."""
    a, ma = _pricer(dtype=dtype)
    b, mb = _pricer(dtype=dtype)
    assert max_param_diff(ma, mb) == 0.0
    cfg = make_training_config(num_batches=4, batch_size=24)
    expect_success(a.train(cfg))
    expect_success(b.train(cfg))
    assert max_param_diff(ma, mb) == 0.0
    assert all(p.dtype == dtype for p in ma.parameters())


def _lockstep_pricer(dtype: torch.dtype, seed: int = 43):
    """The reference's lock-step trainer (tests/test_gbm_trainer.py:122-160): T = 1, N = 16, M = 4096,
    LOG_EULER + RAW, mc_seed = seed, CVNN 6 -> 32 (modReLU) -> 16."""
    from spectralmc.gbm import ForwardNormalization, PathScheme

    prec = Precision.float32 if dtype == torch.float32 else Precision.float64
    sp = make_simulation_params(timesteps=1, network_size=16, batches_per_mc_run=2 ** 12, threads_per_block=256,
                                mc_seed=seed, buffer_size=1, dtype=prec)
    bs = make_black_scholes_config(sim_params=sp, path_scheme=PathScheme.LOG_EULER,
                                   normalization=ForwardNormalization.RAW)
    model = make_test_cvnn(n_inputs=6, n_outputs=16, seed=seed, dtype=dtype)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=bs, domain_bounds=make_domain_bounds())
    return expect_success(GbmCVNNPricer.create(cfg)), model


@pytest.mark.parametrize("dtype", PRECISIONS)
def test_reference_lockstep_contract(oracle, dtype) -> None:
    """Reference tests/test_gbm_trainer.py:182-193 at its own shape: two pricers built alike train
    batches (2, 3, 1) of 8 contracts in lock step, bit-identical after every call (f32: the resident
    kernel's rolled row loop; f64: rows_kernel + cf_kernel); plus one step against the oracle
    (reference-mode targets: RAW, T = 1, odd-T tail draw; torch-cpu _torch_step)."""
    first, m1 = _lockstep_pricer(dtype)
    second, m2 = _lockstep_pricer(dtype)
    assert max_param_diff(m1, m2) == 0.0
    for batches in (2, 3, 1):
        cfg = make_training_config(num_batches=batches, batch_size=8, learning_rate=1.0e-2)
        expect_success(first.train(cfg))
        expect_success(second.train(cfg))
        assert max_param_diff(m1, m2) == 0.0

    one, m_one = _lockstep_pricer(dtype)
    cpu_model = copy.deepcopy(m_one).cpu()
    res = expect_success(one.train(make_training_config(num_batches=1, batch_size=8, learning_rate=1.0e-2)))
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(43, 0, 8, lo, hi)
    sdt = "float32" if dtype == torch.float32 else "float64"
    targets = oracle.training_targets(contracts, 1, 16, 4096, seed=43, ordinal0=0, normalize=False, dtype=sdt)
    x = torch.tensor(contracts, dtype=dtype)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1.0e-2))
    tol = 1e-4 if dtype == torch.float32 else 1e-10
    assert res.final_loss == pytest.approx(ref.loss, rel=tol)
    for pg, pc in zip(m_one.parameters(), cpu_model.parameters(), strict=True):
        a, b = pg.detach().cpu().double(), pc.detach().double()
        assert float((a - b).norm() / max(float(b.norm()), 1e-12)) < tol


@pytest.mark.parametrize("dtype", PRECISIONS)
def test_snapshot_restore_continues_identically(dtype) -> None:
    """Reference tests/test_gbm_trainer.py:201-263 (both precisions)."""
    cfg2 = make_training_config(num_batches=2, batch_size=16)
    straight, m_s = _pricer(dtype=dtype)
    expect_success(straight.train(make_training_config(num_batches=4, batch_size=16)))

    first, m_f = _pricer(dtype=dtype)
    r1 = expect_success(first.train(cfg2))
    snap = r1.updated_config
    assert snap.global_step == 2 and snap.sobol_skip == 32
    assert snap.cfg.sim_params.skip == 32  # normal matrices served (async_normals.py:400-413)
    resumed = expect_success(GbmCVNNPricer.create(snap))
    expect_success(resumed.train(cfg2))
    assert max_param_diff(m_s, m_f) == 0.0


@pytest.mark.parametrize("dtype", PRECISIONS)
def test_adam_state_round_trip(dtype) -> None:
    """Reference tests/test_gbm_trainer.py:271-294 (both precisions)."""
    p, _ = _pricer(dtype=dtype)
    r = expect_success(p.train(make_training_config(num_batches=2, batch_size=8)))
    st = r.updated_config.optimizer_state
    assert st is not None and len(st.param_states) == len(list(r.updated_config.cvnn.parameters()))
    back = expect_success(st.to_torch())
    again = expect_success(type(st).from_torch(back))
    for pid, ps in st.param_states.items():
        assert ps.step == 2
        a = expect_success(ps.exp_avg.to_torch())
        assert a.dtype == dtype
        assert torch.equal(a, expect_success(again.param_states[pid].exp_avg.to_torch()))
        assert torch.equal(expect_success(ps.exp_avg_sq.to_torch()),
                           expect_success(again.param_states[pid].exp_avg_sq.to_torch()))


def test_multi_chunk_equals_single_chunk(monkeypatch) -> None:
    import spectralmc_amd.engine as eng

    a, ma = _pricer(warmup=0)
    expect_success(a.train(make_training_config(num_batches=2, batch_size=20)))
    from spectralmc_amd import _lib

    pitch = int(_lib.lib().smc_path_pitch(N * M, _lib.DTYPE_F32))
    monkeypatch.setattr(eng, "DEFAULT_PATH_BUFFER_BYTES", 3 * T * pitch * 4)  # 3 contracts per launch
    b, mb = _pricer(warmup=0)
    sess = expect_success(b.open_session(make_training_config(num_batches=2, batch_size=20)))
    assert sess.engine.chunk == 3  # 7 equal launches of <= 3 contracts
    sess.close()
    expect_success(b.train(make_training_config(num_batches=2, batch_size=20)))
    assert max_param_diff(ma, mb) == 0.0


def test_terminal_only_store_mode_same_result() -> None:
    a, ma = _pricer()
    b, mb = _pricer()
    b.store_paths = False
    cfg = make_training_config(num_batches=3, batch_size=16)
    expect_success(a.train(cfg))
    expect_success(b.train(cfg))
    assert max_param_diff(ma, mb) == 0.0


def test_predict_price_finite_and_parity() -> None:
    p, _ = _pricer()
    expect_success(p.train(make_training_config(num_batches=3, batch_size=16)))
    contracts = [BlackScholes.Inputs(X0=100.0, K=95.0, T=0.5, r=0.03, d=0.01, v=0.25),
                 BlackScholes.Inputs(X0=120.0, K=105.0, T=1.0, r=0.02, d=0.0, v=0.30)]
    out = expect_success(p.predict_price(contracts))
    assert len(out) == 2
    for r, c in zip(out, contracts):
        vals = r.model_dump().values()
        assert all(math.isfinite(v) for v in vals)
        fwd = c.X0 * math.exp((c.r - c.d) * c.T)
        assert r.call_price - r.put_price == pytest.approx(fwd - c.K * math.exp(-c.r * c.T), rel=1e-9, abs=1e-9)
    assert expect_success(p.predict_price([])) == []


@pytest.mark.parametrize("dtype", PRECISIONS)
def test_predict_price_matches_cpu_ifft_mean(dtype) -> None:
    """predict_price (reference gbm_trainer.py:1709-1767): CVNN spectrum -> ifft(dim=1).mean(1)
    -> put = Re; call by put-call parity.  Compared with a torch-cpu copy of the same trained
    weights running the reference's own arithmetic (forward, ifft, mean) in float64."""
    p, model = _pricer(dtype=dtype)
    expect_success(p.train(make_training_config(num_batches=3, batch_size=16)))
    rng = np.random.default_rng(5)
    contracts = [BlackScholes.Inputs(X0=float(rng.uniform(50, 150)), K=float(rng.uniform(50, 150)),
                                     T=float(rng.uniform(0.1, 3.0)), r=float(rng.uniform(-0.05, 0.08)),
                                     d=float(rng.uniform(0.0, 0.05)), v=float(rng.uniform(0.05, 0.8)))
                 for _ in range(24)]
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # |Im| of an untrained spectrum's mean IFFT
        got = expect_success(p.predict_price(contracts))
    cpu = copy.deepcopy(model).cpu().double().eval()
    x = torch.tensor([[c.X0, c.K, c.T, c.r, c.d, c.v] for c in contracts], dtype=torch.float64)
    with torch.no_grad():
        pr, pi = cpu(x, torch.zeros_like(x))
        coeff = torch.fft.ifft(torch.complex(pr, pi), dim=1).mean(dim=1)
    tol = 1e-5 if dtype == torch.float32 else 1e-10
    for r, c, k in zip(got, contracts, coeff, strict=True):
        scale = max(abs(float(k.real)), float(pr.abs().max()) / pr.shape[1])
        assert r.put_price == pytest.approx(float(k.real), rel=0, abs=tol * scale)
        disc, fwd = math.exp(-c.r * c.T), c.X0 * math.exp((c.r - c.d) * c.T)
        assert r.call_price == pytest.approx(float(k.real) + fwd - c.K * disc, rel=0, abs=tol * scale + 1e-9 * fwd)
        assert r.underlying == pytest.approx(fwd, rel=1e-12)
        assert r.put_price_intrinsic == pytest.approx(disc * max(c.K - fwd, 0.0), rel=1e-12, abs=1e-12)


def test_host_validated_path_logs_and_commits(tmp_path) -> None:
    """A domain whose lower bounds admit invalid contracts (X0 lower = 0) takes the host-validated
    loop: it calls the logger every step with the step's wall time, commits at the interval like
    the device loop (reference _run_batch), trains the same contracts and targets as the device
    loop, and stops with SequenceExhausted past 2^30 Sobol points."""
    import asyncio

    from spectralmc_amd.errors.sampler import SequenceExhausted
    from spectralmc_amd.gbm_trainer import IntervalCommit
    from spectralmc_amd.sobol_sampler import MAX_POINTS
    from spectralmc_amd.storage import AsyncBlockchainModelStore

    sp = _sim()
    bounds = make_domain_bounds(x0=(0.0, 10_000.0))

    def make(seed: int = 123, sobol_skip: int = 0):
        m = make_test_cvnn(n_inputs=6, n_outputs=N, seed=seed, dtype=torch.float32)
        cfg = make_gbm_cvnn_config(m, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                   domain_bounds=bounds, sobol_skip=sobol_skip)
        return expect_success(GbmCVNNPricer.create(cfg)), m

    store = AsyncBlockchainModelStore(tmp_path / "store")
    checked, m_c = make()
    logged = []
    res = expect_success(checked.train(make_training_config(num_batches=3, batch_size=16), logger=logged.append,
                                       blockchain_store=store, commit_plan=IntervalCommit(interval=1)))
    assert [m.step for m in logged] == [1, 2, 3]
    assert all(math.isfinite(m.batch_time) and m.batch_time > 0 for m in logged)
    assert logged[-1].loss == res.final_loss
    versions = asyncio.run(store.list_versions())
    assert len(versions) == 3
    assert res.updated_config.global_step == 3 and res.updated_config.sobol_skip == 48
    # the same three steps on the device loop (positive bounds give the same Sobol rows here)
    dev_bounds = make_domain_bounds(x0=(1e-300, 10_000.0))
    m_d = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32)
    dcfg = make_gbm_cvnn_config(m_d, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                domain_bounds=dev_bounds)
    dev = expect_success(GbmCVNNPricer.create(dcfg))
    dev.fused_network = False  # the checked loop runs the torch _torch_step
    r_d = expect_success(dev.train(make_training_config(num_batches=3, batch_size=16)))
    assert r_d.final_loss == pytest.approx(res.final_loss, rel=1e-5)
    late, _ = make(sobol_skip=MAX_POINTS - 20)
    out = late.train(make_training_config(num_batches=2, batch_size=16))
    assert isinstance(out, Failure) and isinstance(out.error.error, SequenceExhausted)


def test_c1_training_step_pair_matches_reference_fixture() -> None:
    """Two C1 training steps on the GPU (B = 64, T = 16, N = 256, M = 4, mc_seed 7, CVNN
    6 -> 32 modReLU -> 256 seed 123, lr 1e-2) against the loss / grad norm / weights the
    reference's own gbm.py + cvnn_factory + _torch_step produced (tests/golden/gbm_golden.npz)."""
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with np.load(os.path.join(root, "tests", "golden", "gbm_golden.npz"), allow_pickle=False) as data:
        g = {k: data[k] for k in data.files}
    sp = make_simulation_params(timesteps=16, network_size=256, batches_per_mc_run=4, mc_seed=7, buffer_size=1,
                                dtype=Precision.float32)
    for steps in (1, 2):
        model = make_test_cvnn(n_inputs=6, n_outputs=256, seed=123, dtype=torch.float32)
        for k, v in model.state_dict().items():
            np.testing.assert_array_equal(v.cpu().numpy(), g[f"step_init__{k}"])
        cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                   domain_bounds=make_domain_bounds())
        pricer = expect_success(GbmCVNNPricer.create(cfg))
        res = expect_success(pricer.train(make_training_config(num_batches=steps, batch_size=64, learning_rate=1e-2)))
        s = steps - 1
        assert res.final_loss == pytest.approx(float(g[f"step{s}_loss"]), rel=1e-4)       # north-star 1e-4
        assert res.final_grad_norm == pytest.approx(float(g[f"step{s}_gradnorm"]), rel=1e-3)
        for k, v in model.state_dict().items():
            ref = g[f"step{s}_after__{k}"]
            diff = np.abs(v.detach().cpu().numpy() - ref)
            # 2 Adam steps of lr 1e-2 (|update| ~ lr sign(g)): equal to f32 noise except where a
            # gradient element is ~0 and may take either sign
            assert int((diff > 2e-4).sum()) <= max(2, diff.size // 1000), k


def test_gbm_engine_price_vs_black(oracle) -> None:
    """BlackScholes.price_to_host against the closed form (reference tests/test_gbm.py:103-139)."""
    sp = make_simulation_params(timesteps=1, network_size=256, batches_per_mc_run=1024, mc_seed=31,
                                buffer_size=1, dtype=Precision.float32)
    bs = BlackScholes(make_black_scholes_config(sim_params=sp))
    rng = np.random.default_rng(31)
    errs = []
    for _ in range(16):
        c = BlackScholes.Inputs(X0=float(rng.uniform(50, 150)), K=float(rng.uniform(50, 150)),
                                T=float(rng.uniform(0.1, 2.0)), r=float(rng.uniform(0.0, 0.08)),
                                d=float(rng.uniform(0.0, 0.04)), v=float(rng.uniform(0.1, 0.6)))
        host = expect_success(bs.price_to_host(c))
        ref = oracle.black_put(c.X0, c.K, c.T, c.r, c.d, c.v)
        if ref > 1.0:
            errs.append((host.put_price - ref) / ref)
    rmspe = float(np.sqrt(np.mean(np.square(errs))))
    assert rmspe < 0.02
    snap = expect_success(bs.snapshot())
    assert snap.sim_params.skip == 16


def test_normalized_paths_hit_forwards() -> None:
    sp = make_simulation_params(timesteps=8, network_size=64, batches_per_mc_run=64, mc_seed=5, buffer_size=1)
    bs = BlackScholes(make_black_scholes_config(sim_params=sp))
    c = BlackScholes.Inputs(X0=80.0, K=90.0, T=1.5, r=0.04, d=0.01, v=0.35)
    sr = expect_success(bs._simulate(c))
    means = sr.sims.double().mean(dim=1)
    torch.testing.assert_close(means, sr.forwards.double(), rtol=2e-6, atol=0)


def test_overlapped_mc_matches_sequential() -> None:
    """MC part of step s+1 on its own stream beside step s's network part == one stream."""
    seq, m_s = _pricer()
    seq.overlap_mc = False
    ovl, m_o = _pricer()
    assert ovl.overlap_mc
    cfg = make_training_config(num_batches=6, batch_size=16)
    r_s = expect_success(seq.train(cfg))
    r_o = expect_success(ovl.train(cfg))
    assert max_param_diff(m_s, m_o) == 0.0
    assert r_s.final_loss == r_o.final_loss and r_s.final_grad_norm == r_o.final_grad_norm


def test_overlapped_rows_network_matches_sequential() -> None:
    """f64 at P = 2048 (rows_kernel + cf_kernel): step s's network part beside step s+1's rows launch
    (pricer.overlap_rows = True, f64's default) == the one-stream step, bit for bit."""
    def mk(overlap_rows: bool):
        sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=16, threads_per_block=256,
                                    mc_seed=7, buffer_size=512, dtype=Precision.float64)
        model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float64)
        cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                   domain_bounds=make_domain_bounds())
        p = expect_success(GbmCVNNPricer.create(cfg))
        p.overlap_rows = overlap_rows
        return p, model

    seq, m_s = mk(False)
    ovl, m_o = mk(True)
    cfg = make_training_config(num_batches=6, batch_size=24)
    s = expect_success(ovl.open_session(cfg))
    assert s.engine.kernel_name.startswith("rows_kernel") and s.stream is not s.mc_stream
    s.close()
    s = expect_success(seq.open_session(cfg))
    assert s.stream is s.mc_stream
    s.close()
    r_s = expect_success(seq.train(cfg))
    r_o = expect_success(ovl.train(cfg))
    assert max_param_diff(m_s, m_o) == 0.0
    assert r_s.final_loss == r_o.final_loss and r_s.final_grad_norm == r_o.final_grad_norm


def test_session_step_without_prefetch_then_close() -> None:
    """A session driven step by step (prefetch on every step, one unused) ends consistently."""
    p, m = _pricer()
    ref, m_r = _pricer()
    expect_success(ref.train(make_training_config(num_batches=3, batch_size=16)))
    sess = expect_success(p.open_session(make_training_config(num_batches=3, batch_size=16)))
    for _ in range(3):
        expect_success(sess.step())
    st = sess.close()
    assert st.global_step == 3 and st.sobol_skip == 48
    assert max_param_diff(m, m_r) == 0.0


def test_fused_network_matches_torch_modules() -> None:
    """HIP network step (csrc/cvnn.hip) vs the torch-ROCm modules + torch Adam, 3 steps."""
    fused, m_f = _pricer()
    ref, m_r = _pricer()
    ref.fused_network = False
    cfg = make_training_config(num_batches=3, batch_size=32)
    r_f = expect_success(fused.train(cfg))
    r_r = expect_success(ref.train(cfg))
    assert r_f.final_loss == pytest.approx(r_r.final_loss, rel=1e-4)
    assert r_f.final_grad_norm == pytest.approx(r_r.final_grad_norm, rel=1e-3)
    assert max_param_diff(m_f, m_r) < 3 * 1e-2 * 1e-2  # well inside one Adam step (lr = 1e-2)
    st_f = r_f.updated_config.optimizer_state
    st_r = r_r.updated_config.optimizer_state
    assert st_f.param_states.keys() == st_r.param_states.keys()
    for pid in st_f.param_states:
        a = expect_success(st_f.param_states[pid].exp_avg.to_torch())
        b = expect_success(st_r.param_states[pid].exp_avg.to_torch())
        assert st_f.param_states[pid].step == st_r.param_states[pid].step == 3
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3 * float(b.abs().max()) + 1e-12)


def test_fused_network_is_used_and_deterministic() -> None:
    a, ma = _pricer()
    b, mb = _pricer()
    cfg = make_training_config(num_batches=4, batch_size=40)  # ragged last row block
    sess = expect_success(a.open_session(cfg))
    assert sess.program.fused is not None and sess.program.fused.blocks >= 1
    for i in range(4):
        expect_success(sess.step(prefetch_next=i < 3))
    sess.close()
    expect_success(b.train(cfg))
    assert max_param_diff(ma, mb) == 0.0


def test_fused_network_wide_output_matches_torch_modules() -> None:
    """N = 1024 outputs (C3 width): 2-row blocks, ragged last block, vs the torch modules."""
    def make(fused: bool):
        sp = make_simulation_params(timesteps=4, network_size=1024, batches_per_mc_run=2, mc_seed=3,
                                    buffer_size=1, dtype=Precision.float32)
        m = make_test_cvnn(n_inputs=6, n_outputs=1024, seed=17, dtype=torch.float32, hidden_layers=2)
        cfg = make_gbm_cvnn_config(m, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                   domain_bounds=make_domain_bounds())
        p = expect_success(GbmCVNNPricer.create(cfg))
        p.fused_network = fused
        return p, m

    a, ma = make(True)
    b, mb = make(False)
    cfg = make_training_config(num_batches=2, batch_size=21)
    ra = expect_success(a.train(cfg))
    rb = expect_success(b.train(cfg))
    assert ra.final_loss == pytest.approx(rb.final_loss, rel=1e-4)
    assert ra.final_grad_norm == pytest.approx(rb.final_grad_norm, rel=1e-3)
    assert max_param_diff(ma, mb) < 3e-4


def test_batchnorm_residual_model_trains_on_torch_path(oracle) -> None:
    """Architectures outside the fused kernels (batch norm, residual) keep the torch-ROCm
    network path and still match the oracle's torch-cpu step."""
    from spectralmc_amd.cvnn_factory import (ActivationCfg, ActivationKind, CovBNCfg, ExplicitWidth, LinearCfg,
                                             ResidualCfg, SequentialCfg, build_cvnn_config, build_model)
    from spectralmc_amd.models.torch import FullPrecisionDType

    layers = [LinearCfg(width=ExplicitWidth(value=16), activation=ActivationCfg(kind=ActivationKind.MOD_RELU)),
              CovBNCfg(),
              ResidualCfg(body=SequentialCfg(layers=[LinearCfg(width=ExplicitWidth(value=16),
                                                               activation=ActivationCfg(kind=ActivationKind.Z_RELU))])),
              LinearCfg(width=ExplicitWidth(value=N))]
    cfg = expect_success(build_cvnn_config(dtype=FullPrecisionDType.float32, layers=layers, seed=5))
    model = expect_success(build_model(n_inputs=6, n_outputs=N, cfg=cfg))
    cpu_model = copy.deepcopy(model)
    model = model.to("cuda")
    sp = _sim()
    pcfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(pcfg))
    pricer.warmup_steps = 0
    sess = expect_success(pricer.open_session(make_training_config(num_batches=1, batch_size=16)))
    assert sess.program.fused is None
    sess.close()
    res = expect_success(pricer.train(make_training_config(num_batches=1, batch_size=16, learning_rate=1e-2)))
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, 16, lo, hi)
    targets = oracle.training_targets(contracts, T, N, M, seed=7)
    x = torch.tensor(contracts, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert res.final_loss == pytest.approx(ref.loss, rel=1e-4)


@pytest.mark.parametrize("lanes", [2, 4])
def test_mc_lanes_match_one_stream(lanes: int) -> None:
    """MC lanes (consecutive path launches on alternating streams, each with its own cursor, sync area
    and scratch; engine.py) give bit-identical training to the sequential one-stream program, eager
    and graph-replayed, on a shape the resident kernel takes (P = 4096, N | 4096)."""
    sp = make_simulation_params(timesteps=16, network_size=256, batches_per_mc_run=16, threads_per_block=256,
                                mc_seed=7, buffer_size=512, dtype=Precision.float32)

    def pricer(overlap: bool, lanes: int):
        model = make_test_cvnn(n_inputs=6, n_outputs=256, seed=5, dtype=torch.float32)
        cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                                   domain_bounds=make_domain_bounds())
        p = expect_success(GbmCVNNPricer.create(cfg))
        p.overlap_mc, p.mc_lanes, p.math_mode = overlap, lanes, "hw"
        p.mc_lanes_short = lanes  # (a short launch: the policy would run it on one lane)
        return p, model

    cfg = make_training_config(num_batches=9, batch_size=96)
    seq, m_s = pricer(False, 1)
    r_s = expect_success(seq.train(cfg))
    lan, m_l = pricer(True, lanes)
    sess = expect_success(lan.open_session(cfg))
    assert sess.engine.lanes == lanes and len(sess.mc_streams) == lanes
    for _ in range(9):
        expect_success(sess.step())
    st = sess.close()
    assert st.global_step == 9 and st.sobol_skip == 9 * 96
    assert max_param_diff(m_s, m_l) == 0.0
    assert st.loss == r_s.final_loss and st.grad_norm == r_s.final_grad_norm
    for sync in sess.engine._syncs:  # every launch leaves its lane's counters zeroed
        assert int(sync.count_nonzero()) == 0
    # lanes interleave the Sobol stream: after 9 steps + 1 prefetched (10 launches), lane k has run
    # every lanes-th step and its cursor is the position of its next one
    cur = sess.engine.cursors.cpu().tolist()
    launched = [(10 - k + lanes - 1) // lanes for k in range(lanes)]
    for k in range(lanes):
        assert cur[k][0] == (k + lanes * launched[k]) * 96 and cur[k][1] == cur[k][0]
    with pytest.raises(RuntimeError):
        sess.read_metrics()  # closed sessions refuse to synchronise (streams released)


def test_mc_lanes_must_divide_the_step_slots() -> None:
    """A lane's cursor assumes it runs every lanes-th step, and the step slots cycle mod 4: lanes = 3
    would draw other steps' contracts, so the session refuses it."""
    sp = _sim()
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=5, dtype=torch.float32)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    p = expect_success(GbmCVNNPricer.create(cfg))
    p.mc_lanes = 3
    res = p.open_session(make_training_config(num_batches=2, batch_size=16))
    assert isinstance(res, Failure) and "mc_lanes" in res.error.message


@pytest.mark.parametrize("field", ["mc_lanes", "mc_lanes_long", "mc_lanes_short"])
def test_lane_counts_that_do_not_divide_the_slots_are_rejected(field) -> None:
    """Both lane settings are validated when the session opens (mc_lanes_long was checked only by
    an assert inside the step program)."""
    from spectralmc.errors.trainer import InvalidTrainerConfig

    p, _ = _pricer()
    setattr(p, field, 3)
    res = p.open_session(make_training_config(num_batches=1, batch_size=8))
    assert isinstance(res, Failure) and isinstance(res.error, InvalidTrainerConfig)
    assert field in res.error.message
