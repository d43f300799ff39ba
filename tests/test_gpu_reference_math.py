"""SMC_MATH_REF on the GPU (rows_ref_kernel + cf_kernel): the reference kernel's own f32 typing
(/root/reference/src/spectralmc/gbm.py:224-257 under Numba: f64 state and step of the f32 normals, f32
stores).  Bit-exact against the oracle's kernel mode with MATH_REF (stored paths, terminal sums, targets;
tests/test_oracle.py pins that mode to the reference arithmetic's stored paths), smc_train_step in this
mode equal to draw + smc_train_targets, and the trainer's math_mode="reference" one step against the
oracle at the C1-like test shape."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from spectralmc_amd import _lib
from spectralmc_amd.sobol_sampler import SobolEngine, draw_device
from tests.helpers import poisoned, poisoned_like
from tests.test_gpu_engine import _contracts, _L, _run_targets

pytestmark = pytest.mark.gpu

DEV = "cuda"

REF_CASES = [  # (B, T, N, M, scheme, normalize, store)
    (9, 16, 256, 16, 0, 1, _lib.STORE_ALL),        # P = 4096: whole chunks
    (7, 16, 128, 4, 0, 1, _lib.STORE_ALL),         # the e2e shape, P = 512: one partial chunk
    (5, 5, 100, 7, 1, 1, _lib.STORE_ALL),          # P = 700, simple Euler, odd T
    (4, 4, 99, 101, 1, 1, _lib.STORE_TERMINAL),    # P = 9999: a lane straddles P, several chunks
    (6, 1, 16, 256, 0, 0, _lib.STORE_ALL),         # T = 1, RAW (the lock-step trainer's T)
    (3, 33, 64, 64, 0, 1, _lib.STORE_TERMINAL),    # T > 16
    (600, 16, 64, 32, 0, 1, _lib.STORE_ALL),       # more contracts than the persistent grid
]


@pytest.mark.parametrize("B,T,N,M,scheme,normalize,store", REF_CASES)
def test_reference_math_matches_oracle(oracle, golden, B, T, N, M, scheme, normalize, store) -> None:
    c = _contracts(oracle, golden, B, seed=31)
    P = N * M
    pitch = int(_L().smc_path_pitch(P, 0))
    assert _L().smc_train_targets_kernel(T, N, P, _lib.DTYPE_F32 | _lib.MATH_REF, pitch, 0) == \
        b"rows_ref_kernel+cf_kernel"
    got, _, paths = _run_targets(c, T, N, M, scheme, normalize, "float32", store, ordinal0=9, with_rowsum=False,
                                 flags=_lib.MATH_REF, pitch=pitch)
    want_paths, want_term, _ = oracle.kernel_paths(c, T, P, 7, 9, scheme | oracle.MATH_REF, want_paths=True)
    kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme | oracle.MATH_REF,
                                  normalize=bool(normalize))
    np.testing.assert_array_equal(got, kt)
    stored = paths.cpu().numpy()
    np.testing.assert_array_equal(stored, want_paths if store == _lib.STORE_ALL else want_term)
    # and the reference semantics (oracle reference mode) at the f32 engine's tolerance
    want = oracle.training_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme, normalize=bool(normalize))
    den = max(float(np.linalg.norm(want)), 1e-30)
    assert float(np.linalg.norm(got - want)) / den < 1e-6


@pytest.mark.parametrize("B,T,N,M,scheme,normalize,store", REF_CASES)
def test_reference_math_on_hw_normals_within_tolerance(oracle, golden, B, T, N, M, scheme, normalize, store) -> None:
    """SMC_MATH_REF | SMC_MATH_HW (math_mode "reference_hw"): the reference typing's f64 step on the
    hardware-transcendental normals.  Not CPU-reproducible (v_log / v_sqrt / v_sin / v_cos, ~1 ulp), so it is held
    to the "hw" mode's bar against the oracle's MATH_REF kernel mode on the same draws: stored paths within 2e-5
    relative (16 steps of ~1-ulp normals), targets within 1e-5 of each contract's row norm, and the reference
    semantics (oracle reference mode) within 1e-5 overall."""
    c = _contracts(oracle, golden, B, seed=31)
    P = N * M
    pitch = int(_L().smc_path_pitch(P, 0))
    flags = _lib.MATH_REF | _lib.MATH_HW
    assert _L().smc_train_targets_kernel(T, N, P, _lib.DTYPE_F32 | flags, pitch, 0) == b"rows_ref_kernel+cf_kernel"
    got, _, paths = _run_targets(c, T, N, M, scheme, normalize, "float32", store, ordinal0=9, with_rowsum=False,
                                 flags=flags, pitch=pitch)
    want_paths, want_term, _ = oracle.kernel_paths(c, T, P, 7, 9, scheme | oracle.MATH_REF, want_paths=True)
    kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme | oracle.MATH_REF,
                                  normalize=bool(normalize))
    assert np.isfinite(got).all()
    stored = paths.cpu().numpy().astype(np.float64)
    want = (want_paths if store == _lib.STORE_ALL else want_term).astype(np.float64)
    if store == _lib.STORE_ALL:
        stored = stored[..., :P]
        want = want[..., :P]
    np.testing.assert_allclose(stored, want, rtol=2e-5, atol=1e-6 * max(1.0, float(np.abs(want).max())))
    row = np.maximum(np.linalg.norm(kt, axis=1), 1e-30)
    assert float((np.linalg.norm(got - kt, axis=1) / row).max()) < 1e-5
    ref = oracle.training_targets(c, T, N, M, seed=7, ordinal0=9, scheme=scheme, normalize=bool(normalize))
    den = max(float(np.linalg.norm(ref)), 1e-30)
    assert float(np.linalg.norm(got - ref)) / den < 1e-5


def test_reference_math_rejects_f64() -> None:
    L = _L()
    c = torch.zeros((1, 6), dtype=torch.float64, device=DEV)
    out = torch.zeros(64, dtype=torch.complex128, device=DEV)
    paths = torch.zeros(4096, dtype=torch.float64, device=DEV)
    for flags in (_lib.MATH_REF, _lib.MATH_REF | _lib.MATH_HW):
        st = L.smc_train_targets(_lib.ptr(c), 1, 4, 16, 4, 7, None, 0, flags, 1, _lib.DTYPE_F64, _lib.STORE_TERMINAL,
                                 _lib.ptr(paths), 128, 1, None, _lib.ptr(out), None, 0, None)
        assert st == _lib.SMC_ERR_INVALID_ARGUMENT


def test_reference_math_train_step_equals_draw_then_targets(golden) -> None:
    """smc_train_step with SMC_MATH_REF (no fused resident launch: Sobol draw, rows_ref_kernel + cf_kernel,
    cursor update) is bit-identical to the separate draw + smc_train_targets over three steps at the C2
    path shape (P = 65,536, T = 16)."""
    L = _L()
    B, T, N, M = 70, 16, 256, 256
    P = N * M
    pitch = int(L.smc_path_pitch(P, 0))
    assert L.smc_train_step_kernel(T, N, M, _lib.DTYPE_F32 | _lib.MATH_REF, pitch) == b"rows_ref_kernel+cf_kernel"
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo = torch.from_numpy(golden["bounds_lower"]).to(DEV)
    hi = torch.from_numpy(golden["bounds_upper"]).to(DEV)
    paths = poisoned((B, T, pitch), torch.float32, DEV)
    scheme = _lib.SCHEME_LOG_EULER | _lib.MATH_REF
    cur_a = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
    cur_b = cur_a.clone()
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, _lib.DTYPE_F32, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    for _ in range(3):
        ca = poisoned((B, 6), torch.float64, DEV)
        fa = poisoned((B, 6), torch.float32, DEV)
        ta = poisoned((B, N), torch.complex64, DEV)
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur_a), 0, B,
                                    _lib.ptr(ca), _lib.ptr(fa), B, T, N, M, 7, scheme, _lib.NORM_NORMALIZE,
                                    _lib.DTYPE_F32, _lib.STORE_ALL, _lib.ptr(paths), pitch, B, _lib.ptr(ta),
                                    _lib.ptr(sync), nsync, None))
        cb = poisoned_like(ca)
        fb = poisoned_like(fa)
        tb = poisoned_like(ta)
        draw_device(tables, 6, cur_b[0:1], 0, B, lo, hi, cb, fb)
        _lib.check(L.smc_train_targets(_lib.ptr(cb), B, T, N, M, 7, _lib.ptr(cur_b[1:2]), 0, scheme,
                                       _lib.NORM_NORMALIZE, _lib.DTYPE_F32, _lib.STORE_ALL, _lib.ptr(paths), pitch,
                                       B, None, _lib.ptr(tb), None, 0, None))
        cur_b.add_(B)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ca.cpu().numpy(), cb.cpu().numpy())
        np.testing.assert_array_equal(ta.cpu().numpy(), tb.cpu().numpy())
        assert cur_a.tolist() == cur_b.tolist()
        assert not sync.view(torch.int32).any()


@pytest.mark.parametrize("math", ["reference", "reference_hw"])
def test_trainer_reference_math_one_step_matches_oracle(oracle, math) -> None:
    """GbmCVNNPricer(math_mode="reference" / "reference_hw"): the step's loss is the oracle step's on the oracle's
    MATH_REF kernel-mode targets within 1e-4 rel."""
    import copy

    from spectralmc_amd.gbm_trainer import GbmCVNNPricer
    from tests.helpers import (
        expect_success,
        make_black_scholes_config,
        make_domain_bounds,
        make_gbm_cvnn_config,
        make_simulation_params,
        make_test_cvnn,
        make_training_config,
    )

    B, T, N, M = 32, 16, 128, 4
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                mc_seed=7, buffer_size=512)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.math_mode = math
    pricer.warmup_steps = 0
    cpu_model = copy.deepcopy(model).cpu()
    res = expect_success(pricer.train(make_training_config(num_batches=1, batch_size=B, learning_rate=1e-2)))
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    kt, _ = oracle.kernel_targets(contracts, T, N, M, seed=7, ordinal0=0, scheme=oracle.MATH_REF)
    x = torch.tensor(contracts, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, x, torch.zeros_like(x), torch.from_numpy(kt),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert res.final_loss == pytest.approx(ref.loss, rel=1e-4)


def test_reference_math_chunked_launches_equal_one_launch(oracle, golden) -> None:
    """smc_train_targets in reference math over chunked launches (three chunks, a ragged last one) gives the
    one-launch targets bit for bit."""
    B, T, N, M = 600, 5, 64, 32
    c = _contracts(oracle, golden, B, seed=7)
    pitch = int(_L().smc_path_pitch(N * M, 0))
    one, _, _ = _run_targets(c, T, N, M, 1, 1, "float32", _lib.STORE_TERMINAL, ordinal0=3, with_rowsum=False,
                             flags=_lib.MATH_REF, pitch=pitch)
    chunked, _, _ = _run_targets(c, T, N, M, 1, 1, "float32", _lib.STORE_TERMINAL, ordinal0=3, with_rowsum=False,
                                 flags=_lib.MATH_REF, pitch=pitch, chunk=250)
    np.testing.assert_array_equal(chunked, one)
