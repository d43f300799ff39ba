"""HIP path vs numbers the REFERENCE CODE produced (tests/golden/gbm_golden.npz, see
tests/test_reference_fixtures.py), and the exact instantiations bench.py times.

* Every fixture case through ``smc_train_targets`` in both math modes: hardware transcendentals
  (the training default) within 1e-5 per contract, portable math bit-exact with the kernel-mode
  oracle and within 5e-6 of the reference.
* C2 bench shape (T = 16, N = M = 256, P = 65,536, STORE_ALL | MATH_HW, padded pitch, no row-sum
  buffer -> the straight-line 16-row block with full 2048-path chunks) over whole rounds of
  resident workgroups, and the C3 per-contract shape (N = 1024, P = 262,144).
* The C2 network (6 -> 32 -> 32 -> 256) fused step at B = 4096 against the oracle's torch-cpu
  ``_torch_step`` (gbm_trainer.py:819-835).
"""

from __future__ import annotations

import copy
import os

import numpy as np
import pytest
import torch

from spectralmc_amd import _lib
from tests.helpers import poisoned
from tests.test_reference_fixtures import CASE_NAMES, per_contract_rel, unpack

pytestmark = pytest.mark.gpu

DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gbm_golden() -> dict[str, np.ndarray]:
    with np.load(os.path.join(ROOT, "tests", "golden", "gbm_golden.npz"), allow_pickle=False) as data:
        return {k: data[k] for k in data.files}


def train_targets(contracts: np.ndarray, m: dict, *, hw: bool, padded: bool = True, seed: int | None = None,
                  ordinal0: int | None = None, ref: bool = False) -> np.ndarray:
    """smc_train_targets as the trainer calls it: STORE_ALL, no row-sum buffer (terminal sum on
    chip), padded scratch pitch, one launch."""
    B = contracts.shape[0]
    T, N, M = m["T"], m["N"], m["M"]
    P = N * M
    f32 = m["dtype"] == "float32"
    dcode = _lib.DTYPE_F32 if f32 else _lib.DTYPE_F64
    # (reference math: room for the terminal sum after column P even where P is an odd multiple of 4 KiB)
    pitch = int(_lib.lib().smc_path_pitch(P + (4 if ref else 0), dcode)) if padded else P
    paths = poisoned((B, T, pitch), torch.float32 if f32 else torch.float64, DEV)
    tg = poisoned((B, N), torch.complex64 if f32 else torch.complex128, DEV)
    cd = torch.from_numpy(np.ascontiguousarray(contracts)).to(DEV)
    scheme = m["scheme"] | (_lib.MATH_HW if hw else 0) | (_lib.MATH_REF if ref else 0)
    _lib.check(_lib.lib().smc_train_targets(
        _lib.ptr(cd), B, T, N, M, m["seed"] if seed is None else seed, None,
        m["ordinal0"] if ordinal0 is None else ordinal0, scheme, _lib.NORM_NORMALIZE if m["normalize"] else
        _lib.NORM_RAW, dcode, _lib.STORE_ALL, _lib.ptr(paths), pitch, B, None, _lib.ptr(tg), None, 0, None))
    torch.cuda.synchronize()
    return tg.cpu().numpy()


@pytest.mark.parametrize("name", CASE_NAMES)
def test_hw_math_targets_match_reference_fixture(gbm_golden, name) -> None:
    contracts, want, m = unpack(gbm_golden, name)
    got = train_targets(contracts, m, hw=True)
    tol = 1e-5 if m["dtype"] == "float32" else 1e-10  # f64 has no hardware mode: OCML vs libm
    assert per_contract_rel(got, want).max() < tol


@pytest.mark.parametrize("name", CASE_NAMES)
def test_portable_math_targets_bit_exact_and_match_reference(oracle, gbm_golden, name) -> None:
    contracts, want, m = unpack(gbm_golden, name)
    got = train_targets(contracts, m, hw=False, padded=name != "c1")
    if m["dtype"] == "float32":
        kt, _ = oracle.kernel_targets(contracts, m["T"], m["N"], m["M"], seed=m["seed"], ordinal0=m["ordinal0"],
                                      scheme=m["scheme"], normalize=m["normalize"],
                                      wg=oracle.engine_wg(m["T"], m["N"], m["N"] * m["M"], normalize=m["normalize"]))
        np.testing.assert_array_equal(got, kt)
        assert per_contract_rel(got, want).max() < 5e-6
    else:
        assert per_contract_rel(got, want).max() < 1e-10


@pytest.mark.parametrize("name", [n for n in CASE_NAMES if "f64" not in n])
def test_reference_math_targets_bit_exact_and_match_reference(oracle, gbm_golden, name) -> None:
    """SMC_MATH_REF (the reference kernel's own typing, rows_ref_kernel) on every f32 fixture case: bit-exact
    with its kernel-mode restatement and within 4e-6 per contract of the reference's own targets (the paths
    agree with the reference arithmetic to the bit, tests/test_oracle.py; what is left is the CF phase's f64
    sums against the reference's f32 normalisation)."""
    contracts, want, m = unpack(gbm_golden, name)
    got = train_targets(contracts, m, hw=False, ref=True)
    kt, _ = oracle.kernel_targets(contracts, m["T"], m["N"], m["M"], seed=m["seed"], ordinal0=m["ordinal0"],
                                  scheme=m["scheme"] | oracle.MATH_REF, normalize=m["normalize"])
    np.testing.assert_array_equal(got, kt)
    assert per_contract_rel(got, want).max() < 4e-6


@pytest.mark.parametrize("name", [n for n in CASE_NAMES if "f64" not in n])
def test_reference_math_on_hw_normals_matches_reference_fixture(gbm_golden, name) -> None:
    """SMC_MATH_REF | SMC_MATH_HW (math_mode "reference_hw": the reference typing's f64 step on the
    hardware-transcendental normals) on every f32 fixture case: within the hw mode's 1e-5 per contract of the
    reference's own targets (gbm_golden.npz, generated by the reference's gbm.py)."""
    contracts, want, m = unpack(gbm_golden, name)
    got = train_targets(contracts, m, hw=True, ref=True)
    assert np.isfinite(got).all()
    assert per_contract_rel(got, want).max() < 1e-5


def test_c2_bench_instantiation_whole_rounds(oracle, gbm_golden) -> None:
    """The kernel BENCH times, at its shape, over two whole rounds of resident workgroups
    (2 per CU): hw math within 1e-5 per contract of the reference-mode oracle, and the first two
    contracts within 1e-5 of the reference's own output."""
    from tests.helpers import make_domain_bounds

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    B = 4 * cus
    _, _, m = unpack(gbm_golden, "c2shape")
    assert (m["T"], m["N"], m["M"]) == (16, 256, 256) and m["ordinal0"] == 0
    kernel = _lib.lib().smc_train_targets_kernel(16, 256, 65536, _lib.DTYPE_F32, _lib.lib().smc_path_pitch(65536, 0), 0)
    assert kernel in (b"resident_kernel", b"paths_kernel+cf_kernel", b"contract_kernel")
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    np.testing.assert_array_equal(contracts[:2], gbm_golden["c2shape_contracts"])
    got = train_targets(contracts, m, hw=True)
    assert per_contract_rel(got[:2], gbm_golden["c2shape_targets"]).max() < 1e-5
    want = oracle.training_targets(contracts, 16, 256, 256, seed=7, ordinal0=0)
    assert per_contract_rel(got, want).max() < 1e-5
    # portable math at the same instantiation: bit-exact with the kernel-mode restatement
    sub = contracts[:64]
    port = train_targets(sub, m, hw=False)
    kt, _ = oracle.kernel_targets(sub, 16, 256, 256, seed=7, ordinal0=0, wg=oracle.engine_wg(16, 256, 65536))
    np.testing.assert_array_equal(port, kt)


def test_c2_timed_call_train_step(oracle, gbm_golden) -> None:
    """The exact call bench.py times at C2: smc_train_step, B = 4096, T = 16, N = M = 256, STORE_ALL,
    padded pitch, the sync area (dynamic contract tail + Sobol pre-draw), two consecutive steps from a
    non-zero cursor.  Contracts bit-equal to the reference sampler's points; hw math within 1e-5 per
    contract of the reference-mode oracle on a strided sample of 32 contracts (the first two against
    the reference's own c2shape fixture on step 1); portable math bit-exact with the kernel-mode
    oracle on a strided 64-contract sub-batch."""
    from tests.helpers import make_domain_bounds
    from spectralmc_amd.sobol_sampler import SobolEngine

    L = _lib.lib()
    B, T, N, M = 4096, 16, 256, 256
    P = N * M
    pitch = int(L.smc_path_pitch(P, 0))
    assert L.smc_train_step_kernel(T, N, M, 0, pitch) == b"resident_kernel"
    lo, hi = make_domain_bounds().arrays()
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(DEV)
    lo_d, hi_d = torch.from_numpy(lo).to(DEV), torch.from_numpy(hi).to(DEV)
    paths = poisoned((B, T, pitch), torch.float32, DEV)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, 0, pitch))
    sync = torch.zeros(nsync, dtype=torch.uint8, device=DEV)
    for math in (_lib.MATH_HW, 0):
        cur = torch.tensor([0, 0], dtype=torch.int64, device=DEV)
        for step in range(2):
            c = poisoned((B, 6), torch.float64, DEV)
            f = poisoned((B, 6), torch.float32, DEV)
            t = poisoned((B, N), torch.complex64, DEV)
            _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo_d), _lib.ptr(hi_d), _lib.ptr(cur), 0, B,
                                        _lib.ptr(c), _lib.ptr(f), B, T, N, M, 7, _lib.SCHEME_LOG_EULER | math,
                                        _lib.NORM_NORMALIZE, _lib.DTYPE_F32, _lib.STORE_ALL, _lib.ptr(paths), pitch,
                                        B, _lib.ptr(t), _lib.ptr(sync), nsync, None))
            torch.cuda.synchronize()
            assert _lib.sync_status(sync) == 0 and not sync.any()
            contracts = c.cpu().numpy()
            np.testing.assert_array_equal(contracts, oracle.sobol_contracts(7, step * B, B, lo, hi))
            np.testing.assert_array_equal(f.cpu().numpy(), contracts.astype(np.float32))
            got = t.cpu().numpy()
            if math:
                if step == 0:
                    assert per_contract_rel(got[:2], gbm_golden["c2shape_targets"]).max() < 1e-5
                idx = np.arange(step, B, B // 32)
                # the ordinal of contract i is step * B + i (one oracle call per sampled contract)
                want = np.stack([oracle.training_targets(contracts[i:i + 1], T, N, M, seed=7,
                                                         ordinal0=step * B + int(i))[0] for i in idx])
                assert per_contract_rel(got[idx], want).max() < 1e-5
            else:
                idx = np.arange(2 * step + 1, B, B // 64)
                kt = np.stack([oracle.kernel_targets(contracts[i:i + 1], T, N, M, seed=7, ordinal0=step * B + int(i),
                                                     wg=1024)[0][0] for i in idx])
                np.testing.assert_array_equal(got[idx], kt)
        assert cur.tolist() == [2 * B, 2 * B]


def test_c3_per_contract_shape(oracle, gbm_golden) -> None:
    """C3: N = 1024, M = 256 (P = 262,144 paths per contract), T = 16, hw math."""
    from tests.helpers import make_domain_bounds

    _, _, m = unpack(gbm_golden, "c3shape")
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, 10, lo, hi)[2:]  # row 2 = the fixture's contract, ordinal 0
    np.testing.assert_array_equal(contracts[:1], gbm_golden["c3shape_contracts"])
    got = train_targets(contracts, m, hw=True)
    assert per_contract_rel(got[:1], gbm_golden["c3shape_targets"]).max() < 1e-5
    want = oracle.training_targets(contracts, 16, 1024, 256, seed=7, ordinal0=0)
    assert per_contract_rel(got, want).max() < 1e-5


def test_c2_network_fused_step_matches_oracle(oracle) -> None:
    """One fused network step of the C2 CVNN (6 -> 32 -> 32 -> 256, 19,520 parameters) at
    B = 4096 vs the oracle's torch-cpu _torch_step: loss 1e-4 rel, grad norm 1e-3, gradients
    1e-4 norm-relative, post-Adam parameters within 1e-5 wherever the gradient is resolved."""
    from spectralmc_amd.net import FusedNetworkStep
    from tests.helpers import make_domain_bounds, make_test_cvnn

    B, N = 4096, 256
    lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)
    base = oracle.training_targets(contracts[:64], 16, N, 4, seed=7)  # CF-magnitude targets, tiled
    targets = np.tile(base, (B // 64, 1))
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device=DEV, hidden_layers=2)
    cpu_model = copy.deepcopy(model).cpu()
    params = list(model.parameters())
    adam = torch.optim.Adam(params, lr=1e-2)
    n = sum(p.numel() for p in params)
    flat = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
    loss = torch.zeros((), dtype=torch.float32, device=DEV)
    gnorm = torch.zeros((), dtype=torch.float32, device=DEV)
    step = FusedNetworkStep(model, adam, params, flat, loss, gnorm, B, fuse_adam=True)
    x = torch.tensor(contracts, dtype=torch.float32, device=DEV)
    step.fwd_bwd(x, torch.zeros_like(x), torch.from_numpy(targets).to(DEV))
    torch.cuda.synchronize()
    xc = torch.tensor(contracts, dtype=torch.float32)
    ref = oracle.torch_step(cpu_model, xc, torch.zeros_like(xc), torch.from_numpy(targets),
                            torch.optim.Adam(cpu_model.parameters(), lr=1e-2))
    assert float(loss) == pytest.approx(ref.loss, rel=1e-4)
    assert float(gnorm) == pytest.approx(ref.grad_norm, rel=1e-3)
    # gradients (the flat buffer the kernels reduce into, before Adam) vs torch autograd
    g_cpu = torch.cat([p.grad.reshape(-1) for p in cpu_model.parameters()]).double()
    g_gpu = flat[:n].cpu().double()
    assert float((g_gpu - g_cpu).norm() / g_cpu.norm()) < 1e-4
    # Adam's first step is lr * g / (|g| + eps) ~ lr * sign(g): equal wherever the gradient is
    # resolved above the f32 summation noise of a B = 4096 reduction; an element whose gradient
    # is ~0 may take either sign on either device
    off = 0
    for (name, pg), pc in zip(model.named_parameters(), cpu_model.parameters(), strict=True):
        k = pc.numel()
        a, b = pg.detach().cpu().double().reshape(-1).numpy(), pc.detach().double().reshape(-1).numpy()
        resolved = (g_cpu[off:off + k].abs() > 1e-5 * float(g_cpu.abs().max())).numpy()
        assert float(np.abs(a - b)[resolved].max(initial=0.0)) < 1e-5, name
        assert int((~resolved & (np.abs(a - b) > 1e-5)).sum()) <= max(2, k // 1000), name
        off += k
