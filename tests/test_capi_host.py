"""libspectralmc_hip.so: loads, exports every symbol include/spectralmc_hip.h declares, host-side
Sobol is bit-exact with the reference's golden vectors, and argument errors come back as status
codes without touching a GPU.  CPU only (no kernel launches)."""

from __future__ import annotations

import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle
from spectralmc_amd import _lib
from spectralmc_amd.sobol_sampler import SobolEngine

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "spectralmc_hip.h")
TESTING_HEADER = os.path.join(os.path.dirname(HEADER), "spectralmc_hip_testing.h")


def declared_symbols(header: str = HEADER) -> list[str]:
    text = open(header).read()
    return sorted(set(re.findall(r"\b(smc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol() -> None:
    L = _lib.lib()
    names = declared_symbols()
    assert len(names) >= 14
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"
    assert L.smc_abi_version() == _lib.ABI_VERSION
    # the test-only entry points live in their own header and signature table, none in the product ABI
    testing = declared_symbols(TESTING_HEADER)
    assert testing == sorted(_lib.TEST_SIGNATURES) and not set(testing) & set(names)
    for name in testing:
        assert hasattr(L, name), name


def test_test_hooks_are_inert_without_the_environment_switch() -> None:
    """smc_test_exchange_fault does nothing and fails unless SMC_ENABLE_TEST_HOOKS=1 (a fresh process
    without it; no GPU call)."""
    code = ("import ctypes, sys; sys.path.insert(0, %r); from spectralmc_amd import _lib; L = _lib.lib(); "
            "print(L.smc_test_exchange_fault(1, 5), _lib.last_error())" % os.path.dirname(os.path.dirname(HEADER)))
    env = {k: v for k, v in os.environ.items() if k != "SMC_ENABLE_TEST_HOOKS"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split()[0] == str(_lib.SMC_ERR_INVALID_ARGUMENT) and "disabled" in out.stdout


INTEGRATION = os.path.join(os.path.dirname(HEADER), "..", "INTEGRATION.md")
_CTYPES = {"c_int32": ctypes.c_int32, "c_int64": ctypes.c_int64, "c_uint64": ctypes.c_uint64,
           "c_void_p": ctypes.c_void_p, "c_char_p": ctypes.c_char_p, "None": None,
           "ctypes.POINTER(c_void_p)": ctypes.POINTER(ctypes.c_void_p), "c_uint32": ctypes.c_uint32,
           "ctypes.POINTER(c_int32)": ctypes.POINTER(ctypes.c_int32),
           "ctypes.POINTER(c_int64)": ctypes.POINTER(ctypes.c_int64)}


def test_integration_doc_bindings_match_abi() -> None:
    """Every ctypes binding INTEGRATION.md shows a maintainer (argtypes and restype) equals the
    library's own binding table, which test_library_exports_every_declared_symbol ties to the
    header: the documented reference-side stub cannot drift from the ABI."""
    text = open(INTEGRATION).read()
    code = "\n".join(re.findall(r"```python\n(.*?)```", text, flags=re.S))
    code = re.sub(r"#[^\n]*", "", code)
    argtypes = re.findall(r"_lib\.(smc_\w+)\.argtypes\s*=\s*\[(.*?)\]\s*\n", code, flags=re.S)
    restypes = re.findall(r"_lib\.(smc_\w+)\.restype\s*=\s*([\w.()]+)", code)
    assert len(argtypes) >= 14
    for name, body in argtypes:
        items = [t.strip() for t in body.replace("\n", " ").split(",") if t.strip()]
        assert [_CTYPES[t] for t in items] == _lib.SIGNATURES[name][1], name
    for name, rt in restypes:
        assert _CTYPES[rt] == _lib.SIGNATURES[name][0], name
    assert {n for n, _ in argtypes} == {n for n, _ in restypes}
    # every header line the stub cites declares the function it binds
    header = open(HEADER).read().splitlines()
    for name, line in re.findall(r"_lib\.(smc_\w+)\.argtypes[^#]*?#\s*spectralmc_hip\.h:(\d+)", text, flags=re.S):
        assert f"{name}(" in header[int(line) - 1], (name, line)
    # every documented call passes as many arguments as the header declares
    calls = re.findall(r"_check\(_lib\.(smc_\w+)\((.*?)\)\)\n", code, flags=re.S)
    assert len(calls) >= 3
    for name, args in calls:
        depth, count = 0, 1
        for ch in args:
            depth += ch in "([{"
            depth -= ch in ")]}"
            count += ch == "," and depth == 0
        assert count == len(_lib.SIGNATURES[name][1]), name


@pytest.mark.parametrize("seed", [7, 31, 42, 123])
@pytest.mark.parametrize("skip", [0, 8, 4096])
def test_host_sobol_bit_exact_with_reference(golden, seed, skip) -> None:
    lo, hi = golden["bounds_lower"], golden["bounds_upper"]
    eng = SobolEngine(6, seed, skip)
    got = lo + (hi - lo) * eng.random(64)
    np.testing.assert_array_equal(got, golden[f"sobol_s{seed}_k{skip}"])
    got2 = lo + (hi - lo) * eng.random(32)
    np.testing.assert_array_equal(got2, golden[f"sobol_s{seed}_k{skip}_next"])
    assert eng.cursor == skip + 96


def test_sobol_tables_layout() -> None:
    eng = SobolEngine(6, 7, 0)
    shift, sv = eng.state()
    tab = eng.tables()
    np.testing.assert_array_equal(tab[:6], shift)
    np.testing.assert_array_equal(tab[6:].reshape(6, 30), sv)
    # first point of a scrambled sequence is the digital shift itself
    np.testing.assert_array_equal(eng.random(1)[0], shift.astype(np.float64) * 2.0 ** -30)


def test_sobol_argument_errors() -> None:
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.smc_sobol_create(0, 7, 0, ctypes.byref(h)) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert "dim" in _lib.last_error()
    assert L.smc_sobol_create(65, 7, 0, ctypes.byref(h)) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert L.smc_sobol_create(6, 7, (1 << 30) + 1, ctypes.byref(h)) == _lib.SMC_ERR_SEQUENCE_EXHAUSTED
    assert L.smc_sobol_create(6, 1 << 63, 0, ctypes.byref(h)) == _lib.SMC_ERR_SEED_OUT_OF_RANGE
    eng = SobolEngine(6, 7, (1 << 30) - 4)
    with pytest.raises(_lib.SmcError) as exc:
        eng.random(5)
    assert exc.value.code == _lib.SMC_ERR_SEQUENCE_EXHAUSTED


def test_engine_argument_errors_do_not_launch() -> None:
    L = _lib.lib()
    # NULL contracts / bad shapes / bad enums are rejected before any HIP call
    assert L.smc_gbm_simulate(None, 1, 16, 1024, 7, None, 0, 0, 0, None, None, None) == _lib.SMC_ERR_INVALID_ARGUMENT
    dummy = ctypes.c_double(0.0)
    p = ctypes.addressof(dummy)
    assert L.smc_gbm_simulate(p, 1, 0, 1024, 7, None, 0, 0, 0, p, None, None) == _lib.SMC_ERR_INVALID_SHAPE
    assert L.smc_gbm_simulate(p, 1, 16, 1024, 7, None, 0, 5, 0, p, None, None) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert L.smc_gbm_simulate(p, 1, 16, 1024, 7, None, 0, 0, 9, p, None, None) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert L.smc_train_targets(p, 4, 16, 0, 4, 7, None, 0, 0, 1, 0, 2, p, 0, 4, None, p, None, 0, None) == \
        _lib.SMC_ERR_INVALID_SHAPE
    assert L.smc_train_targets(p, 4, 16, 8, 4, 7, None, 0, 0, 1, 0, 3, p, 0, 4, None, p, None, 0, None) == \
        _lib.SMC_ERR_INVALID_ARGUMENT
    # an N too large for the LDS budget is a shape error, reported before launching
    assert L.smc_train_targets(p, 4, 16, 1 << 14, 1, 7, None, 0, 0, 1, 0, 2, p, 0, 4, None, p, None, 0, None) == \
        _lib.SMC_ERR_INVALID_SHAPE
    # a row pitch below P, or not a multiple of 4, is a shape error
    assert L.smc_train_targets(p, 4, 16, 8, 4, 7, None, 0, 0, 1, 0, 2, p, 31, 4, None, p, None, 0, None) == \
        _lib.SMC_ERR_INVALID_SHAPE
    assert L.smc_train_targets(p, 4, 16, 8, 4, 7, None, 0, 0, 1, 0, 2, p, 34, 4, None, p, None, 0, None) == \
        _lib.SMC_ERR_INVALID_SHAPE
    # smc_train_step checks the pitch before choosing the fused resident launch: a pitch below P
    # would make the contract rows overlap and the last ones write past the caller's buffer
    for pitch in (4, 65532, 65538):
        assert L.smc_train_step(p, 6, p, p, p, 0, 0, p, None, 4, 16, 256, 256, 7, 0, 1, 0, 2, p, pitch, 4, p, p, 8,
                                None) == _lib.SMC_ERR_INVALID_SHAPE, pitch
    # whole-contract step shapes need no device query: done counter, status word, contract queue
    assert L.smc_train_step_sync_bytes(16, 256, 256, 0, 66560) == 128
    out = ctypes.c_int32(-1)
    assert L.smc_sync_status(None, 1, ctypes.byref(out), None) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert L.smc_test_exchange_fault(2, 0) == _lib.SMC_ERR_INVALID_ARGUMENT
    assert L.smc_test_exchange_fault(0, 0) == _lib.SMC_OK
    assert L.smc_normals(7, 0, 0, 10, 0, p, None) == _lib.SMC_ERR_INVALID_SHAPE
    assert L.smc_sobol_draw(None, 6, None, 0, 4, p, p, p, None, None) == _lib.SMC_ERR_INVALID_ARGUMENT


def test_zero_contracts_is_a_noop() -> None:
    L = _lib.lib()
    dummy = ctypes.c_double(0.0)
    p = ctypes.addressof(dummy)
    assert L.smc_train_targets(p, 0, 16, 8, 4, 7, None, 0, 0, 1, 0, 2, p, 0, 4, None, p, None, 0, None) == _lib.SMC_OK


def test_path_pitch_is_an_odd_multiple_of_4k() -> None:
    L = _lib.lib()
    assert L.smc_path_pitch(65536, _lib.DTYPE_F32) == 65536 + 1024
    assert L.smc_path_pitch(1024, _lib.DTYPE_F32) == 1024
    assert L.smc_path_pitch(1000, _lib.DTYPE_F32) == 1024
    assert L.smc_path_pitch(65536, _lib.DTYPE_F64) == 65536 + 512
    for P in (4, 100, 4096, 262144, 1 << 20):
        q = L.smc_path_pitch(P, _lib.DTYPE_F32)
        assert q >= P and (q * 4) % 4096 == 0 and ((q * 4) // 4096) % 2 == 1


def test_train_targets_kernel_choice() -> None:
    """Which path/CF kernels smc_train_targets runs: the sliced queue kernel with a workspace;
    resident_kernel for the f32 training shapes it covers (any T, 4096 | P <= 65,536, N | 4096,
    N <= 1024); else a split pair with the terminal-row sum parked in the scratch row's padding (so it
    needs a padded pitch such as smc_path_pitch): the straight-line paths_kernel + cf_kernel at T = 16,
    rows_kernel + cf_kernel for other T and for f64; contract_kernel otherwise."""
    L = _lib.lib()
    split = b"paths_kernel+cf_kernel"
    assert L.smc_train_targets_kernel(16, 256, 65536, 0, 66560, 0) == b"resident_kernel"    # C2
    assert L.smc_train_targets_kernel(16, 256, 65536, 0, 0, 0) == b"resident_kernel"        # no pad needed
    assert L.smc_train_targets_kernel(16, 2048, 65536, 0, 66560, 0) == split                 # N > 1024
    assert L.smc_train_targets_kernel(16, 1024, 262144, 0, L.smc_path_pitch(262144, 0), 0) == split  # C3
    assert L.smc_train_targets_kernel(16, 1024, 262144, 0, 0, 0) == b"contract_kernel"      # no padding
    assert L.smc_train_targets_kernel(16, 256, 65536, 0, 66560, 1) == b"queue_kernel"
    rows = b"rows_kernel+cf_kernel"
    assert L.smc_train_targets_kernel(17, 256, 65536, 0, 0, 0) == b"resident_kernel"        # any T
    assert L.smc_train_targets_kernel(1, 16, 65536, 0, 66560, 0) == b"resident_kernel"      # lock-step, NORMALIZE
    raw = _lib.QUERY_RAW
    assert L.smc_train_targets_kernel(1, 16, 65536, raw, 66560, 0) == b"wave_kernel"        # lock-step, RAW
    assert L.smc_train_step_kernel(1, 16, 4096, raw, 66560) == b"wave_kernel"
    # any P: one wave walks the whole contract (P > 65,536 took the sliced resident kernel)
    assert L.smc_train_step_kernel(1, 16, 8192, raw, L.smc_path_pitch(131072, 0)) == b"wave_kernel"
    assert L.smc_train_step_kernel(2, 64, 4096, raw, 0) == b"wave_kernel"          # P = 262,144
    # QUERY_RAW has its own bit: a dtype carrying SMC_MATH_HW is a NORMALIZE query
    assert _lib.QUERY_RAW & _lib.MATH_HW == 0
    assert L.smc_train_step_kernel(1, 16, 8192, _lib.MATH_HW, 0) == b"resident_kernel(sliced)"
    assert L.smc_train_step_kernel(1, 16, 4096, _lib.MATH_HW, 0) == b"resident_kernel"
    assert L.smc_train_targets_kernel(3, 16, 65536, raw, 66560, 0) == b"resident_kernel"    # RAW, T > 2
    assert L.smc_train_targets_kernel(16, 128, 512, 0, 1024, 0) == b"packed_kernel"         # e2e shape, P = 512
    assert L.smc_train_targets_kernel(17, 2048, 65536, 0, 66560, 0) == rows                 # N > 1024, T != 16
    assert L.smc_train_targets_kernel(17, 2048, 65536, 0, 0, 0) == b"contract_kernel"       # no padding
    assert L.smc_train_targets_kernel(16, 256, 65536, 1, 66048, 0) == b"rows_kernel+cf_kernel"  # f64
    assert L.smc_train_targets_kernel(16, 256, 65536, 1, 0, 0) == b"contract_kernel"        # f64, no padding
    assert L.smc_train_targets_kernel(16, 6, 6144, 0, 6144, 0) == b"contract_kernel"        # pitch == P
    assert L.smc_train_targets_kernel(16, 6, 6144, 0, 7168, 0) == split                     # N not | 4096
    # SMC_MATH_REF: the name only where launch_engine takes the shape
    ref = _lib.MATH_REF
    assert L.smc_train_targets_kernel(16, 256, 65536, ref, 66560, 0) == b"rows_ref_kernel+cf_kernel"
    assert L.smc_train_step_kernel(16, 256, 256, ref, 66560) == b"rows_ref_kernel+cf_kernel"
    assert L.smc_train_targets_kernel(16, 256, 65536, 1 | ref, 66560, 0) == b"unsupported"  # f64
    assert L.smc_train_targets_kernel(16, 256, 65536, ref, 0, 0) == b"unsupported"          # no room for the sum
    assert L.smc_train_step_kernel(16, 256, 256, ref, 65536) == b"unsupported"
    assert L.smc_train_targets_kernel(16, 256, 65536, ref, 66560, 1) == b"unsupported"      # sliced
    # SMC_MATH_REF | SMC_MATH_HW (ABI 15): the same kernels on the hardware-transcendental normals
    hwref = _lib.MATH_REF | _lib.MATH_HW
    assert L.smc_train_targets_kernel(16, 256, 65536, hwref, 66560, 0) == b"rows_ref_kernel+cf_kernel"
    assert L.smc_train_step_kernel(16, 256, 256, hwref, 66560) == b"rows_ref_kernel+cf_kernel"
    assert L.smc_train_targets_kernel(16, 256, 65536, 1 | hwref, 66560, 0) == b"unsupported"  # f64


def test_engine_rejects_reference_math_it_cannot_run() -> None:
    """TrainingEngine(math="reference") fails at construction (before touching a device) for f64 and for
    sliced engines, instead of on the first step's launch."""
    import torch

    from spectralmc_amd.engine import TrainingEngine
    from spectralmc_amd.gbm import BlackScholes
    from spectralmc_amd.models.numerical import Precision
    from spectralmc_amd.sobol_sampler import SobolSampler, build_sobol_config
    from tests.helpers import expect_success, make_black_scholes_config, make_domain_bounds, make_simulation_params

    for math in ("reference", "reference_hw"):
        for dtype, sliced, msg in ((Precision.float32, True, "sliced"), (Precision.float64, False, "float32")):
            sp = make_simulation_params(timesteps=16, network_size=64, batches_per_mc_run=8, threads_per_block=256,
                                        mc_seed=7, buffer_size=4, dtype=dtype)
            cfg = make_black_scholes_config(sim_params=sp)
            sampler = expect_success(SobolSampler.create(BlackScholes.Inputs, make_domain_bounds(),
                                                         config=build_sobol_config(seed=7, skip=0).unwrap()))
            with pytest.raises(ValueError, match=msg):
                TrainingEngine(cfg, sampler, 4, model_dtype=torch.float32, device=torch.device("cpu"), math=math,
                               sliced=sliced)
    with pytest.raises(ValueError, match="reference_hw"):
        TrainingEngine(cfg, sampler, 4, model_dtype=torch.float32, device=torch.device("cpu"), math="fast")


def test_basket_entry_points_validate_before_any_device_work() -> None:
    """Bad basket arguments are rejected on the host (no GPU needed): asset count, shapes, math."""
    L = _lib.lib()
    assert L.smc_basket_resident_slots(0, 256, 0) == -1
    assert L.smc_basket_resident_slots(9, 256, 0) == -1
    assert L.smc_basket_resident_slots(4, 0, 0) == -1
    assert L.smc_basket_resident_slots(4, 8192, 0) == -1
    fake = 1 << 20  # never dereferenced: validation fails first
    assert L.smc_basket_train_targets(None, 1, 4, 16, 256, 8, 7, None, 0, 0, 1, 2, fake, 0, 1, None, fake,
                                      None, 0, None) == 1
    assert L.smc_basket_train_targets(fake, 1, 0, 16, 256, 8, 7, None, 0, 0, 1, 2, fake, 0, 1, None, fake,
                                      None, 0, None) == 1
    assert L.smc_basket_train_targets(fake, 1, 4, 16, 256, 3, 7, None, 0, 0, 1, 2, fake, 0, 1, None, fake,
                                      None, 0, None) == 2  # N*M not a multiple of 2048
    assert L.smc_basket_train_targets(fake, 1, 4, 16, 256, 8, 7, None, 0, 7, 1, 2, fake, 0, 1, None, fake,
                                      None, 0, None) == 1  # bad math flag
    assert L.smc_basket_train_targets(fake, 1, 4, 16, 256, 8, 7, None, 0, 0, 1, 3, fake, 0, 1, None, fake,
                                      None, 0, None) == 1  # bad store mode
    assert L.smc_basket_train_targets(fake, 1, 4, 16, 256, 8, 7, None, 0, 0, 1, 2, fake, 100, 1, None, fake,
                                      None, 0, None) == 2  # pitch < P


def test_basket_sync_bytes_and_kernel_choice_on_host() -> None:
    """smc_basket_sync_bytes rejects bad arguments and returns 0 (no sync area, no device query)
    for shapes the resident kernel does not take; the kernel-name query mirrors the dispatch
    (oracle.basket_order states the same conditions)."""
    L = _lib.lib()
    assert L.smc_basket_sync_bytes(0, 16, 256, 512, 64) == -1
    assert L.smc_basket_sync_bytes(9, 16, 256, 512, 64) == -1
    assert L.smc_basket_sync_bytes(4, 16, 0, 512, 64) == -1
    assert L.smc_basket_sync_bytes(4, 16, 256, 512, 0) == -1     # chunk_contracts <= 0
    assert L.smc_basket_sync_bytes(4, 5, 256, 512, 64) == 0          # T != 16
    assert L.smc_basket_sync_bytes(4, 16, 256, 8, 64) == 0           # P = 2048: not a multiple of 4096
    assert L.smc_basket_sync_bytes(4, 16, 256, 1024, 64) == 0        # W = 64 > 32
    assert L.smc_basket_sync_bytes(4, 16, 12, 1024, 64) == 0         # N does not divide 4096
    assert L.smc_basket_sync_bytes(8, 16, 2048, 8, 64) == 0          # LDS plan over 160 KiB
    name = lambda *a: L.smc_basket_train_targets_kernel(*a).decode()  # noqa: E731
    assert name(4, 16, 256, 512, 1, 1) == "basket_resident_kernel"
    assert name(4, 16, 256, 512, 0, 1) == "basket_kernel+basket_cf_kernel"
    assert name(4, 16, 256, 512, 0, 0) == "basket_kernel"
    assert name(4, 5, 256, 512, 1, 1) == "basket_kernel+basket_cf_kernel"
    for A, T, N, M in [(4, 16, 256, 512), (1, 16, 64, 64), (8, 16, 256, 16), (8, 16, 2048, 8), (4, 16, 256, 1024),
                       (3, 16, 1024, 8), (2, 4, 256, 16), (6, 16, 256, 32), (7, 16, 256, 32), (6, 16, 2048, 8)]:
        wg, _ = oracle.basket_order(A, T, N, M)
        assert (wg == 1024) == (name(A, T, N, M, 1, 1) == "basket_resident_kernel"), (A, T, N, M)


def test_engine_workspace_size_and_check() -> None:
    """Sliced contracts (8192-path workgroup slices): f64 slice sums + a u32 arrival counter
    per contract; too small a workspace is a shape error raised before any launch."""
    L = _lib.lib()
    assert L.smc_engine_workspace_bytes(4096, 16, 8192, 0) == 0          # one slice: no workspace
    assert L.smc_engine_workspace_bytes(4096, 16, 65536, 0) == 4096 * 8 * 8 + (4096 + 16) * 4
    assert L.smc_engine_workspace_bytes(10, 16, 65536, 1) == 10 * 8 * 16 * 8 + (10 + 16) * 4
    assert L.smc_engine_workspace_bytes(3, 20, 25000, 0) == 3 * 4 * 8 + (3 + 16) * 4   # 13 chunks -> 4 slices
    dummy = ctypes.c_double(0.0)
    p = ctypes.addressof(dummy)
    assert L.smc_train_targets(p, 4, 16, 256, 64, 7, None, 0, 0, 1, 0, 2, p, 0, 4, None, p, p, 8, None) == \
        _lib.SMC_ERR_INVALID_SHAPE
