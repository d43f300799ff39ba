"""ctypes binding of ``libspectralmc_hip.so`` — the C ABI declared in ``include/spectralmc_hip.h``.

There is deliberately no fallback: if the shared library is missing, or a device entry
point is called without a ROCm GPU, the call raises.  Build the library with
``python __graft_entry__.py`` (or ``make -C spectralmc_amd/csrc``).
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Any

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMC_LIB_PATH") or os.path.join(_HERE, "libspectralmc_hip.so")

# status codes (spectralmc_hip.h)
SMC_OK = 0
SMC_ERR_INVALID_ARGUMENT = 1
SMC_ERR_INVALID_SHAPE = 2
SMC_ERR_SEED_OUT_OF_RANGE = 3
SMC_ERR_SEQUENCE_EXHAUSTED = 4
SMC_ERR_MEMORY_LIMIT = 5
SMC_ERR_HIP = 6
SMC_ERR_EXCHANGE_TIMEOUT = 7
SYNC_STATUS_OFFSET = 32
SYNC_EXCHANGE_TIMEOUT = 1

SCHEME_LOG_EULER = 0
SCHEME_SIMPLE_EULER = 1
NORM_RAW = 0
NORM_NORMALIZE = 1
DTYPE_F32 = 0
DTYPE_F64 = 1
QUERY_RAW = 0x1000  # smc_train_step_kernel / smc_train_targets_kernel: the targets use RAW normalisation
STORE_TERMINAL = 1
MATH_HW = 0x100
TRAIN_DYNAMIC = 0x200
MATH_REF = 0x400  # the reference kernel's typing: f64 state and step, f32 normals and stores
STORE_ALL = 2
SOBOL_BITS = 30
ABI_VERSION = 15

_c_i32, _c_i64, _c_u64, _c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p

# name -> (restype, argtypes); every symbol the header declares.
SIGNATURES: dict[str, tuple[Any, list[Any]]] = {
    "smc_abi_version": (_c_i32, []),
    "smc_last_error_string": (ctypes.c_char_p, []),
    "smc_time_launches": (_c_i32, [_c_vp, _c_vp]),
    "smc_sync_status": (_c_i32, [_c_vp, _c_i32, ctypes.POINTER(_c_i32), _c_vp]),
    "smc_sobol_create": (_c_i32, [_c_i32, _c_u64, _c_u64, ctypes.POINTER(_c_vp)]),
    "smc_sobol_destroy": (None, [_c_vp]),
    "smc_sobol_state": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp]),
    "smc_sobol_fast_forward": (_c_i32, [_c_vp, _c_u64]),
    "smc_sobol_random_host": (_c_i32, [_c_vp, _c_i64, _c_vp]),
    "smc_sobol_export_tables": (_c_i32, [_c_vp, _c_vp]),
    "smc_sobol_draw": (_c_i32, [_c_vp, _c_i32, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "smc_gbm_simulate": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i64, _c_u64, _c_vp, _c_i64, _c_i32, _c_i32,
                                  _c_vp, _c_vp, _c_vp]),
    "smc_gbm_normalize": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i64, _c_i32, _c_vp, _c_vp, _c_vp]),
    "smc_cf_targets": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_vp, _c_vp, _c_vp,
                                _c_vp]),
    "smc_train_targets": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_u64, _c_vp, _c_i64, _c_i32,
                                   _c_i32, _c_i32, _c_i32, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_i64,
                                   _c_vp]),
    "smc_train_step": (_c_i32, [_c_vp, _c_i32, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_i64, _c_i32, _c_i32,
                                _c_i32, _c_u64, _c_i32, _c_i32, _c_i32, _c_i32, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp,
                                _c_i64, _c_vp]),
    "smc_train_step_sync_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i64]),
    "smc_train_step_kernel": (ctypes.c_char_p, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i64]),
    "smc_engine_workspace_bytes": (_c_i64, [_c_i64, _c_i32, _c_i64, _c_i32]),
    "smc_train_targets_kernel": (ctypes.c_char_p, [_c_i32, _c_i32, _c_i64, _c_i32, _c_i64, _c_i32]),
    "smc_path_pitch": (_c_i64, [_c_i64, _c_i32]),
    "smc_normals": (_c_i32, [_c_u64, _c_i64, _c_i32, _c_i64, _c_i32, _c_vp, _c_vp]),
    "smc_cvnn_plan": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_i64, ctypes.POINTER(_c_i64)]),
    "smc_cvnn_forward_backward": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_i64,
                                           _c_vp, _c_i64, _c_vp]),
    "smc_cvnn_reduce_grads": (_c_i32, [_c_i32, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp]),
    "smc_adam_step": (_c_i32, [_c_i32, _c_i64, _c_vp, _c_vp, _c_vp]),
    "smc_adam_norm_partials": (_c_i64, [_c_i64]),
    "smc_cvnn_mfma_plan": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_i64, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "smc_cvnn_mfma_forward_backward": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_i64,
                                                _c_vp, _c_i64, _c_vp, _c_i64, _c_vp]),
    "smc_cvnn_mfma_pack_plan": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_i64, _c_vp, _c_vp]),
    "smc_basket_train_targets": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_i32, _c_u64, _c_vp, _c_i64,
                                          _c_i32, _c_i32, _c_i32, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp,
                                          _c_i64, _c_vp]),
    "smc_basket_sync_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i64]),
    "smc_basket_train_targets_kernel": (ctypes.c_char_p, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32]),
    "smc_basket_resident_slots": (_c_i64, [_c_i32, _c_i32, _c_i32]),
}

# include/spectralmc_hip_testing.h: test-only entry points, inert unless SMC_ENABLE_TEST_HOOKS=1
TEST_SIGNATURES: dict[str, tuple[Any, list[Any]]] = {
    "smc_test_exchange_fault": (_c_i32, [_c_i32, ctypes.c_uint32]),
}

CVNN_MAX_LAYERS = 8
ACT_NONE, ACT_MODRELU, ACT_ZRELU = 0, 1, 2
CVNN_MFMA_F32, CVNN_MFMA_BF16 = 1, 2
CVNN_MFMA_PACKED = 0x100  # forward_backward mode flag: the last Adam update wrote the packed weights


class CvnnLayer(ctypes.Structure):
    """smc_cvnn_layer (include/spectralmc_hip.h)."""

    _fields_ = [("in_features", _c_i32), ("out_features", _c_i32), ("activation", _c_i32), ("reserved", _c_i32),
                ("w_re", _c_i64), ("w_im", _c_i64), ("b_re", _c_i64), ("b_im", _c_i64), ("act_bias", _c_i64)]


class AdamArgs(ctypes.Structure):
    """smc_adam_args (include/spectralmc_hip.h)."""

    _fields_ = [("params", _c_vp), ("exp_avg", _c_vp), ("exp_avg_sq", _c_vp), ("step", _c_vp),
                ("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("weight_decay", ctypes.c_double), ("norm_partials", _c_vp),
                ("grad_norm", _c_vp), ("loss", _c_vp), ("pack", _c_vp)]


class CvnnPackLayer(ctypes.Structure):
    """smc_cvnn_pack_layer (include/spectralmc_hip.h)."""

    _fields_ = [("w_re", _c_i64), ("w_im", _c_i64), ("ni", _c_i32), ("no", _c_i32), ("win", _c_i32),
                ("wout", _c_i32), ("wc", _c_i64), ("wct", _c_i64)]


class CvnnPack(ctypes.Structure):
    """smc_cvnn_pack (include/spectralmc_hip.h): where Adam writes the MFMA operand copies."""

    _fields_ = [("ws", _c_vp), ("bf16", _c_i32), ("n_layers", _c_i32), ("layer", CvnnPackLayer * CVNN_MAX_LAYERS)]


class HipExtensionMissing(ImportError):
    """libspectralmc_hip.so is not built (no silent CPU fallback exists)."""


class SmcError(RuntimeError):
    """Non-zero status from the C ABI."""

    def __init__(self, code: int, message: str) -> None:
        super().__init__(f"libspectralmc_hip status {code}: {message}")
        self.code = code
        self.message = message


class DeviceUnavailable(RuntimeError):
    """A device entry point was called without a ROCm GPU."""


_lock = threading.Lock()
_lib: ctypes.CDLL | None = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipExtensionMissing(
                    f"{LIB_PATH} not found: build it with `python __graft_entry__.py` "
                    "(hipcc --offload-arch=gfx950); there is no CPU fallback")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (restype, argtypes) in {**SIGNATURES, **TEST_SIGNATURES}.items():
                fn = getattr(handle, name)
                fn.restype = restype
                fn.argtypes = argtypes
            if handle.smc_abi_version() != ABI_VERSION:
                raise HipExtensionMissing(f"{LIB_PATH}: ABI {handle.smc_abi_version()} != {ABI_VERSION}")
            _lib = handle
    return _lib


def last_error() -> str:
    raw = lib().smc_last_error_string()
    return raw.decode() if raw else ""


def check(status: int) -> None:
    if status != SMC_OK:
        raise SmcError(status, last_error())


def sync_status(sync: Any, clear: bool = True, stream: Any = None) -> int:
    """The status word of an exchanging launch's sync area (waits for the stream; 0: no failure)."""
    out = _c_i32(0)
    check(lib().smc_sync_status(ptr(sync), 1 if clear else 0, ctypes.byref(out), stream_handle(stream)))
    return int(out.value)


def require_device() -> None:
    import torch

    if not torch.cuda.is_available() or torch.version.hip is None:
        raise DeviceUnavailable("the HIP path needs a ROCm GPU (torch.cuda on ROCm); no CPU fallback exists")


def ptr(t: Any) -> int | None:
    """Raw device/host address of a torch tensor / numpy array (None passes NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return int(t.data_ptr())
    return int(t.ctypes.data)


def stream_handle(stream: Any = None) -> int | None:
    """hipStream_t of a torch stream (default: the current stream)."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream) or None
