"""Kernel-only driver for rocprofv3: launches smc_train_targets on a C2-sized batch
`--iters` times (no CVNN), for PMC / kernel-trace collection.

    rocprofv3 --pmc SQ_WAVES ... -- python tools/kprof.py --math hw --store all
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from spectralmc_amd import _lib  # noqa: E402
from spectralmc_amd.sobol_sampler import SobolEngine  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--math", default="hw", choices=["hw", "portable"])
    ap.add_argument("--store", default="all", choices=["all", "terminal"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--pitch", type=int, default=-1, help="row pitch (-1: smc_path_pitch, 0: P)")
    ap.add_argument("--unsliced", action="store_true", help="one workgroup per contract (no workspace)")
    ap.add_argument("--trace", default="", help="save per-workgroup timestamps (SMC_EXPERIMENT_TRACE builds)")
    a = ap.parse_args()
    lo = np.array([0.001, 0.001, 0.0, -0.2, -0.2, 0.0])
    hi = np.array([1e4, 2e4, 10.0, 0.2, 0.2, 2.0])
    c = lo + (hi - lo) * SobolEngine(6, 7).random(a.B)
    dev = torch.device("cuda", 0)
    cd = torch.from_numpy(c).to(dev)
    P = a.N * a.M
    store = _lib.STORE_ALL if a.store == "all" else _lib.STORE_TERMINAL
    pitch = int(_lib.lib().smc_path_pitch(P, 0)) if a.pitch < 0 else (a.pitch or P)
    paths = torch.empty((a.B, a.T, pitch) if store == _lib.STORE_ALL else (a.B, pitch), dtype=torch.float32, device=dev)
    tg = torch.empty((a.B, a.N), dtype=torch.complex64, device=dev)
    scheme = _lib.SCHEME_LOG_EULER | (_lib.MATH_HW if a.math == "hw" else 0)
    L = _lib.lib()
    wsb = 0 if a.unsliced else int(L.smc_engine_workspace_bytes(a.B, a.T, P, 0))
    ws = torch.zeros(max(wsb, 8), dtype=torch.uint8, device=dev) if wsb else None

    def launch():
        _lib.check(L.smc_train_targets(_lib.ptr(cd), a.B, a.T, a.N, a.M, 7, None, 0, scheme, 1, 0, store,
                                       _lib.ptr(paths), pitch, a.B, None, _lib.ptr(tg), _lib.ptr(ws), wsb, None))

    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    if a.trace:
        import ctypes
        n = 1024 * 40  # gbm.hip g_trace: [workgroup][40] s_memrealtime stamps (SMC_EXPERIMENT_TRACE builds)
        buf = np.zeros((1024, 40), dtype=np.uint64)
        fn = getattr(L, "smc_debug_trace")
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, n) == 0
        np.save(a.trace, buf)
    print(f"{os.environ.get('SMC_LIB_PATH', 'default')} {a.math} {a.store} pitch={pitch} sliced={not a.unsliced}: "
          f"{e0.elapsed_time(e1) / a.iters:.3f} ms/launch",
          "checksum", float(tg.abs().double().mean()))


if __name__ == "__main__":
    main()
