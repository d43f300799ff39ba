"""Kernel-only driver for rocprofv3: launches smc_basket_train_targets on one C5-sized launch
(1024 contracts x 4 assets x 131072 paths x T=16, store all, padded pitch) `--iters` times.

    rocprofv3 --kernel-trace --pmc WRITE_SIZE -- python tools/kprof_basket.py
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from spectralmc_amd import _lib  # noqa: E402
from spectralmc_amd.basket import BasketConfig  # noqa: E402
from spectralmc_amd.sobol_sampler import SobolEngine  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--A", type=int, default=4)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--M", type=int, default=512)
    ap.add_argument("--math", default="hw", choices=["hw", "portable"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--store", default="all", choices=["all", "terminal"])
    ap.add_argument("--split", action="store_true", help="no sync area: the basket_kernel (+ CF) launches")
    ap.add_argument("--trace", default="", help="save per-workgroup [start, xcc, group, end] (SMC_EXPERIMENT_TRACE builds)")
    a = ap.parse_args()
    cfg = BasketConfig(n_assets=a.A, timesteps=a.T, network_size=a.N, batches_per_mc_run=a.M, math=a.math)
    lo, hi = cfg.arrays()
    c = lo + (hi - lo) * SobolEngine(cfg.dim, 7).random(a.B)
    dev = torch.device("cuda", 0)
    cd = torch.from_numpy(c).to(dev)
    P = cfg.total_paths
    pitch = int(_lib.lib().smc_path_pitch(P, 0))
    store = _lib.STORE_ALL if a.store == "all" else _lib.STORE_TERMINAL
    paths = torch.empty((a.B, a.A, a.T if a.store == "all" else 1, pitch), dtype=torch.float32, device=dev)
    tg = torch.empty((a.B, a.N), dtype=torch.complex64, device=dev)
    L = _lib.lib()
    mh = _lib.MATH_HW if a.math == "hw" else 0
    ns = 0 if a.split else max(int(L.smc_basket_sync_bytes(a.A, a.T, a.N, a.M, a.B)), 0)
    sync = torch.zeros(ns, dtype=torch.uint8, device=dev) if ns else None

    def launch():
        _lib.check(L.smc_basket_train_targets(_lib.ptr(cd), a.B, a.A, a.T, a.N, a.M, 7, None, 0, mh, 1,
                                              store, _lib.ptr(paths), pitch, a.B, None, _lib.ptr(tg), _lib.ptr(sync), ns,
                                              None))

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
        buf = np.zeros((1024, 4), dtype=np.uint64)
        fn = L.smc_debug_btrace
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        assert fn(buf.ctypes.data, buf.size) == 0
        np.save(a.trace, buf)
    kname = L.smc_basket_train_targets_kernel(a.A, a.T, a.N, a.M, 1 if ns else 0, 0).decode()
    print(f"basket A={a.A} {a.math} {a.store} {kname}: {e0.elapsed_time(e1) / a.iters:.3f} ms/launch checksum",
          float(tg.abs().double().mean()))


if __name__ == "__main__":
    main()
