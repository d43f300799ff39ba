"""Round-4 failure hunt: the multi-round test's split-pair shape (B = 520, T = 16,
N = 2048, M = 2, RAW, padded pitch -> paths_kernel + cf_kernel) run repeatedly on dirty memory with
poisoned (NaN) outputs, several chunkings and both store modes, against the oracle's kernel mode.
Prints the bad contracts per run.  --lib loads another build of the library (same smc_train_targets
signature) to compare builds in one process-free way (one library per process)."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from spectralmc_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)


def load(path: str | None) -> ctypes.CDLL:
    if not path:
        return _lib.lib()
    L = ctypes.CDLL(path)
    for name in ("smc_train_targets", "smc_path_pitch"):
        rt, args = _lib.SIGNATURES[name]
        fn = getattr(L, name)
        fn.restype, fn.argtypes = rt, args
    return L


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    L = load(a.lib)
    oracle.build()
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
    B, T, N, M = 520, 16, 2048, 2
    P = N * M
    c = oracle.sobol_contracts(7, 3, B, g["bounds_lower"], g["bounds_upper"])
    kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=0, normalize=False,
                                  wg=oracle.engine_wg(T, N, P, normalize=False))
    cd = torch.from_numpy(c).to(DEV)
    pitch = int(L.smc_path_pitch(P, 0))
    total_bad = 0
    for rep in range(a.reps):
        for store in (_lib.STORE_TERMINAL, _lib.STORE_ALL):
            for chunk in (B // 2 + 1, 64, B, 173):
                # dirty the allocator's blocks with garbage of large magnitude, then free them
                junk = torch.empty(64 << 20, dtype=torch.int32, device=DEV).random_(-2 ** 31, 2 ** 31 - 1)
                del junk
                shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
                paths = torch.full(shape, float("nan"), dtype=torch.float32, device=DEV)
                tg = torch.full((B, N), complex("nan"), dtype=torch.complex64, device=DEV)
                _lib.check(L.smc_train_targets(_lib.ptr(cd), B, T, N, M, 7, None, 9, 0, 0, 0, store, _lib.ptr(paths),
                                               pitch, chunk, None, _lib.ptr(tg), None, 0, None))
                torch.cuda.synchronize()
                got = tg.cpu().numpy()
                bad = np.nonzero(~np.all(got == kt, axis=1))[0]
                total_bad += len(bad)
                print(f"rep {rep} store {store} chunk {chunk}: {len(bad)} bad {bad[:16].tolist()} "
                      f"nan-rows {int(np.isnan(got).any(axis=1).sum())}", flush=True)
    print(f"total bad contracts: {total_bad}", flush=True)


if __name__ == "__main__":
    main()
