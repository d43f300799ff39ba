"""Which contracts of the paths_kernel + cf_kernel launch come out wrong: the multi-round test case
(N = 2048, M = 2, T = 16, RAW, padded pitch, B = 520 Sobol contracts of the golden bounds, chunk 261),
against the oracle's kernel mode, with the paths / targets buffers pre-filled (NaN or garbage) so that
an unwritten element shows."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from spectralmc_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)


def run(c, T, N, M, store, pitch, chunk, fill_paths, fill_targets):
    L = _lib.lib()
    B = c.shape[0]
    cd = torch.from_numpy(c).to(DEV)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = torch.full(shape, fill_paths, dtype=torch.float32, device=DEV)
    tg = torch.full((B, N), fill_targets, dtype=torch.complex64, device=DEV)
    _lib.check(L.smc_train_targets(_lib.ptr(cd), B, T, N, M, 7, None, 9, 0, 0, 0, store, _lib.ptr(paths), pitch,
                                   chunk, None, _lib.ptr(tg), None, 0, None))
    torch.cuda.synchronize()
    return tg.cpu().numpy()


def main() -> None:
    oracle.build()
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
    B, T, N, M = 520, 16, 2048, 2
    c = oracle.sobol_contracts(7, 3, B, g["bounds_lower"], g["bounds_upper"])
    kt, _ = oracle.kernel_targets(c, T, N, M, seed=7, ordinal0=9, scheme=0, normalize=False,
                                  wg=oracle.engine_wg(T, N, N * M, normalize=False))
    L = _lib.lib()
    pitch = int(L.smc_path_pitch(N * M, 0))
    for store in (_lib.STORE_TERMINAL, _lib.STORE_ALL):
        for pp, chunk in ((N * M, B), (pitch, B), (pitch, B // 2 + 1), (pitch, 64)):
            for fp, ft in ((0.0, complex("nan")), (-1e20, 0j)):
                got = run(c, T, N, M, store, pp, chunk, fp, ft)
                bad = np.nonzero(~np.all(got == kt, axis=1))[0]
                nan = np.nonzero(np.isnan(got).any(axis=1))[0]
                print(f"store {store} pitch {pp} chunk {chunk} fill ({fp:g}, {ft}): {len(bad)} bad "
                      f"{bad[:24].tolist()} nan-rows {len(nan)} "
                      f"max|got| {float(np.abs(got).max()):.3g}", flush=True)


if __name__ == "__main__":
    main()
