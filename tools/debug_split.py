"""Which contracts of the paths_kernel + cf_kernel launch come out wrong (N = 2048, M = 2, T = 16, RAW,
terminal store, padded pitch): the multi-round test case, run with several chunkings against the
contract_kernel result of the same contracts (unpadded pitch: the fused kernel)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from spectralmc_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)


def run(c, T, N, M, store, pitch, chunk, poison):
    L = _lib.lib()
    B = c.shape[0]
    P = N * M
    cd = torch.from_numpy(c).to(DEV)
    shape = (chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch)
    paths = torch.full(shape, poison, dtype=torch.float32, device=DEV)
    tg = torch.empty((B, N), dtype=torch.complex64, device=DEV)
    _lib.check(L.smc_train_targets(_lib.ptr(cd), B, T, N, M, 7, None, 9, 0, 0, 0, store, _lib.ptr(paths), pitch,
                                   chunk, None, _lib.ptr(tg), None, 0, None))
    torch.cuda.synchronize()
    return tg.cpu().numpy()


def main() -> None:
    rng = np.random.default_rng(5)
    B, T, N, M = 520, 16, 2048, 2
    c = np.stack([rng.uniform(50, 150, B), rng.uniform(50, 150, B), rng.uniform(0.1, 2, B), rng.uniform(0, 0.1, B),
                  rng.uniform(0, 0.05, B), rng.uniform(0.1, 0.5, B)], axis=1)
    L = _lib.lib()
    pitch = int(L.smc_path_pitch(N * M, 0))
    for store in (_lib.STORE_TERMINAL, _lib.STORE_ALL):
        ref = run(c, T, N, M, store, N * M, B, 0.0)
        print("store", store, "kernel (pitch P):", L.smc_train_targets_kernel(T, N, N * M, 0x100, N * M, 0),
              "padded:", L.smc_train_targets_kernel(T, N, N * M, 0x100, pitch, 0), flush=True)
        for chunk in (B, B // 2 + 1, 64, 1):
            for poison in (0.0, 1e30):
                got = run(c, T, N, M, store, pitch, chunk, poison)
                bad = np.nonzero(~np.all(got == ref, axis=1))[0]
                print(f"  chunk {chunk} poison {poison:g}: {len(bad)} bad contracts {bad[:40].tolist()}", flush=True)


if __name__ == "__main__":
    main()
