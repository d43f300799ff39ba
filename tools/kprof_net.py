"""Network-only driver for rocprofv3: the fused network step (FusedNetworkStep.fwd_bwd + Adam) of
the C2 / C2-H256 / C3 CVNN on synthetic inputs, `--iters` times.

    rocprofv3 --kernel-trace --stats -- python tools/kprof_net.py --arch c2 --compute auto
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from spectralmc_amd.net import FusedNetworkStep  # noqa: E402
from tests.helpers import make_test_cvnn  # noqa: E402

ARCH = {"c2": (4096, 256, 32), "h256": (4096, 256, 256), "c3": (16384, 1024, 32)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="c2", choices=sorted(ARCH))
    ap.add_argument("--compute", default="auto", choices=["auto", "valu", "mfma", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, N, H = ARCH[a.arch]
    dev = torch.device("cuda", 0)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device=dev, hidden_layers=2,
                           hidden_width=H)
    params = list(model.parameters())
    n = sum(p.numel() for p in params)
    flat = torch.zeros(n + 1, device=dev)
    loss, gn = torch.zeros((), device=dev), torch.zeros((), device=dev)
    step = FusedNetworkStep(model, torch.optim.Adam(params, lr=1e-3), params, flat, loss, gn, B, fuse_adam=True,
                            compute=a.compute)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand((B, 6), device=dev, generator=g)
    t = torch.complex(torch.randn((B, N), device=dev, generator=g), torch.randn((B, N), device=dev, generator=g))
    step.fwd_bwd(x, torch.zeros_like(x), t)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        step.fwd_bwd(x, torch.zeros_like(x), t)
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.arch} {step.kernels}: {e0.elapsed_time(e1) / a.iters * 1e3:.1f} us/step, loss {float(loss):.4e}")


if __name__ == "__main__":
    main()
