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

# arch: (batch, outputs N, hidden width, hidden layers): C2 / C2-H256 / C3 and the reference's lock-step and e2e
# shapes (tests/test_gbm_trainer.py:122-131, tests/test_e2e/test_full_stack_cvnn_pricer.py:40-51) at C2's batch
ARCH = {"c2": (4096, 256, 32, 2), "h256": (4096, 256, 256, 2), "c3": (16384, 1024, 32, 2),
        "lockstep": (4096, 16, 32, 2), "e2e": (4096, 128, 32, 1)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="c2", choices=sorted(ARCH))
    ap.add_argument("--compute", default="auto", choices=["auto", "valu", "mfma", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cus", type=int, default=0, help="run on a CU-masked stream of this many CUs (0: whole chip)")
    ap.add_argument("--storm", action="store_true",
                    help="an HBM write storm (torch fill_ of 8 GiB, repeatedly) on the other CUs meanwhile: the "
                         "path kernel's store stream the network runs beside in the step")
    a = ap.parse_args()
    B, N, H, HL = ARCH[a.arch]
    dev = torch.device("cuda", 0)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device=dev, hidden_layers=HL,
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
    xi = torch.zeros_like(x)
    owned: list[int] = []
    stream, storm = torch.cuda.current_stream(), None
    if a.cus:
        from spectralmc_amd.gbm_trainer import _cu_masks, _destroy_streams, _masked_stream

        net_mask, rest = _cu_masks(dev, a.cus, "low")
        stream = _masked_stream(dev, net_mask, owned)
        storm = _masked_stream(dev, rest, owned) if a.storm else None
    elif a.storm:
        storm = torch.cuda.Stream(device=dev)
    buf = torch.empty((8 << 30) // 4, dtype=torch.float32, device=dev) if storm is not None else None
    with torch.cuda.stream(stream):
        step.fwd_bwd(x, xi, t)
    torch.cuda.synchronize()
    if storm is not None:  # keep the storm running across the timed region
        with torch.cuda.stream(storm):
            for _ in range(8):
                buf.fill_(1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        for _ in range(a.iters):
            step.fwd_bwd(x, xi, t)
        e1.record(stream)
    torch.cuda.synchronize()
    print(f"{a.arch} {step.kernels} cus={a.cus or 'all'} storm={a.storm}: {e0.elapsed_time(e1) / a.iters * 1e3:.1f} "
          f"us/step, loss {float(loss):.4e}")
    if owned:
        _destroy_streams(owned)


if __name__ == "__main__":
    main()
