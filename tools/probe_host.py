"""Probe: is a config's training step bound by the host?  Times the host side of each
TrainingSession.step() call (enqueue only) and the wall time per step of the same loop, for a bench.py
config.  When the host time per call is close to the wall time per step, the GPU waits for the host.
    python tools/probe_host.py --config e2e --steps 200
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="e2e")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch

    import bench
    from spectralmc_amd.gbm import ForwardNormalization
    from spectralmc_amd.gbm_trainer import GbmCVNNPricer
    from spectralmc_amd.models.numerical import Precision
    from tests.helpers import (expect_success, make_black_scholes_config, make_domain_bounds,
                               make_gbm_cvnn_config, make_simulation_params, make_test_cvnn, make_training_config)

    dev = torch.device("cuda", 0)
    B, T, N, M, widths, _ = bench.CONFIGS[args.config]
    f64 = bench.SIM_DTYPE.get(args.config) == "float64"
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256, mc_seed=7,
                                buffer_size=512, dtype=Precision.float64 if f64 else Precision.float32)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float64 if f64 else torch.float32,
                           device=dev, hidden_layers=len(widths), hidden_width=widths[0])
    norm = ForwardNormalization.RAW if args.config in bench.RAW_NORMALIZATION else ForwardNormalization.NORMALIZE
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(
        sim_params=sp, normalization=norm), domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    session = expect_success(pricer.open_session(make_training_config(num_batches=args.steps + 10, batch_size=B,
                                                                      learning_rate=1e-2)))
    for _ in range(5):
        expect_success(session.step())
    session.sync()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h0 = time.perf_counter()
        expect_success(session.step())
        host.append(time.perf_counter() - h0)
    session.sync()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    host.sort()
    print(f"{args.config}: wall {wall * 1e6:.1f} us/step, host per step() call median {host[len(host) // 2] * 1e6:.1f} "
          f"us, mean {sum(host) / len(host) * 1e6:.1f} us, p90 {host[int(0.9 * len(host))] * 1e6:.1f} us", flush=True)
    session.close()


if __name__ == "__main__":
    main()
