"""Probe: does what runs between two path launches change the path launch's duration?

Per-call HIP-event durations of the targets launch (rows_kernel + cf_kernel for C2-f64) when the
launches run (a) back to back, (b) with a GPU sleep between them, (c) with the fused network part
between them, and (d) the whole training step (captured graph).  Prints one line per mode.
    python tools/probe_gap.py --config c2f64 --iters 12 --sleep-us 300
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2f64")
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--sleep-us", type=int, default=300)
    args = ap.parse_args()
    import torch

    import bench
    from spectralmc_amd import _lib
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
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(
        sim_params=sp, normalization=ForwardNormalization.NORMALIZE), domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    session = expect_success(pricer.open_session(make_training_config(num_batches=4 * args.iters + 8, batch_size=B,
                                                                      learning_rate=1e-2)))
    for _ in range(3):
        expect_success(session.step())
    session.sync()
    eng, prog = session.engine, session.program
    fused = prog.fused
    stream = torch.cuda.Stream(device=dev)
    cycles = int(args.sleep_us * 2.4e3)  # ~2.4 GHz shader clock

    slot0 = prog.slots[0]

    def launch(mode: str = ""):
        if mode == "enqueue":  # the MC part exactly as the step enqueues it (draw, targets, cursor)
            eng.enqueue_step(slot0)
        elif mode == "slot":  # the targets launch on the last drawn contracts, device ordinal
            eng.launch_targets(_lib.stream_handle(stream), _lib.ptr(eng.cursor[1:2]), 0, slot0)
        else:
            eng.launch_targets(_lib.stream_handle(stream), None, 0)

    def net():
        if fused is not None:
            fused.fwd_bwd(prog.real_in[0], prog.imag_in, prog.targets[0])
            if not fused.fuse_adam:
                fused.adam()

    def run(mode: str) -> list[float]:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
        with torch.cuda.stream(stream):
            for e0, e1 in ev:
                e0.record(stream)
                launch(mode)
                e1.record(stream)
                if mode == "sleep":
                    torch.cuda._sleep(cycles)
                elif mode == "network":
                    net()
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in ev]

    c = eng.buffers.contracts
    print("engine-buffer contracts: min %.4g max %.4g; slot contracts: min %.4g max %.4g" % (
        float(c.min()), float(c.max()), float(slot0.contracts.min()), float(slot0.contracts.max())), flush=True)
    for mode in ("alone", "slot", "enqueue", "sleep", "network", "alone"):
        t = run(mode)
        print(f"{mode:8s} " + " ".join(f"{x:.3f}" for x in t) + f"  | last half mean {sum(t[len(t)//2:])/(len(t)-len(t)//2):.3f}",
              flush=True)
    # whole steps (graph replays), per-step wall time from events on the session's stream
    ts = []
    for _ in range(args.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(session.stream)
        expect_success(session.step())
        e1.record(session.stream)
        ts.append((e0, e1))
    session.sync()
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ts]
    print("step     " + " ".join(f"{x:.3f}" for x in t), flush=True)
    session.close()


if __name__ == "__main__":
    main()
