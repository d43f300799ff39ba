"""Host cost of the calls an eager e2e training step makes (round 5): the session's MC launch
(smc_train_step through TrainingEngine.enqueue_step), the fused network launch (FusedNetworkStep.fwd_bwd),
event record / wait, a timing-event pair as bench.py's live MC timing creates per step, and one whole
TrainingSession.step().  Each is timed over `--iters` back-to-back calls (the GPU work they enqueue is real;
the device queue drains at the end).

    python tools/probe_host_calls.py [--config e2e] [--iters 500]
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
    ap.add_argument("--iters", type=int, default=500)
    a = ap.parse_args()
    import torch

    import bench
    from tests.helpers import expect_success, make_training_config

    args = bench.parse(["--config", a.config])
    dev = torch.device("cuda", 0)
    pricer, _ = bench.make_pricer(args, dev)
    B = bench.CONFIGS[a.config][0]
    session = expect_success(pricer.open_session(make_training_config(num_batches=10 ** 6, batch_size=B)))
    for _ in range(5):
        expect_success(session.step())
    torch.cuda.synchronize()
    prog, eng = session.program, session.engine
    ms, ns = session.mc_streams[0], session.stream
    h_ms, h_ns = ms.cuda_stream, ns.cuda_stream
    ev = torch.cuda.Event()
    ev.record(ms)

    def timed(name: str, fn) -> None:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        dt = (time.perf_counter() - t0) / a.iters * 1e6
        torch.cuda.synchronize()
        print(f"{name:48s} {dt:7.1f} us/call", flush=True)

    print(f"config {a.config}: kernel {eng.kernel_name}, explicit streams {prog.explicit_streams}, "
          f"captured {prog.captured}")
    timed("ptr(tensor) x 1", lambda: eng.buffers.targets.data_ptr())
    timed("torch.cuda.current_stream()", lambda: torch.cuda.current_stream())
    timed("Event.record(stream)", lambda: ev.record(ms))
    timed("Stream.wait_event(event)", lambda: ns.wait_event(ev))
    timed("Event(enable_timing) x2 + record x2", lambda: (torch.cuda.Event(enable_timing=True).record(ms),
                                                         torch.cuda.Event(enable_timing=True).record(ms)))
    def ctx():
        with torch.cuda.stream(ms):
            pass

    timed("with torch.cuda.stream(s): pass", ctx)
    slot = [0]

    def mc():
        prog.mc(slot[0] % 4, h_ms)
        slot[0] += 1

    timed("MC launch (enqueue_step, explicit stream)", mc)

    def nn():
        prog.fwd_bwd(slot[0] % 4, h_ns)
        slot[0] += 1

    timed("network launch (fused fwd_bwd, explicit stream)", nn)
    session.sync()
    timed("TrainingSession.step() (no live timing)", lambda: expect_success(session.step()))
    session.mc_events = []
    timed("TrainingSession.step() (live timing, new events)", lambda: expect_success(session.step()))
    pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters + 2)]
    for e0, e1 in pool:
        e0.record()
        e1.record()
    torch.cuda.synchronize()
    session.mc_event_pool = pool
    timed("TrainingSession.step() (live timing, event pool)", lambda: expect_success(session.step()))
    session.close()


if __name__ == "__main__":
    main()
