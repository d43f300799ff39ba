"""Kernel-only driver for rocprofv3: the MC part of one training step exactly as the trainer enqueues
it — smc_train_step (Sobol draw + path/CF kernel + cursor advance; resident_kernel at C2, its sliced
form at C3) — `--iters` times after one warm-up, no CVNN.

    rocprofv3 --kernel-trace --pmc WRITE_SIZE -- python tools/kprof_step.py --config c3
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

SHAPES = {"c2": (4096, 16, 256, 256), "c3": (16384, 16, 1024, 256), "e2e": (4096, 16, 128, 4),
          "lockstep": (4096, 1, 16, 4096)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--B", type=int, default=0, help="contracts per step (default: the config's)")
    ap.add_argument("--math", default="hw", choices=["hw", "portable", "reference", "reference_hw"])
    ap.add_argument("--store", default="all", choices=["all", "terminal"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--budget-gb", type=float, default=0.0,
                    help="path scratch budget (0: the engine's, engine.path_buffer_budget: half the HBM)")
    ap.add_argument("--pitch", type=int, default=0, help="row pitch in elements (0: smc_path_pitch)")
    ap.add_argument("--lanes", type=int, default=1, help="launches alternate over this many streams, each with "
                    "its own cursor, sync area and path scratch (consecutive launches may overlap)")
    ap.add_argument("--split", type=int, default=0, help="each call: this many concurrent launches of B / split "
                    "contracts, each on its own CU-masked stream of 1 / split of the CUs (every XCD in each)")
    ap.add_argument("--cus", type=int, default=0, help="run every lane on a CU-masked stream of this many CUs")
    ap.add_argument("--stream", default="current", choices=["current", "created", "high", "low"],
                    help="lane 0's stream: torch's current stream, or a created one (high: priority -1)")
    ap.add_argument("--one-stream", action="store_true", help="--lanes buffers and sync areas, all on one stream")
    ap.add_argument("--dynamic", action="store_true", help="SMC_TRAIN_DYNAMIC: every contract from the queue")
    ap.add_argument("--trace", default="", help="trace variant library (tools/micro/trace_variant.sh): after the timed "
                    "loop run one launch alone and save its per-workgroup timestamps to this .npy file")
    ap.add_argument("--trace-timed", default="", help="trace variant library: save the per-workgroup stamps of the "
                    "timed launches (16 slots of 256 workgroups, one per launch) to this .npy")
    ap.add_argument("--norm", default="", choices=["", "raw", "normalize"],
                    help="targets normalisation (default: RAW for the lock-step shape, else NORMALIZE)")
    a = ap.parse_args()
    B, T, N, M = SHAPES[a.config]
    B = a.B or B
    if a.split:  # one call = a.split concurrent launches of B / a.split contracts on complementary CU-masked streams
        B //= a.split
        a.lanes = a.split
    P = N * M
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    f64 = a.dtype == "f64"
    dcode = _lib.DTYPE_F64 if f64 else _lib.DTYPE_F32
    store = _lib.STORE_ALL if a.store == "all" else _lib.STORE_TERMINAL
    pitch = a.pitch or int(L.smc_path_pitch(P, dcode))
    esz = 8 if f64 else 4
    per = (T if store == _lib.STORE_ALL else 1) * pitch * esz
    from spectralmc_amd.engine import path_buffer_budget

    budget = int(a.budget_gb * (1 << 30)) if a.budget_gb else path_buffer_budget(dev)
    chunk = max(1, min(B, budget // per))
    if chunk < B:  # the engine's rounding: whole rounds of resident workgroups (2 per CU)
        slots = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
        if chunk >= slots:
            chunk -= chunk % slots
    launches = -(-B // chunk)
    chunk = -(-B // launches)
    lanes = a.lanes
    pathss = [torch.empty((chunk, T, pitch) if store == _lib.STORE_ALL else (chunk, pitch),
                          dtype=torch.float64 if f64 else torch.float32, device=dev) for _ in range(lanes)]
    eng = SobolEngine(6, 7, 0)
    tables = torch.from_numpy(eng.tables().view(np.int32)).to(dev)
    lo = torch.tensor([0.001, 0.001, 0.0, -0.2, -0.2, 0.0], dtype=torch.float64, device=dev)
    hi = torch.tensor([1e4, 2e4, 10.0, 0.2, 0.2, 2.0], dtype=torch.float64, device=dev)
    cur = torch.tensor([[k * B, k * B] for k in range(lanes)], dtype=torch.int64, device=dev)
    c = torch.empty((B, 6), dtype=torch.float64, device=dev)
    f = torch.empty((B, 6), dtype=torch.float32, device=dev)
    t = torch.empty((B, N), dtype=torch.complex128 if f64 else torch.complex64, device=dev)
    nsync = int(L.smc_train_step_sync_bytes(T, N, M, dcode, pitch))
    syncs = [torch.zeros(max(nsync, 8), dtype=torch.uint8, device=dev) for _ in range(lanes)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(lanes - 1)]
    owned: list[int] = []
    if a.split:
        from spectralmc_amd.gbm_trainer import _masked_stream

        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        per_lane = ncu // a.split
        streams = []
        for k in range(a.split):
            mask = [0] * ((ncu + 31) // 32)
            for cu in range(k * per_lane, (k + 1) * per_lane):  # logical ids interleave the XCDs (gbm_trainer._cu_masks)
                mask[cu // 32] |= 1 << (cu % 32)
            streams.append(_masked_stream(dev, mask, owned))
    if a.cus:  # every lane on a stream masked to logical CUs [0, cus): cus / 32 CUs of every shader engine
        from spectralmc_amd.gbm_trainer import _masked_stream

        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        mask = [0] * ((ncu + 31) // 32)
        for cu in range(a.cus):
            mask[cu // 32] |= 1 << (cu % 32)
        streams = [_masked_stream(dev, mask, owned) for _ in range(lanes)]
    elif a.stream != "current":  # lane 0 on a created stream instead of torch's current (default) stream
        prio = {"created": 0, "high": -1, "low": 0}[a.stream]
        streams[0] = torch.cuda.Stream(priority=prio)
        streams[0].wait_stream(torch.cuda.current_stream())
    if a.one_stream:  # the lanes' buffers, one stream: launches serialised, rotating over the path buffers
        streams = [torch.cuda.current_stream()] * lanes
    scheme = _lib.SCHEME_LOG_EULER | {"hw": _lib.MATH_HW, "reference": _lib.MATH_REF,
                                        "reference_hw": _lib.MATH_REF | _lib.MATH_HW}.get(a.math, 0) | \
        (_lib.TRAIN_DYNAMIC if a.dynamic else 0)
    n_launched = [0]
    raw = a.norm == "raw" or (a.norm == "" and a.config == "lockstep")
    norm = _lib.NORM_RAW if raw else _lib.NORM_NORMALIZE

    def step():
        k = n_launched[0] % lanes
        n_launched[0] += 1
        _lib.check(L.smc_train_step(_lib.ptr(tables), 6, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(cur[k]), 0, lanes * B,
                                    _lib.ptr(c), None if f64 else _lib.ptr(f), B, T, N, M, 7, scheme,
                                    norm, dcode, store, _lib.ptr(pathss[k]), pitch, chunk, _lib.ptr(t),
                                    _lib.ptr(syncs[k]), nsync, _lib.stream_handle(streams[k])))

    for _ in range(lanes):
        step()
    torch.cuda.synchronize()
    if a.trace_timed:  # trace the timed launches themselves (16 slots of 256 workgroups by launch)
        import ctypes

        tbuf = np.zeros((4096, 40), dtype=np.uint64)
        L.smc_trace_copy.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        assert L.smc_trace_copy(tbuf.ctypes.data, 1) == 0
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s_ in streams:
        if s_ is not torch.cuda.current_stream():
            s_.wait_stream(torch.cuda.current_stream())
    for _ in range(a.iters * (a.split or 1)):
        step()
    for s_ in streams:
        if s_ is not torch.cuda.current_stream():
            torch.cuda.current_stream().wait_stream(s_)
    e1.record()
    torch.cuda.synchronize()
    assert all(_lib.sync_status(sy) == 0 for sy in syncs)
    name = L.smc_train_step_kernel(T, N, M, dcode | (_lib.QUERY_RAW if raw else 0) |
                                   (_lib.MATH_REF if a.math.startswith("reference") else 0), pitch).decode()
    ms = e0.elapsed_time(e1) / a.iters  # per call (a.split launches with --split)
    if a.trace_timed:
        assert L.smc_trace_copy(tbuf.ctypes.data, 0) == 0
        np.save(a.trace_timed, tbuf)
    if a.trace:
        import ctypes

        buf = np.zeros((4096, 40), dtype=np.uint64)
        L.smc_trace_copy.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        assert L.smc_trace_copy(buf.ctypes.data, 1) == 0
        torch.cuda.synchronize()
        # one launch alone, or (lanes > 1) 4 consecutive launches in flight, traced in slots by launch (ord / B mod 4)
        for s_ in streams[1:]:
            s_.wait_stream(torch.cuda.current_stream())
        for _ in range(1 if lanes == 1 else 4):
            step()
        torch.cuda.synchronize()
        assert L.smc_trace_copy(buf.ctypes.data, 0) == 0
        np.save(a.trace, buf)
        for k in range(16):
            if buf[k * 256:(k + 1) * 256, 39].any():
                print(f"-- trace slot {k}")
                summarize(buf[k * 256:(k + 1) * 256])
    print(f"{a.config} {'raw' if raw else 'normalize'} pitch={pitch} B={B} T={T} N={N} M={M} {a.dtype} {a.math} {a.store} {name}: {ms:.3f} ms/step "
          f"({launches} launch(es) of {chunk}), checksum {float(t.abs().double().mean()):.6g}")


def summarize(buf: np.ndarray) -> None:
    """Per-workgroup timeline of one launch (trace variant): start spread, per-XCD end times, idle tail."""
    used = buf[:, 39] > 0
    t = buf[used].astype(np.int64)
    us = 0.01  # s_memrealtime: 100 MHz
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) * us, (t[:, 39] - t0) * us
    span = end.max()
    print(f"trace: {used.sum()} workgroups, span {span:.1f} us, starts {start.min():.1f}..{start.max():.1f} us, "
          f"ends {end.min():.1f}..{end.max():.1f} us, mean idle tail {np.mean(span - end):.1f} us "
          f"({np.mean(span - end) / span:.2%} of the CU-time)")
    rounds = t[:, 38]
    print(f"  contracts per workgroup: min {rounds.min()} max {rounds.max()} mean {rounds.mean():.2f}")
    for x in sorted(set(t[:, 1].tolist())):
        m = t[:, 1] == x
        per = (t[m, 39] - t[m, 0]) * us / np.maximum(rounds[m], 1)
        print(f"  XCC {x}: {m.sum()} WGs, end {end[m].min():.1f}..{end[m].max():.1f} us, "
              f"{per.mean():.1f} us per contract, contracts {rounds[m].min()}..{rounds[m].max()}")
    first = (t[:, 2] - t[:, 0]) * us
    print(f"  first contract {first.mean():.1f} us (min {first.min():.1f} max {first.max():.1f})")
    last_start = np.array([(t[i, 2 + min(r, 34) - 2] if r >= 2 else t[i, 0]) for i, r in enumerate(rounds)], dtype=np.int64)
    print(f"  last contract starts {((last_start - t0) * us).min():.1f}..{((last_start - t0) * us).max():.1f} us")


if __name__ == "__main__":
    main()
