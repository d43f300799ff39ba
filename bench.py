"""Benchmark: GbmCVNNPricer training steps on MI355X (BASELINE.json metric / config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1] [--store all|terminal]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one full training step (reference gbm_trainer.py:1532-1597): Sobol draw of B
contracts, GBM simulation of P paths x T steps per contract (full [B][T][P] path matrix
written to HBM, the reference kernel's output contract), forward normalisation, put payoff,
M-batch mean + N-point DFT -> targets, CVNN forward/backward, Adam, grad norm.  Weak scaling:
every rank processes B contracts per step (contract-sharded data parallel, one RCCL all-reduce).

Rank 0 prints ONE JSON line.  `value` = contracts x paths per second over the whole job.
The roofline object is for the dominant kernel (the MC part of the step: resident_kernel at C2,
its sliced form at C3, basket_resident_kernel at C5): algorithmic bytes per launch over the
launch's duration, timed with HIP events on its own stream right after the timed region (`kernel_ms`;
`kernel_ms_live` / `kernel_ms_steady`: the launches inside the timed region).  `cpu_baseline` is the
reference CPU path (torch-cpu + numpy.fft, oracle/torch_cpu.py) on a bounded sample, with the
C/OpenMP oracle as a second leg and C1 timed over 10 whole steps.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (B per GPU, T, N, M, hidden widths, description)
    "c1": (64, 16, 256, 4, [32], "C1: 64 contracts x 1024 paths (N=256 x M=4), T=16, 2-layer CVNN 6->32->256 fp32"),
    "c2": (4096, 16, 256, 256, [32, 32],
           "C2: 4096 contracts x 65536 paths (N=256 x M=256), T=16, 3-layer CVNN 6->32->32->256 fp32"),
    # SURVEY 8(d) C2 "H=256 variant for MFMA": the same step with 256-wide hidden layers (267,264 params)
    "c2h256": (4096, 16, 256, 256, [256, 256],
               "C2/H=256: 4096 contracts x 65536 paths (N=256 x M=256), T=16, 3-layer CVNN 6->256->256->256 fp32"),
    # BASELINE configs[2]: bf16 CVNN (bf16 MFMA operands, f32 master weights / Adam: an extension, the
    # reference accepts full precision only, gbm_trainer.py:679-686); 275 GB of paths per step run as
    # equal launches through the scratch
    "c3": (16384, 16, 1024, 256, [32, 32],
           "C3: 16384 contracts x 262144 paths (N=1024 x M=256), T=16, 3-layer CVNN 6->32->32->1024 bf16 "
           "(f32 master weights)"),
    # BASELINE configs[4] (per GPU): 4 correlated assets (Cholesky in LDS), equal-weight basket put
    "c5": (8192, 16, 256, 512, [32, 32],
           "C5: 8192 contracts x 131072 paths (N=256 x M=512), 4 correlated assets, T=16, basket put, "
           "3-layer CVNN 16->32->32->256 fp32"),
    # the reference's other legal shapes (not BASELINE configs; parity-tested, timed for coverage):
    # the lock-step trainer shape (tests/test_gbm_trainer.py:122-131, T = 1, N = 16, M = 4096) at C2's
    # batch, and C2 in float64 (Precision.float64: f64 paths, complex128 targets, f64 CVNN)
    "lockstep": (4096, 1, 16, 4096, [32, 32],
                 "lock-step shape: 4096 contracts x 65536 paths (N=16 x M=4096), T=1, LOG_EULER + RAW, 3-layer CVNN "
                 "6->32->32->16 fp32"),
    # the reference's e2e shape (tests/test_e2e/test_full_stack_cvnn_pricer.py:40-51: T = 16, N = 128, M = 4)
    # at C2's batch: P = 512, packed_kernel (8 contracts per workgroup)
    "e2e": (4096, 16, 128, 4, [32],
            "e2e shape: 4096 contracts x 512 paths (N=128 x M=4), T=16, 2-layer CVNN 6->32->128 fp32"),
    "c2f64": (4096, 16, 256, 256, [32, 32],
              "C2 in float64: 4096 contracts x 65536 paths (N=256 x M=256), T=16, 3-layer CVNN 6->32->32->256 fp64"),
}
SIM_DTYPE = {"c2f64": "float64"}  # default float32
RAW_NORMALIZATION = {"lockstep"}  # ForwardNormalization.RAW (reference tests/test_gbm_trainer.py:138-142)
BASKET_ASSETS = {"c5": 4}
NETWORK_COMPUTE = {"c3": "bf16"}  # default "auto": f32 on the f32 MFMA kernels
MFMA_PEAK_TFLOPS = {"mfma_bf16": 2516.6, "mfma_f32": 157.3, "valu": 157.3}  # MI355X_MICROARCH.md, dense


def parse(argv: list[str] | None = None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); N > 1 without a launcher starts the N ranks itself")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1: nccl (= RCCL over xGMI) or gloo (rehearsal: with fewer "
                         "GPUs than ranks, rank r runs on GPU r mod device_count)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--store", default="all", choices=["all", "terminal"])
    ap.add_argument("--math", default="hw", choices=["portable", "hw", "reference", "reference_hw"],
                    help="path math: hw (hardware f32 transcendentals), portable (CPU-reproducible f32), reference "
                         "(the reference kernel's typing: f64 state and step, f32 normals and stores; float32 configs), "
                         "reference_hw (that step on the hardware-transcendental normals)")
    ap.add_argument("--network", default=None, choices=["auto", "valu", "mfma", "bf16"],
                    help="network kernels (default: bf16 for c3, auto otherwise)")
    ap.add_argument("--overlap-rows", default="auto", choices=["auto", "on", "off"],
                    help="pricer.overlap_rows: the rows_kernel / rows_ref_kernel steps' network beside the next rows "
                         "launch (auto: f64 overlapped, the reference typing on one stream)")
    ap.add_argument("--overlap", default="on", choices=["on", "off"],
                    help="MC part of step s+1 on its own stream beside step s's network part (pricer.overlap_mc)")
    ap.add_argument("--priority", default="network", choices=["network", "mc", "none"],
                    help="stream with the high queue priority (pricer.high_priority_stream)")
    ap.add_argument("--lanes-long", type=int, default=None,
                    help="pricer.mc_lanes_long (MC lanes for long path launches beside a narrow network)")
    ap.add_argument("--lanes", type=int, default=2, choices=[1, 2, 4], help="MC lanes (pricer.mc_lanes): consecutive path launches "
                    "on alternating streams, each starting in the previous one's tail")
    ap.add_argument("--lanes-short", type=int, default=None,
                    help="pricer.mc_lanes_short (MC lanes for launches below --net-cu-min-path-steps)")
    ap.add_argument("--net-cus", type=int, default=32, help="CUs reserved for the network (pricer.network_cus)")
    ap.add_argument("--exchanging-masks", default="auto", choices=["auto", "on", "off"],
                    help="CU-masked network stream beside the exchanging C3 / C5 launches (pricer.exchanging_masks; "
                         "auto: data-parallel runs only)")
    ap.add_argument("--net-cus-small", type=int, default=None,
                    help="pricer.network_cus_small (network CUs beside launches below --net-cu-min-path-steps)")
    ap.add_argument("--net-cu-min-path-steps", type=int, default=None,
                    help="pricer.network_cu_min_path_steps (CU masks only for launches of at least this many path-steps)")
    ap.add_argument("--net-cus-wide", type=int, default=64,
                    help="CUs reserved for a wide (layered GEMM) network (pricer.network_cus_wide)")
    ap.add_argument("--net-cu-pattern", default="low", choices=["spread", "low"])
    ap.add_argument("--graphs", default="on", choices=["on", "off"], help="replay the step as hipGraphs")
    ap.add_argument("--kernel-iters", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget for the CPU-baseline sample")
    return ap.parse_args(argv)


ON_CHIP_KERNELS = ("resident_kernel", "wave_kernel", "packed_kernel", "basket_resident_kernel")


def algorithmic_bytes_per_contract(T: int, N: int, M: int, store_all: bool, esz: int = 4) -> int:
    """path matrix store + terminal-row re-read + complex targets (+ 48 B contract in);
    esz = 4 (f32 paths, complex64 targets) or 8 (f64, complex128)."""
    P = N * M
    return (T * P * esz if store_all else P * esz) + P * esz + N * 2 * esz


def progress(msg: str) -> None:
    """A progress line on stderr (stdout carries only the JSON line): long CPU legs stay visibly alive."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_threads() -> int:
    """Host threads for the CPU legs: the process's affinity set, capped by OMP_NUM_THREADS (the
    GPU box gives one GPU's job a 16-core share; os.cpu_count() there is the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(B: int, T: int, N: int, M: int, widths: list[int], budget_s: float, n_assets: int = 0,
                 dtype: str = "float32", normalize: bool = True) -> dict:
    """The reference CPU path (north_star: torch-cpu + numpy.fft; oracle/torch_cpu.py) timed on the
    host cores: MC for a time-boxed sample of the B contracts (extrapolated to B) + one full-size
    CVNN/Adam step on torch-cpu; plus C1 (BASELINE configs[0]) timed over 10 whole steps, and the
    C/OpenMP oracle as a second, separately labelled leg."""
    import numpy as np
    import torch

    import oracle
    from oracle.torch_cpu import cpu_path_targets, cpu_training_step
    from tests.helpers import make_domain_bounds, make_test_cvnn

    oracle.build()
    threads = cpu_threads()
    torch.set_num_threads(threads)
    if n_assets:
        from spectralmc_amd.basket import BasketConfig

        lo, hi = BasketConfig(n_assets=n_assets, timesteps=T, network_size=N, batches_per_mc_run=M).arrays()
    else:
        lo, hi = make_domain_bounds().arrays()
    contracts = oracle.sobol_contracts(7, 0, B, lo, hi)

    def sample(fn, budget: float, chunk: int) -> tuple[float, int, list]:
        done, t_mc, out = 0, 0.0, []
        while done < B and t_mc < budget:
            n = min(chunk, B - done)
            t0 = time.perf_counter()
            out.append(fn(contracts[done:done + n], done))
            t_mc += time.perf_counter() - t0
            done += n
        return t_mc / done, done, out

    if n_assets:  # kernel-mode basket restatement (the basket has no reference-mode CPU path)
        per_c, done, tg = sample(lambda c, o: oracle.basket_kernel(c, n_assets, T, N, M, 7, ordinal0=o)[2],
                                 budget_s * 0.8, threads)
        path = "oracle C basket kernel-mode (f32)"
    else:
        per_c, done, tg = sample(lambda c, o: cpu_path_targets(c, T, N, M, 7, o, dtype=dtype, normals="numpy",
                                                               normalize=normalize),
                                 budget_s * 0.6, 2 * threads)
        path = ("torch-cpu paths (f64 recursion, numpy default_rng normals per contract) + numpy.fft "
                "(oracle/torch_cpu.py)")
    tdt = torch.float64 if dtype == "float64" else torch.float32
    model = make_test_cvnn(n_inputs=contracts.shape[1], n_outputs=N, seed=123, dtype=tdt, device="cpu",
                           hidden_layers=len(widths), hidden_width=widths[0])
    adam = torch.optim.Adam(model.parameters(), lr=1e-2)
    x = torch.tensor(contracts, dtype=tdt)
    tgt = torch.from_numpy(np.concatenate(tg))
    tgt = tgt.repeat((B + tgt.shape[0] - 1) // tgt.shape[0], 1)[:B]
    oracle.torch_step(model, x, torch.zeros_like(x), tgt, adam)  # warm
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        oracle.torch_step(model, x, torch.zeros_like(x), tgt, adam)
    t_nn = (time.perf_counter() - t0) / reps
    step_s = per_c * B + t_nn
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    line = {
        "value": B * N * M / step_s,
        "unit": "contracts*paths/s",
        "steps_per_sec": 1.0 / step_s,
        "cores": threads,
        "affinity_cores": len(os.sched_getaffinity(0)),
        "machine_cores": os.cpu_count(),
        "kind": "port",
        "sample": (f"{path}, {threads} threads, on {done}/{B} contracts x {N * M} paths x T={T} "
                   f"({per_c * done:.1f}s), extrapolated x{B / done:.1f}, + full B={B} CVNN/Adam step on torch-cpu "
                   f"({t_nn * 1e3:.1f} ms)"),
        "cpu_model": cpu_model,
    }
    # the same leg on every core of the process's affinity set (BASELINE.md section 2.2 plans
    # torch.set_num_threads(len(os.sched_getaffinity(0)))): the GPU box shows the whole host there, while one
    # GPU's job gets a 16-core share (OMP_NUM_THREADS), which the leg above uses
    aff = len(os.sched_getaffinity(0))
    progress(f"cpu_baseline: {threads}-thread leg done ({per_c * done + t_nn * reps:.1f} s)")
    if aff != threads and not n_assets:
        # contract-level parallelism over the affinity set: one worker thread per core, each contract's torch ops
        # single-threaded (nested intra-op pools of `aff` threads in each of `aff` workers oversubscribe a shared
        # host by aff^2); the CVNN/Adam step on up to 64 intra-op threads
        workers = min(aff, 256)
        nn_threads = min(aff, 64)
        torch.set_num_threads(1)
        try:
            per_a, done_a, _ = sample(lambda c, o: cpu_path_targets(c, T, N, M, 7, o, dtype=dtype, normals="numpy",
                                                                    normalize=normalize, workers=workers),
                                      budget_s * 0.4, 2 * workers)
            torch.set_num_threads(nn_threads)
            oracle.torch_step(model, x, torch.zeros_like(x), tgt, adam)  # warm at this thread count
            t0 = time.perf_counter()
            for _ in range(reps):
                oracle.torch_step(model, x, torch.zeros_like(x), tgt, adam)
            t_nn_a = (time.perf_counter() - t0) / reps
        finally:
            torch.set_num_threads(threads)
        line["affinity_leg"] = {
            "value": B * N * M / (per_a * B + t_nn_a), "unit": "contracts*paths/s", "cores": workers, "kind": "port",
            "sample": (f"{path}, {workers} worker threads over the process's {aff}-core affinity set (BASELINE.md 2.2: "
                       f"len(os.sched_getaffinity(0))), one single-threaded contract each, on {done_a}/{B} contracts "
                       f"({per_a * done_a:.1f}s), extrapolated x{B / done_a:.1f}, + full B={B} CVNN/Adam step on "
                       f"{nn_threads} threads ({t_nn_a * 1e3:.1f} ms)")}
        progress(f"cpu_baseline: affinity leg done ({per_a * done_a + t_nn_a * reps:.1f} s)")
    else:
        line["affinity_leg"] = {"value": line["value"], "unit": "contracts*paths/s", "cores": aff, "kind": "port",
                                "sample": "the affinity set is the leg above's thread count" if aff == threads else
                                "basket: kernel-mode C oracle leg only"}
    if not n_assets:
        # second leg: the C/OpenMP oracle (f64 recursion, this build's normal streams)
        per_c2, done2, _ = sample(lambda c, o: oracle.training_targets(c, T, N, M, seed=7, ordinal0=o, dtype=dtype,
                                                                       normalize=normalize),
                                  budget_s * 0.2, threads)
        line["c_openmp_leg"] = {"value": B * N * M / (per_c2 * B + t_nn), "unit": "contracts*paths/s",
                                "cores": threads, "kind": "port",
                                "sample": f"oracle/gbm_oracle.c (OpenMP) on {done2}/{B} contracts, extrapolated"}
        progress("cpu_baseline: C/OpenMP leg done")
        # C1, the reference's own CPU-runnable config (BASELINE configs[0]): 10 whole steps
        c1B, c1N, c1M = 64, 256, 4
        m1 = make_test_cvnn(n_inputs=6, n_outputs=c1N, seed=123, dtype=torch.float32, device="cpu", hidden_layers=1)
        a1 = torch.optim.Adam(m1.parameters(), lr=1e-2)
        c1 = oracle.sobol_contracts(7, 0, 11 * c1B, lo, hi)
        cpu_training_step(m1, a1, c1[:c1B], T, c1N, c1M, 7, 0, normals="numpy")  # warm-up step
        t0 = time.perf_counter()
        for s in range(1, 11):
            cpu_training_step(m1, a1, c1[s * c1B:(s + 1) * c1B], T, c1N, c1M, 7, s * c1B, normals="numpy")
        t1 = (time.perf_counter() - t0) / 10
        line["c1"] = {"steps_per_sec": 1.0 / t1, "value": c1B * c1N * c1M / t1, "unit": "contracts*paths/s",
                      "ms_per_step": t1 * 1e3, "steps": 10, "warmup": 1,
                      "workload": "C1: 64 contracts x 1024 paths (N=256 x M=4), T=16, 2-layer CVNN 6->32->256, "
                                  "torch-cpu + numpy.fft, whole steps"}
        progress(f"cpu_baseline: C1 done ({t1 * 11:.1f} s)")
    return line


def make_pricer(args: argparse.Namespace, dev):
    """The pricer of one bench configuration with the bench's step policy (MC lanes, CU-masked network
    stream, graphs, math mode ...) set from ``args`` (``parse([])`` gives the defaults the driver runs);
    tests/test_gpu_c2_session.py trains this exact object against the oracle.  Returns (pricer, model)."""
    import torch

    from spectralmc_amd.gbm import ForwardNormalization
    from spectralmc_amd.gbm_trainer import GbmCVNNPricer
    from spectralmc_amd.models.numerical import Precision
    from tests.helpers import (
        expect_success,
        make_black_scholes_config,
        make_domain_bounds,
        make_gbm_cvnn_config,
        make_simulation_params,
        make_test_cvnn,
    )

    B, T, N, M, widths, desc = CONFIGS[args.config]
    f64 = SIM_DTYPE.get(args.config) == "float64"
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256,
                                mc_seed=7, buffer_size=512, dtype=Precision.float64 if f64 else Precision.float32)
    n_assets = BASKET_ASSETS.get(args.config, 0)
    n_inputs = 3 * n_assets + 4 if n_assets else 6
    model = make_test_cvnn(n_inputs=n_inputs, n_outputs=N, seed=123, dtype=torch.float64 if f64 else torch.float32,
                           device=dev, hidden_layers=len(widths), hidden_width=widths[0])
    norm = ForwardNormalization.RAW if args.config in RAW_NORMALIZATION else ForwardNormalization.NORMALIZE
    cfg = make_gbm_cvnn_config(model, sim_params=sp,
                               bs_config=make_black_scholes_config(sim_params=sp, normalization=norm),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.store_paths = args.store == "all"
    pricer.math_mode = args.math
    pricer.warmup_steps = max(1, min(2, args.warmup)) if args.graphs == "on" else 0
    pricer.network_compute = args.network or NETWORK_COMPUTE.get(args.config, "auto")
    pricer.overlap_mc = args.overlap == "on"
    pricer.overlap_rows = {"auto": None, "on": True, "off": False}[args.overlap_rows]
    pricer.high_priority_stream = args.priority
    pricer.mc_lanes = args.lanes
    if args.lanes_long is not None:
        pricer.mc_lanes_long = args.lanes_long
    if args.lanes_short is not None:
        pricer.mc_lanes_short = args.lanes_short
    pricer.network_cus = args.net_cus
    pricer.exchanging_masks = {"auto": None, "on": True, "off": False}[args.exchanging_masks]
    pricer.network_cus_wide = args.net_cus_wide
    pricer.network_cu_pattern = args.net_cu_pattern
    if args.net_cus_small is not None:
        pricer.network_cus_small = args.net_cus_small
    if args.net_cu_min_path_steps is not None:
        pricer.network_cu_min_path_steps = args.net_cu_min_path_steps
    if n_assets:
        from spectralmc_amd.basket import BasketConfig, use_basket_engine

        use_basket_engine(pricer, BasketConfig(n_assets=n_assets, timesteps=T, network_size=N, batches_per_mc_run=M,
                                               mc_seed=7, math=args.math), store_paths=pricer.store_paths)
    return pricer, model


def launcher_command(argv: list[str], gpus: int, port: int, script: str | None = None) -> list[str]:
    """The torch.distributed.run command that starts `gpus` ranks of this script with the same arguments
    (the driver's own form: one node, 127.0.0.1 rendezvous)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__), *argv]


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return int(sk.getsockname()[1])


def maybe_launch_ranks(args: argparse.Namespace, argv: list[str], script: str | None = None) -> int | None:
    """`bench.py --gpus N` (N > 1) started without a launcher (no WORLD_SIZE in the environment): run the
    N ranks as ONE child process tree through torch.distributed.run and return its exit code.  Called
    before anything touches the GPU (this process only waits); None when this process is a rank or N = 1."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    return subprocess.call(launcher_command(argv, args.gpus, free_port(), script), env=env)


def main() -> None:
    argv = sys.argv[1:]
    args = parse(argv)
    rc = maybe_launch_ranks(args, argv)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    from spectralmc_amd import _lib, dp
    from tests.helpers import expect_success, make_training_config

    if args.backend == "gloo" and "LOCAL_RANK" in os.environ:  # rehearsal: rank r on GPU r mod #GPUs
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]) % max(1, torch.cuda.device_count()))
    ctx = dp.init_from_env(backend=args.backend if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    world = ctx.world_size if ctx else 1
    rank = ctx.rank if ctx else 0
    if world != args.gpus:
        # a line for another world size than asked would be mislabelled in the driver's scaling table
        print(f"bench.py: --gpus {args.gpus} but the job has {world} rank(s)", file=sys.stderr)
        sys.exit(3)
    dev = torch.device("cuda", torch.cuda.current_device())

    B, T, N, M, widths, desc = CONFIGS[args.config]
    P = N * M
    f64 = SIM_DTYPE.get(args.config) == "float64"
    esz = 8 if f64 else 4
    n_assets = BASKET_ASSETS.get(args.config, 0)
    n_inputs = 3 * n_assets + 4 if n_assets else 6
    pricer, model = make_pricer(args, dev)
    tcfg = make_training_config(num_batches=args.warmup + args.steps, batch_size=B, learning_rate=1e-2)
    session = expect_success(pricer.open_session(tcfg))

    for _ in range(args.warmup):
        expect_success(session.step())
    session.sync()
    if ctx:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events around each MC-part launch on its stream (timed region), created and recorded once beforehand
    pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps + 2)]
    for e0, e1 in pool:
        e0.record()
        e1.record()
    torch.cuda.synchronize()
    session.mc_event_pool = pool[::-1]
    session.mc_events = []
    if ctx:
        session.program.ar_events = []  # ... and around each step's all-reduce on the network stream
    t0 = time.perf_counter()
    for _ in range(args.steps):
        expect_success(session.step())
    t_enq = time.perf_counter() - t0  # host time to enqueue the K steps (the host limits the step when ~ elapsed)
    session.sync()
    torch.cuda.synchronize()
    if ctx:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ctx:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final = session.close()

    # ---- data parallel: the step's one all-reduce (flat [grads..., loss] buffer) -----------------
    data_parallel = None
    if ctx:
        ar = [a.elapsed_time(b_) for a, b_ in (session.program.ar_events or [])]
        flat = session.program.flat.clone()
        s_ar = torch.cuda.Stream(device=dev)
        iters = 20
        dist.barrier()
        with torch.cuda.stream(s_ar):
            ctx.all_reduce_mean(flat)  # warm
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record(s_ar)
            for _ in range(iters):
                ctx.all_reduce_mean(flat)
            a1.record(s_ar)
        a1.synchronize()
        iso = torch.tensor([a0.elapsed_time(a1) / iters], dtype=torch.float64, device=dev)
        dist.all_reduce(iso, op=dist.ReduceOp.MAX)
        data_parallel = {"backend": args.backend, "world": world,
                         "rccl_world": world if args.backend == "nccl" else None,
                         "allreduce_bytes": flat.numel() * flat.element_size(),
                         "allreduce_per_step": 1,
                         "allreduce_ms_in_step": (sum(ar) / len(ar)) if ar else None,
                         "allreduce_ms_isolated": float(iso.item()),
                         "collective_stream": ("the step's network stream (dp.RcclComm: ncclAllReduce on it, CU-masked "
                                               "with the network)" if ctx.comm is not None else
                                               "torch.distributed's internal stream"),
                         "note": "allreduce_ms_in_step: HIP events around each step's eager all-reduce (sum, then / "
                                 "world) on the network stream inside the timed region (rank 0); isolated: 20 "
                                 "back-to-back all-reduces of the same buffer after it, max over ranks"}

    # ---- dominant kernel, timed alone with HIP events on its own stream ----------------
    eng = session.engine
    stream = torch.cuda.Stream(device=dev)
    L = _lib.lib()
    launches_per_call = (eng.B + eng.chunk - 1) // eng.chunk
    prog = session.program
    # the contracts of the last timed step: the engine's own buffers are never drawn into when the steps
    # write their slots directly, and the path kernels run faster on all-zero contracts (C2-f64 rows_kernel
    # + cf_kernel: 7.43 ms on zeros, 8.04 ms on drawn contracts; profiles/r04/probe_gap_f64.txt)
    last = prog.slots[(session.steps - 1) % len(prog.slots)] if getattr(prog, "direct", False) else None
    with torch.cuda.stream(stream):

        def run_kernel() -> None:
            # the launch(es) the training step makes: smc_train_step (Sobol draw, targets and cursor
            # update fused into the resident kernel) where the engine uses it, else the targets call
            if getattr(eng, "_uses_train_step", False):
                eng.enqueue_step()
            else:
                eng.launch_targets(_lib.stream_handle(stream), None, 0, last)

        run_kernel()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(args.kernel_iters):
            run_kernel()
        ev1.record(stream)
    ev1.synchronize()
    kernel_ms_events = ev0.elapsed_time(ev1) / (args.kernel_iters * launches_per_call)
    # the same launches again, each call's kernels timed by their own execution timestamps (smc_time_launches:
    # hipExtLaunchKernel start / stop events, the figure a kernel trace gives, without the dispatch gap a pair
    # of stream events around back-to-back launches also holds: round 5's e2e line was +3.4 % against rocprof)
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             for _ in range(args.kernel_iters)]
    with torch.cuda.stream(stream):
        for t0_, t1_ in pairs:  # create the events (recorded once by torch), then arm them per call
            t0_.record(stream)
            t1_.record(stream)
        for t0_, t1_ in pairs:
            # each call alone (the stream drained first): a kernel queued behind the previous call's would take its
            # start timestamp while it still waits for it
            stream.synchronize()
            _lib.check(L.smc_time_launches(t0_.cuda_event, t1_.cuda_event))
            try:
                run_kernel()
            finally:
                _lib.check(L.smc_time_launches(None, None))
    stream.synchronize()
    kernel_ms = sum(t0_.elapsed_time(t1_) for t0_, t1_ in pairs) / (args.kernel_iters * launches_per_call)
    kernel_timing = (f"mean over {args.kernel_iters} calls, each alone on the drained stream, of the first kernel's "
                     "start to the last kernel's end (smc_time_launches: hipExtLaunchKernel events); kernel_ms_events: "
                     f"HIP events around the {args.kernel_iters} back-to-back calls")
    contracts_per_launch = min(eng.chunk, eng.B)
    if n_assets:
        bytes_survey = eng.algorithmic_bytes_per_contract() * contracts_per_launch
    else:
        bytes_survey = algorithmic_bytes_per_contract(T, N, M, pricer.store_paths, esz) * contracts_per_launch + \
            48 * contracts_per_launch
    # the kernel's own algorithmic bytes: SURVEY §8(d)'s per-contract figure counts a terminal-row re-read
    # (P values per asset) that the kernels keeping the terminal row on chip never make; for those the
    # figure with it would credit bytes nobody moves (at the lock-step shape it is twice the real
    # traffic and implies more than the HBM peak)
    on_chip = eng.kernel_name.split("(")[0] in ON_CHIP_KERNELS  # "resident_kernel(sliced)": C3
    reread = ((n_assets or 1) * P * (4 if n_assets else esz) * contracts_per_launch) if on_chip else 0
    bytes_launch = bytes_survey - reread
    # live: HIP events on the MC stream around each MC-part launch inside the timed region
    # (Sobol draw + path/CF kernel + cursor update; the path/CF kernel is >99 % of it)
    live = [a.elapsed_time(b_) for a, b_ in (session.mc_events or [])]
    live_ms = (sum(live) / len(live) / launches_per_call) if live else None
    lanes = getattr(eng, "lanes", 1)
    steady_ms = None
    if lanes > 1 and live:
        # MC lanes: step s + 1's launch starts in step s's tail, so an event pair around one launch also
        # spans its wait for CUs (no launch duration); the MC part's steady rate is the span of all live
        # launches over their number
        ev = session.mc_events
        steady_ms = ev[0][0].elapsed_time(ev[-1][1]) / len(ev) / launches_per_call
        live_ms = None
    # roofline: the launch's own duration, the same definition for every config (round 5; before, configs without
    # MC lanes used the live event pairs, which also hold launch gaps and the CUs the concurrent network takes):
    # the dominant launch alone, repeated on its own stream after the timed region -- the figure a rocprofv3
    # kernel trace of that launch shape reproduces (tools/kprof_step.py, profiles/r05)
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9

    # ---- network part alone (fused HIP kernels), HIP events on its own stream ------------
    network = None
    fused = session.program.fused
    if fused is not None:
        prog = session.program
        widths_all = [n_inputs] + list(widths) + [N]
        macs = sum(4 * a_ * b_ for a_, b_ in zip(widths_all[:-1], widths_all[1:]))  # complex = 4 real MACs
        macs_bwd = macs + sum(4 * a_ * b_ for a_, b_ in zip(widths_all[1:-1], widths_all[2:]))
        flops = 2.0 * (macs + macs_bwd) * B  # forward + weight grads + input grads (not layer 0)
        with torch.cuda.stream(stream):
            fused.fwd_bwd(prog.real_in[0], prog.imag_in, prog.targets[0])
            n0, n1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n0.record(stream)
            for _ in range(args.kernel_iters):
                fused.fwd_bwd(prog.real_in[0], prog.imag_in, prog.targets[0])
                if not fused.fuse_adam:
                    fused.adam()
            n1.record(stream)
        n1.synchronize()
        net_ms = n0.elapsed_time(n1) / args.kernel_iters
        kern = fused.kernels
        peak = 78.6 if (f64 and kern == "valu") else MFMA_PEAK_TFLOPS[kern]  # f64 vector peak (dense)
        layered = kern == "mfma_f32" and 2 * max(widths) >= 256  # csrc/cvnn_mfma.hip make_plan
        desc_k = {"mfma_bf16": "pack + fb + wgrad (csrc/cvnn_mfma.hip, v_mfma_f32_16x16x32_bf16, bf16 operands, "
                               "f32 accumulate / master weights) + reduce/Adam + finalize",
                  "mfma_f32": "pack + fb + wgrad (csrc/cvnn_mfma.hip, v_mfma_f32_16x16x4_f32) + reduce/Adam + "
                              "finalize",
                  "valu": "forward_backward + reduce/Adam + finalize (csrc/cvnn.hip), VALU "
                          + ("f64" if f64 else "f32")}[kern]
        if layered:
            desc_k = ("lpack + one lgemm_kernel per layer and direction (v_mfma_f32_16x16x4_f32, 64x64 tiles, "
                      "fused epilogues) + wgrad + reduce/Adam + finalize (csrc/cvnn_mfma.hip)")
        network = {"kernels": desc_k, "compute": kern, "flops_per_step": flops, "ms": net_ms,
                   "achieved": flops / (net_ms * 1e-3) / 1e12, "peak": peak, "unit": "TFLOP/s",
                   "frac": flops / (net_ms * 1e-3) / 1e12 / peak,
                   "peak_note": ("f64 vector peak 78.6 TF (dense), MI355X_MICROARCH.md" if peak == 78.6 else
                                 "dense MFMA peak of the operand type (bf16 2.52 PF; f32 MFMA = f32 VALU "
                                 "157.3 TF), MI355X_MICROARCH.md"),
                   "note": "small complex GEMMs (K = 12..512) plus the targets read, timed alone; " + (
                       "in the step it runs after the path kernel on the same stream (rows_kernel holds every "
                       "CU slot for its whole duration; gbm_trainer.py)"
                       if session.engine.kernel_name.startswith("rows_") or not pricer.overlap_mc else
                       "in the step it is enqueued on its own stream and its workgroups take the CUs the path "
                       "kernels leave" + (f" ({session.network_cus_used} CU-masked CUs)" if session.network_cus_used else
                                            " (no CU masks: the tails)"))}

    # ---- measured HBM ceilings on this device (STREAM-style, 8 GiB buffers) --------------
    stream_gbs = {}
    if rank == 0:
        n = (8 << 30) // 4
        buf = torch.empty(n, dtype=torch.float32, device=dev)
        src = torch.empty(n, dtype=torch.float32, device=dev)
        for name, fn, nbytes in (("write", lambda: buf.fill_(1.0), 4 * n),
                                 ("copy", lambda: buf.copy_(src), 8 * n)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            e1.synchronize()
            stream_gbs[name] = nbytes * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9
        del buf, src
        torch.cuda.empty_cache()

    # PMC traffic of THIS kernel at this config (profiles/pmc_traffic.json, tools/pmc_summary.py): an
    # entry counts only if it measured the same kernel (engine.kernel_name), config, store and math;
    # the latest round wins
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                tj = json.load(f)
            hits = sorted((v.get("round", ""), k) for k, v in tj.items()
                          if v.get("kernel_name") == eng.kernel_name and v.get("config") == args.config
                          and v.get("store") == args.store and v.get("math") == args.math)
            if hits:  # per-launch bytes of the profiled launch, scaled to this launch's contracts
                traffic_src = hits[-1][1]
                ent = tj[traffic_src]
                traffic = ent["hbm_bytes_per_launch"] / ent["contracts_per_launch"] * contracts_per_launch
        except (OSError, ValueError, KeyError):
            traffic, traffic_src = None, None

    total_units = world * B * P * args.steps
    value = total_units / elapsed
    line = {
        "metric": "training-steps/sec (contracts*paths/s) + HBM GB/s, GBM 4096x65536"
                  + (f" [{args.config}: basket of {n_assets} correlated assets]" if n_assets else ""),
        "value": value,
        "unit": "contracts*paths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
        "steps_per_sec": args.steps / elapsed,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if f64 else "f32",
        "network_dtype": ("f64" if f64 else
                          {"mfma_bf16": "bf16 operands, f32 accumulate / master weights"}.get(network["compute"], "f32")
                          if network else "f32 (torch-ROCm modules)"),
        "data": ("synthetic: Sobol basket contracts (seed 7, basket.default_basket_bounds), random-init CVNN (seed 123)"
                 if n_assets else
                 "synthetic: Sobol contracts (seed 7, make_domain_bounds defaults), random-init CVNN (seed 123)"),
        "config": {"workload": desc, "contracts_per_gpu": B, "global_contracts": world * B, "paths": P,
                   "timesteps": T, "network_size": N, "batches_per_mc_run": M, "assets": n_assets or 1,
                   "path_store": args.store, "math": args.math, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": eng.kernel_name, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     # bytes the kernel actually moved (PMC) over its live time, against the same peak
                     "frac_moved": (traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                     "kernel_ms": kernel_ms, "kernel_ms_isolated": kernel_ms, "kernel_timing": kernel_timing,
                     "kernel_ms_events": kernel_ms_events, "kernel_iters": args.kernel_iters,
                     "live_launches": len(live),
                     # one MC lane: the launch inside the timed region (HIP events on the MC stream), next to the
                     # network kernels of the previous step
                     "kernel_ms_live": live_ms,
                     "frac_live": (bytes_launch / (live_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if live_ms else None,
                     "mc_lanes": lanes,
                     # lanes > 1: consecutive launches overlap; the MC part's steady
                     # time per launch and the fraction of peak it corresponds to
                     "kernel_ms_steady": steady_ms,
                     "frac_steady": (bytes_launch / (steady_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if steady_ms else None,
                     "mc_note": (f"consecutive path launches overlap ({lanes} MC lanes on the CUs the network's "
                                 f"{session.network_cus_used} masked CUs leave); kernel_ms = the launch alone on the whole chip, "
                                 "kernel_ms_steady = launch spacing in the timed region; a rocprofv3 trace "
                                 "of this run records each overlapped launch from its dispatch to its end"
                                 if lanes > 1 else None),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "algorithmic_bytes_survey_per_launch": bytes_survey,
                     # the f64 rows kernel is bound by VALU issue at the clock the chip sustains under it, not
                     # by HBM (PMC): the HBM fraction above is not its ceiling
                     "bound_note": ("rows_kernel (f64) runs at the clock the power limiter allows (1.3-1.67 GHz): 38 VALU "
                                    "instructions per path-step (math v4) hold the SIMDs 80-83 % of the launch "
                                    "(profiles/r06/pmc_clock.txt)" if eng.kernel_name.startswith("rows_")
                                   and f64 else
                                    "rows_ref_kernel runs at the VALU issue ceiling (profiles/r06/pmc_c2ref.txt)"
                                    if eng.kernel_name.startswith("rows_ref") else None),
                     "bytes_note": ("the kernel keeps each contract's terminal row on chip: achieved counts the path "
                                    "store, targets and contract rows, not the terminal re-read of SURVEY 8(d)'s "
                                    "per-contract figure (algorithmic_bytes_survey_per_launch)" if on_chip else None),
                     "contracts_per_launch": contracts_per_launch,
                     # SURVEY 8(d)'s step level (its headline definition): the step's algorithmic bytes (8(d)'s
                     # per-contract figure x B per GPU) over the measured step time (Sobol, paths, CF, CVNN, Adam)
                     "step_level": {"bytes_per_step": bytes_survey / contracts_per_launch * B,
                                    "achieved": bytes_survey / contracts_per_launch * B / (elapsed / args.steps) / 1e9,
                                    "frac": bytes_survey / contracts_per_launch * B / (elapsed / args.steps) / 1e9
                                    / HBM_PEAK_GBS},
                     "measured_stream_gbs": stream_gbs,
                     "frac_of_measured_write": (achieved / stream_gbs["write"]) if "write" in stream_gbs else None},
        "network": network,
        "data_parallel": data_parallel,
        "final_loss": final.loss,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(B, T, N, M, widths, args.cpu_seconds, n_assets, "float64" if f64 else "float32",
                          normalize=args.config not in RAW_NORMALIZATION)
        line["cpu_baseline"] = cb
        line["speedup_vs_cpu"] = value / cb["value"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if ctx:
        dist.barrier()
        dp.shutdown()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
