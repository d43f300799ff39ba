"""`bench.py --gpus 2` run the way the driver runs `--gpus 1` (no launcher): it starts both ranks itself and
rank 0 prints one line for the whole job.  On a 1-GPU box the ranks rendezvous over
gloo and both run on cuda:0 (--backend gloo); on an 8-GPU node the default backend is nccl (RCCL)."""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_print_one_job_line() -> None:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--config", "e2e",
           "--steps", "4", "--warmup", "2", "--kernel-iters", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_contracts"] == 2 * line["config"]["contracts_per_gpu"] == 8192
    dpi = line["data_parallel"]
    assert dpi["world"] == 2 and dpi["backend"] == "gloo" and dpi["rccl_world"] is None
    assert dpi["allreduce_ms_in_step"] is not None and dpi["allreduce_ms_in_step"] > 0
    assert dpi["allreduce_ms_isolated"] > 0
    assert line["value"] > 0 and "cpu_baseline" not in line
