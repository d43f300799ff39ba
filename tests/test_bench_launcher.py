"""bench.py's multi-rank launch, on the CPU: `bench.py --gpus N` started without a
launcher runs N ranks through torch.distributed.run as one child, a rank never re-launches, and a job
whose world size differs from --gpus exits non-zero instead of printing a mislabelled line."""

from __future__ import annotations

import json
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = """
import json, os, sys
out = sys.argv[sys.argv.index("--out") + 1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({"env": {k: os.environ.get(k) for k in keys}, "argv": sys.argv[1:]}, f)
"""


def test_launcher_command_is_the_drivers_form() -> None:
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")


def test_no_relaunch_for_one_gpu_or_inside_a_rank(monkeypatch) -> None:
    args = bench.parse(["--gpus", "1"])
    assert bench.maybe_launch_ranks(args, ["--gpus", "1"]) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    args = bench.parse(["--gpus", "2"])
    assert bench.maybe_launch_ranks(args, ["--gpus", "2"]) is None


def test_unlaunched_multi_gpu_run_starts_every_rank(tmp_path, monkeypatch) -> None:
    """--gpus 2 with no WORLD_SIZE: two ranks, ranks 0 and 1 of a world of 2, each with the original
    arguments and a 127.0.0.1 rendezvous."""
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    argv = ["--gpus", "2", "--steps", "3", "--out", str(tmp_path)]
    args = bench.parse(["--gpus", "2", "--steps", "3"])
    assert bench.maybe_launch_ranks(args, argv, script=str(script)) == 0
    seen = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(2)]
    for r, s in enumerate(seen):
        assert s["env"]["RANK"] == str(r) and s["env"]["LOCAL_RANK"] == str(r) and s["env"]["WORLD_SIZE"] == "2"
        assert s["env"]["MASTER_ADDR"] == "127.0.0.1"
        assert s["argv"] == argv


def test_world_size_mismatch_exits_nonzero() -> None:
    """A rank whose job has another world size than --gpus stops before any GPU work (exit 3)."""
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr
    assert "--gpus 2 but the job has 1 rank" in r.stderr
