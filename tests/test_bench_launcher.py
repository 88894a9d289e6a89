"""bench.py --gpus N brings up N ranks itself (VERDICT r4 "next" #1), on the CPU.

* ``--gpus 2 --launch-check`` with every rank on one device (M3D_BENCH_SAME_DEVICE=1, gloo): the
  launcher starts torch.distributed.run as a child, both ranks join, rank 0's line says
  ``n_gpus: 2``.
* ``--gpus 2`` with fewer than 2 visible GPUs (this container has none) exits non-zero and prints
  no line: an N = 1 line is never printed for ``--gpus N``.
* WORLD_SIZE that disagrees with ``--gpus`` is refused.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def run_bench(args, **env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=600, env=env, cwd=str(ROOT))


def json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_launcher_brings_up_two_ranks():
    p = run_bench(["--gpus", "2", "--launch-check"], M3D_BENCH_SAME_DEVICE="1", M3D_BENCH_BACKEND="gloo")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_joined"] == 2


def test_launcher_refuses_more_ranks_than_gpus():
    p = run_bench(["--gpus", "2", "--launch-check"])  # no GPU here: 0 < 2
    assert p.returncode != 0
    assert json_lines(p.stdout) == []
    assert "refusing" in p.stderr


def test_world_size_mismatch_is_refused():
    p = run_bench(["--gpus", "4", "--launch-check"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0
    assert json_lines(p.stdout) == []


def test_single_gpu_launch_check_unchanged():
    p = run_bench(["--gpus", "1", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json_lines(p.stdout)[0]["n_gpus"] == 1
