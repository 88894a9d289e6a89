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


def test_summary_is_the_last_key_and_survives_a_truncated_tail():
    """the JSON line ends with a compact `summary` of every sub-leg (grid, cold,
    strong, RANSAC, cfg3, ranks), so a driver that keeps only the last ~1,000 characters of stdout
    still records them.  The dry line of --launch-check carries it; a full-size line (round 5's
    recorded bench line, 11 kB) keeps every field and value in its last 1,000 characters."""
    sys.path.insert(0, str(ROOT))
    import bench

    p = run_bench(["--gpus", "2", "--launch-check"], M3D_BENCH_SAME_DEVICE="1", M3D_BENCH_BACKEND="gloo")
    assert p.returncode == 0, p.stderr[-2000:]
    raw = [x for x in p.stdout.splitlines() if x.startswith("{")][0]
    line = json.loads(raw)
    assert list(line)[-1] == "summary"
    assert tuple(line["summary"]) == bench.SUMMARY_FIELDS
    assert line["summary"]["n_gpus"] == 2 and line["summary"]["comm_ranks"] == 2
    full = json.loads((ROOT / "profiles" / "r05_recheck_bench.json").read_text())
    full.pop("summary", None)
    full["summary"] = bench.build_summary(full)
    s = full["summary"]
    assert len(json.dumps({"summary": s})) < 600
    assert s["icp_grid"] is not None and s["cfg1_cold_grid_ms"] is not None and s["ransac_strong"] is not None
    assert s["cfg3_grid"] is not None and s["cfg1_strong"] is not None
    tail = json.dumps(full)[-1000:]
    for k, v in s.items():
        assert f'"{k}": {json.dumps(v)}' in tail, k
