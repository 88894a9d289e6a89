#!/bin/bash
# The driver's N > 1 bench path at world 1 on a one-GPU box: torch.distributed.run with one rank,
# the nccl (RCCL) process group AND libm3d's own RCCL communicator in the same process, the
# source-sharded (default) and target-sharded native loops, cfg1_strong, the sharded RANSAC and
# cfg3's target-shard loop.  Checks that the two RCCL users coexist and that rank 0 prints the line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sh in source target; do
  M3D_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 \
    bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --shard $sh --cfg3-n 200000 --cfg3-iters 5 \
    --no-ransac-api --no-cfg4 > gpurun_out/dist1_$sh.log 2>&1
  rc=$?; echo "dist1 $sh rc=$rc"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/dist1_$sh.log; exit $rc; }
  python - "$sh" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/dist1_{sys.argv[1]}.log") if x.startswith("{")]
d = json.loads(l[-1])
s = d["cfg1_strong"]; r = d["ransac"]; c3 = d["cfg3"]
print(sys.argv[1], "comm", d["config"]["comm"], "| cfg1 %.1f it/s err %.2e" % (d["value"], d["check"]["max_abs_err_vs_T_true"]),
      "| strong %.1f grid %s" % (s["value"], s.get("grid_value")),
      "| ransac %.3g strong %.3g best %s" % (r["value"], r["strong"]["value"], r["strong"].get("best_count")),
      "| cfg3 %.1f grid %.1f" % (c3["value"], c3["grid"]["value"]))
keys = ("per_evaluation_ms_with_events", "nn_ms_per_evaluation", "terms_ms_per_evaluation",
        "exchange_ms_per_evaluation", "allreduces_per_evaluation")
for name, sec in (("cfg1_strong", s), ("cfg3", c3), ("cfg3.grid", c3["grid"]),
                  ("cfg3.split_off", c3.get("split_off") or {}), ("cfg3.grid.split_off", c3["grid"].get("split_off") or {})):
    print("  %-20s" % name, " ".join("%s=%s" % (k.replace("_per_evaluation", ""), None if sec.get(k) is None else round(sec[k], 4)) for k in keys))
print("  ransac.strong score_ms %s exchange_ms %s" % (r["strong"].get("score_ms_per_run"), r["strong"].get("exchange_ms_per_run")))
PY
done
