#!/bin/bash
# GPU tests, then cfg1 brute-force ICP: the one-launch iteration (default) against M3D_NN_FUSE=0
# (scan + fused tail as two launches), alternating, same library.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in 1 2 0; do
    M3D_NN_FUSE_ORDER=$([ $f = 2 ] && echo 0 || echo 1) M3D_NN_FUSE=$([ $f = 0 ] && echo 0 || echo 1) timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cfg3 --no-ransac --no-ransac-api --no-cfg4 --no-cpu-baseline > gpurun_out/fuse_$f.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc fuse=$f"; tail -5 gpurun_out/fuse_$f.log; exit $rc; }
    python - $f <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/fuse_{sys.argv[1]}.log") if x.startswith("{")][-1])
print("fuse", sys.argv[1], "cfg1 %.1f it/s, ms/step %.3f, nn(+tail) %.4f ms, terms %.4f ms, err %.2e, fit %.6f | grid %.0f | strong %s"
      % (d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["terms_avg_launch_ms"],
         d["check"]["max_abs_err_vs_T_true"], d["check"]["icp_fitness"], d["icp_grid"]["value"], d["cfg1_strong"]["value"]))
PY
  done
done
