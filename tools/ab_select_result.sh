#!/bin/bash
# RANSAC run tail: the last batch's select writes the result (ab/libm3d_new.so) against a separate
# copy_result launch (ab/libm3d_old.so): RANSAC + multi-GPU GPU tests with the new library, then
# alternating bench cfg2 runs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d-matching_amd/m3d
cp $L/libm3d.so $L/ab/libm3d_cur.so
cp $L/ab/libm3d_new.so $L/libm3d.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_ransac.py tests/test_gpu_multi.py tests/test_gpu_prep.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in old new; do
    cp $L/ab/libm3d_$v.so $L/libm3d.so
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cfg3 --no-grid --no-ransac-api --no-cfg4 --no-cpu-baseline --ransac-steps 40 > gpurun_out/bs_$v.log 2>&1 || exit 1
    python - $v <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/bs_{sys.argv[1]}.log") if x.startswith("{")][-1])
r = d["ransac"]
print(sys.argv[1], "ransac %.4g hyp/s, ms/run %.4f, score %.4f ms, best_fitness %s" % (r["value"], r["ms_per_run"], r["roofline"]["avg_launch_ms"], r["best_fitness"]))
PY
  done
done
cp $L/ab/libm3d_cur.so $L/libm3d.so
