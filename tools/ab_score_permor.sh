#!/bin/bash
# Scoring sign count: two v_perm joined by one OR per v_bcnt (M3D_SCORE_PERM_OR=1, _p1) against
# one v_bcnt per v_perm (_p0): RANSAC GPU tests with _p1, then alternating score_ab + bench cfg2.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d-matching_amd/m3d
cp $L/libm3d.so $L/ab/libm3d_cur.so
cp $L/ab/libm3d_p1.so $L/libm3d.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ransac.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_p1.log 2>&1
rc=$?; echo "pytest p1 rc=$rc"; tail -2 gpurun_out/pytest_p1.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in p0 p1; do
    cp $L/ab/libm3d_$v.so $L/libm3d.so
    AB_TAG=$v NC=100000 H=100000 timeout -k 10 120 python tools/score_ab.py || exit 1
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cfg3 --no-grid --no-ransac-api --no-cfg4 --no-cpu-baseline > gpurun_out/bp_$v.log 2>&1 || exit 1
    python - $v <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/bp_{sys.argv[1]}.log") if x.startswith("{")][-1])
r = d["ransac"]
print(sys.argv[1], "ransac %.4g hyp/s, ms/run %.4f, score %.4f ms" % (r["value"], r["ms_per_run"], r["roofline"]["avg_launch_ms"]))
PY
  done
done
cp $L/ab/libm3d_cur.so $L/libm3d.so
