#!/bin/bash
# Scoring tile size A/B (3d-matching_amd/m3d/ab/libm3d_t256.so vs _t512.so): RANSAC GPU tests with
# the 512 build, then alternating score_ab (H = Nc = 1e5, counts crc) and the bench's cfg2 line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d-matching_amd/m3d
cp $L/libm3d.so $L/ab/libm3d_cur.so
cp $L/ab/libm3d_t512.so $L/libm3d.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ransac.py tests/test_gpu_prep.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_t512.log 2>&1
rc=$?; echo "pytest t512 rc=$rc"; tail -3 gpurun_out/pytest_t512.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in t256 t512; do
    cp $L/ab/libm3d_$v.so $L/libm3d.so
    AB_TAG=$v NC=100000 H=100000 timeout -k 10 120 python tools/score_ab.py || exit 1
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cfg3 --no-grid --no-ransac-api --no-cfg4 --no-cpu-baseline > gpurun_out/bt_$v.log 2>&1 || exit 1
    python - $v <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/bt_{sys.argv[1]}.log") if x.startswith("{")][-1])
r = d["ransac"]
print(sys.argv[1], "ransac %.4g hyp/s, ms/run %.4f, score %.4f ms, best %s" % (r["value"], r["ms_per_run"], r["roofline"]["avg_launch_ms"], r.get("best_count", r.get("check"))))
PY
  done
done
cp $L/ab/libm3d_cur.so $L/libm3d.so
