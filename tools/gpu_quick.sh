#!/bin/bash
# quick loop: GPU tests (selected by PYTEST_K), then ICP/RANSAC bench; stops on a fault.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -rf ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
python - <<'PY'
import json
l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')]
if l:
    d=json.loads(l[-1]); r=d.get('ransac') or {}
    print('icp it/s %.1f nn ms %.3f frac %.3f | ransac %.4g hyp/s score ms %.4f frac %.3f | err %.2e' % (
      d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], r.get('value', 0),
      (r.get('roofline') or {}).get('avg_launch_ms', 0), (r.get('roofline') or {}).get('frac', 0),
      d['check']['max_abs_err_vs_T_true']))
    g=d.get('icp_grid')
    if g: print('grid icp it/s %.1f same %s nn ms %.4f terms ms %.4f' % (g['value'], g['same_result_as_brute'], g['roofline']['avg_launch_ms'], g['roofline']['terms_avg_launch_ms']))
PY
exit $rc
