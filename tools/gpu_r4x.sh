#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4x_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4x_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/cloud_upload_timing.py --ns 100000 --nt 100000 --reps 15 2>&1 | grep -v amdgpu | head -5
timeout -k 10 300 python3 -u bench.py --no-ransac --no-ransac-api --no-cpu-baseline --no-cfg4 --steps 3 > gpurun_out/r4x_bench.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r4x_bench.json') if l.startswith('{')][-1]); print('cold', d['cfg1_cold']['grid'], d['cfg1_cold']['refine_registration_ms'])"
