#!/bin/bash
# Round 4: direct Morton source — full GPU suite, then cold timings (direct vs round-3 derivation).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r4g_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for m in 1 0 1 0; do
  M3D_MORTON_DIRECT=$m timeout -k 10 120 python -u tools/cold_timing.py --reps 9 --tag direct$m 2>&1 | grep -v amdgpu.ids
done
M3D_CREATE_PROF=1 timeout -k 10 120 python -u tools/cold_timing.py --reps 3 2>&1 | grep "m3d create" | tail -2
timeout -k 10 180 python3 -u tools/refine_timing.py 2>&1 | grep -v amdgpu.ids | tail -2
