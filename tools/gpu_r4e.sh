#!/bin/bash
# Round 4: full GPU suite on the one-shot ICP changes, then cold / refine timings per upload mode.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r4e_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/cold_timing.py --reps 7 2>&1 | grep -v amdgpu.ids
M3D_CREATE_PROF=1 timeout -k 10 120 python -u tools/cold_timing.py --reps 3 2>&1 | grep "m3d create" | tail -2
for m in pageable register stage; do
  M3D_UPLOAD=$m timeout -k 10 180 python3 -u tools/refine_timing.py > gpurun_out/refine_$m.log 2>&1 || exit $?
  echo "upload=$m"; grep -v amdgpu.ids gpurun_out/refine_$m.log | tail -2
done
M3D_RUN_PROF=1 timeout -k 10 180 python3 -u tools/refine_timing.py --reps 3 2>&1 | grep "m3d run" | tail -2
