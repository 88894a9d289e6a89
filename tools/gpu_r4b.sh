#!/bin/bash
# Round 4: world-1 rehearsal of the N > 1 bench path (exchange fields), then the drop-in
# refine_registration stage split and the loop-create stage timings.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_dist1_rehearsal.sh > gpurun_out/dist1_summary.log 2>&1
rc=$?; cat gpurun_out/dist1_summary.log; [ $rc -eq 0 ] || exit $rc
M3D_CREATE_PROF=1 timeout -k 10 180 python3 -u tools/refine_timing.py > gpurun_out/refine_timing.log 2>&1
rc=$?; grep -v "m3d create" gpurun_out/refine_timing.log | tail -5; grep "m3d create" gpurun_out/refine_timing.log | tail -3; exit $rc
