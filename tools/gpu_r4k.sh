#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
M3D_RUN_PROF=1 M3D_CREATE_PROF=1 timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 3 > gpurun_out/cfg4_refine_prof.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/cfg4_refine_prof.log | grep -v "m3d run\|m3d create" | tail -4; grep "m3d run\|m3d create" gpurun_out/cfg4_refine_prof.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 5 2>&1 | grep -v amdgpu | tail -2
