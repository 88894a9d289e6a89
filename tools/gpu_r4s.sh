#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp tools/ab/libm3d_dbg.so 3d-matching_amd/m3d/libm3d.so
M3D_GRID_HEAVY=8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_icp.py -x -q --timeout 200 --timeout-method thread -k "graph_replay" > gpurun_out/r4s_dbg.log 2>&1
rc=$?; grep -c "\[guard\]" gpurun_out/r4s_dbg.log; grep "\[guard\]" gpurun_out/r4s_dbg.log | sort | uniq -c | sort -rn | head -20; tail -3 gpurun_out/r4s_dbg.log; exit $rc
