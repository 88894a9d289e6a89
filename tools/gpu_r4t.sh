#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp tools/ab/libm3d_dbg.so 3d-matching_amd/m3d/libm3d.so
M3D_GRID_HEAVY=8 timeout -k 10 120 python3 -u tools/heavy_probe.py > gpurun_out/r4t_probe.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r4t_probe.log | sed -E 's/slot [0-9]+/slot N/; s/\(t [0-9]+\)//; s/count [0-9]+/count N/' | uniq -c | head -60; grep -m3 "slot" gpurun_out/r4t_probe.log; exit $rc
