#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg4prof
for m in pageable register stage; do
  M3D_UPLOAD=$m timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 3 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/$m: /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg4prof/t -o c4 --output-format csv -- python3 tools/cfg4_refine_timing.py --reps 2 > gpurun_out/cfg4prof/run.log 2>&1
rc=$?; echo "prof rc=$rc"
python3 tools/split_kernel_trace.py $(find gpurun_out/cfg4prof/t -name "*kernel_trace.csv" | head -1) | grep -E "grid_nn|terms|solve|reduce|keyinit" | head -20
