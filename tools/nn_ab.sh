#!/bin/bash
# Alternating A/B of library builds (tools/ab_build.sh → tools/ab/<variant>.so): ROUNDS × each
# variant of a timing script that honours AB_LIB (SCRIPT, default tools/nn_timing.py; ARGS, default
# 20), every run under its own time limit; the first failure ends the script.
# Usage (GPU box): [SCRIPT=tools/grid_timing.py] bash tools/nn_ab.sh VARIANT [VARIANT ...]
#   -> gpurun_out/nn_ab.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=${SCRIPT:-tools/nn_timing.py}
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in "$@"; do
    echo "round $r $v:" >> gpurun_out/nn_ab.log
    AB_LIB=tools/ab/$v.so timeout -k 10 300 python3 "$S" ${ARGS:-20} 2>&1 | grep -v amdgpu.ids >> gpurun_out/nn_ab.log
    rc=$?; [ $rc -eq 0 ] || { echo "stopping after $v rc=$rc"; tail -20 gpurun_out/nn_ab.log; exit $rc; }
  done
done
cat gpurun_out/nn_ab.log
