#!/bin/bash
# rocprofv3 passes on the GPU box: kernel trace + stats, then separate PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:-}
run() { # name, extra rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d gpurun_out/prof/$name -o $name --output-format csv -- \
    python3 tools/prof_kernels.py $ARGS > gpurun_out/prof/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run trace --kernel-trace --stats
run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run pmc2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA
run pmc3 --pmc FETCH_SIZE
run pmc4 --pmc WRITE_SIZE
find gpurun_out/prof -name "*.csv" | head -50
