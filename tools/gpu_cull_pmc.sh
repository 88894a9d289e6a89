#!/bin/bash
# PMC passes over the culled RANSAC run (one counter group per run): where cull_classify_kernel's
# time goes.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cullpmc
run() { local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -d gpurun_out/cullpmc/$name -o $name --output-format csv -- python3 tools/cull_timing.py 2 > gpurun_out/cullpmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM
run p2 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA
python3 tools/prof_summary.py gpurun_out/cullpmc 2>&1 | grep -E "cull_classify|score_mfma" | cut -c1-900
