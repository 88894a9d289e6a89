#!/bin/bash
# PMC counters of the ICP NN kernels (brute force), separate passes; then the summary
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/nnpmc
A="python3 tools/prof_kernels.py --skip-ransac --nn brute --icp-iters ${ICP_ITERS:-10}"
run() { local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d gpurun_out/nnpmc/$name -o $name --output-format csv -- $A > gpurun_out/nnpmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run trace --kernel-trace --stats
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run p2 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY
run p3 --pmc SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
python3 tools/prof_summary.py gpurun_out/nnpmc | cut -c1-400
