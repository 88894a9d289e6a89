#!/bin/bash
# scoring A/B (tools/score_ab.py) over environment settings: AB="K=V K=V ..." (default below)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for kv in ${AB:-M3D_SCORE_MFMA=0 M3D_SCORE_MFMA=1 M3D_SCORE_EXP=1}; do
  env $kv timeout -k 10 120 python3 tools/score_ab.py || exit $?
done
