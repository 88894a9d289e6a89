#!/bin/bash
# Round-end check on the final tree: GPU tests + smoke + bench (tools/gpu_check.sh), then the
# round profile set (tools/gpu_prof_round.sh).  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_round.sh
