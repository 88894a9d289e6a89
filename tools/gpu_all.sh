#!/bin/bash
# tests + smoke + bench, then rocprof passes — stops at the first GPU fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "${SKIP_PROF:-0}" = "1" ] && exit 0
bash tools/gpu_prof.sh
