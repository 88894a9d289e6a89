#!/bin/bash
# grid scan block -> XCD mapping sweep (M3D_SCAN_XCHUNK): cfg1, 1M x 125k index shard, 1M x 1M, and
# the 8 spatial / index shards of cfg3 (grid only).  Run on the GPU box: bash tools/xchunk_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${XCHUNKS:-0 2 8 32}; do
  echo "== M3D_SCAN_XCHUNK=$c"
  M3D_SCAN_XCHUNK=$c timeout -k 10 300 python3 tools/grid_timing.py 20 || exit $?
  M3D_SCAN_XCHUNK=$c timeout -k 10 300 python3 tools/spatial_shard_timing.py 1000000 grid || exit $?
done
