#!/bin/bash
# GPU-box tuning sweep for the ICP tail and grid path: grid lanes per query × terms sources per
# thread (M3D_GRID_LANES, M3D_TERMS_PTS).  Each bench run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LANES:-16 8 4}; do for P in ${PTS:-4 2 8}; do
  M3D_GRID_LANES=$L M3D_TERMS_PTS=$P timeout -k 10 200 python bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-ransac > gpurun_out/tune_${L}_${P}.log 2>&1 || exit $?
  python - "$L" "$P" <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/tune_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1])
g = d["icp_grid"]
print(f"lanes {sys.argv[1]:>2} pts {sys.argv[2]}: brute {d['value']:.0f} it/s terms {d['roofline']['terms_avg_launch_ms']*1e3:.1f} us | "
      f"grid {g['value']:.0f} it/s nn {g['roofline']['avg_launch_ms']*1e3:.1f} us terms {g['roofline']['terms_avg_launch_ms']*1e3:.1f} us same {g['same_result_as_brute']}")
PY
done; done
