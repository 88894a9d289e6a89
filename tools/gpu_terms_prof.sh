#!/bin/bash
# rocprofv3 kernel stats of the grid ICP loop, fused tail vs the separate terms/reduce/solve launches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/termsprof
for f in 1 0; do
  timeout -k 10 300 env M3D_ICP_FUSED=$f rocprofv3 --kernel-trace --stats -d gpurun_out/termsprof/f$f -o f$f --output-format csv -- \
    python3 tools/prof_kernels.py --icp-iters 30 --skip-ransac --nn ${NN:-grid} > gpurun_out/termsprof/f$f.log 2>&1
  rc=$?; echo "fused=$f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$f" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/termsprof/f{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.2f} us")
PY
done
