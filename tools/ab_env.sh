#!/bin/bash
# A/B of tuning environment knobs on the cfg1 ICP bench: AB="M3D_NN_MG=1 M3D_NN_MG=2 ..."
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for kv in ${AB}; do
  env $kv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ransac --no-grid > gpurun_out/ab_$i.log 2>&1
  rc=$?; echo "$kv rc=$rc $(python3 -c "import json,sys; l=[x for x in open('gpurun_out/ab_$i.log') if x.startswith('{')]; d=json.loads(l[-1]); print(round(d['value'],1), round(d['roofline']['avg_launch_ms'],4))")"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
