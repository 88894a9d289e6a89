#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg4prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg4prof2/t -o c4 --output-format csv -- python3 tools/cfg4_refine_timing.py --reps 2 > gpurun_out/cfg4prof2/run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - $(find gpurun_out/cfg4prof2/t -name "*kernel_trace.csv" | head -1) <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted(((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"]) for r in rows))
# last icp run: from the last icp_init_kernel
last = max(k for k, x in enumerate(seq) if "icp_init_kernel" in x[2])
t0 = seq[last][0]
tot = {}
for s, d, n in seq[last:]:
    key = n.split("(")[0][:48]
    tot.setdefault(key, [0, 0.0, 0.0])
    tot[key][0] += 1; tot[key][1] += d; tot[key][2] = max(tot[key][2], d)
end = seq[-1][0] + seq[-1][1] * 1e3
print(f"last icp run span {(end - t0) / 1e3:.1f} us")
for k, (c, d, m) in sorted(tot.items(), key=lambda x: -x[1][1])[:12]:
    print(f"{k:50s} n={c:3d} sum={d:8.1f} us max={m:7.1f}")
P
