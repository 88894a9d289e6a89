#!/usr/bin/env python3
"""Per-workload kernel averages from a rocprofv3 --kernel-trace CSV of bench.py.

bench.py runs several legs (cfg1 brute/grid, cfg3 brute/grid, cfg2 RANSAC, the per-call drop-in
leg, cfg4), so one kernel's --stats average mixes launch sizes.  This groups every launch of the
hot kernels by its grid dimensions (one grid shape per leg) and prints calls / average / min / max
per (kernel, grid) — the figures to set beside the bench line's per-leg HIP-event averages.
Usage: python tools/split_kernel_trace.py TRACE.csv [> profiles/rXX_bench_kernel_split.txt]"""
import csv
import sys
from collections import defaultdict

HOT = ("nn_mfma_kernel", "score_mfma_kernel", "grid_nn_batched_kernel", "terms_solve_kernel", "reduce_groups_kernel",
       "terms_kernel", "kabsch3_kernel", "kabsch3_one_kernel", "reduce_kernel", "solve_kernel",
       "validate_kernel")


def main():
    groups = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("m3d::", "")
        if not any(h in short for h in HOT):
            continue
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        wg = int(r["Workgroup_Size_X"])
        groups[(short, grid, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':36s} {'grid (threads x,y,z)':>26s} {'wg':>5s} {'calls':>7s} {'avg us':>10s} {'min us':>10s} {'max us':>10s}")
    for (k, g, wg), v in sorted(groups.items(), key=lambda kv: (kv[0][0], -sum(kv[1]))):
        print(f"{k[:36]:36s} {str(g):>26s} {wg:5d} {len(v):7d} {sum(v) / len(v):10.2f} {min(v):10.2f} {max(v):10.2f}")


if __name__ == "__main__":
    main()
