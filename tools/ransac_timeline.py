#!/usr/bin/env python3
"""cfg2 RANSAC runs back to back (bench.py's ransac leg: Nc = 1e5, 1e5 hypotheses, no early
stop, run_async), for a rocprofv3 --kernel-trace timeline; `--parse CSV` prints, per run, every
kernel's duration and the gap before it (µs), and the run's span."""
import csv
import sys
import time
from pathlib import Path


def parse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "ransac_init_kernel" in name:
            cur = []
            runs.append(cur)
        if cur is not None:
            cur.append((name.split("(")[0].replace("m3d::", "")[:34], int(r["Start_Timestamp"]),
                        int(r["End_Timestamp"])))
        if "copy_result_kernel" in name:
            cur = None
    for run in runs[-3:]:
        t0, prev = run[0][1], run[0][1]
        for n, s, e in run:
            print(f"  {n:34s} gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}")
            prev = e
        print(f"  span {(run[-1][2] - t0) / 1e3:.1f} us")
    if len(runs) > 1:
        starts = [r[0][1] for r in runs]
        print("run-to-run period (us):", [round((b - a) / 1e3, 1) for a, b in zip(starts, starts[1:])][-6:])


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
        return
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
    import torch

    from m3d import _lib, synth
    from m3d.core import RESULT_WORDS, CorrSet, RansacParams

    src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
    cs = CorrSet(src, tgt, corr)
    res = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
    p = RansacParams(max_iter=100_000, seed=42, thr=0.45, mode=_lib.SCORE_NORM, early_stop=False)
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        cs.run_async(p, res)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        cs.run_async(p, res)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / 8 * 1e3:.3f} ms per run")


if __name__ == "__main__":
    main()
