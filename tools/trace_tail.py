#!/usr/bin/env python3
"""Per-launch durations from a rocprofv3 --kernel-trace CSV: the durations of every launch whose
name contains PATTERN, and the last N launches of the trace with their start offsets (µs)."""
import csv
import sys


def main():
    path, pattern = sys.argv[1], sys.argv[2]
    n_tail = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
           if pattern in r["Kernel_Name"]]
    print(f"{pattern}: {len(dur)} launches, µs:", [round(d, 1) for d in dur])
    tail = rows[-n_tail:]
    t0 = int(tail[0]["Start_Timestamp"])
    for r in tail:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{r['Kernel_Name'][:40]:40s} start {s:9.1f}  dur {d:8.1f}")


if __name__ == "__main__":
    main()
