#!/usr/bin/env python3
"""Summarise rocprofv3 CSVs (kernel stats + PMC passes) per kernel.

Usage: python tools/prof_summary.py gpurun_out/prof [--json profiles/pmc_rXX.json]
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads ½ of a wide coalesced stream on
gfx950 → reported raw and ×2-corrected; WRITE_SIZE exact for 16-B stores.  Effective clock =
GRBM_GUI_ACTIVE / 8 / kernel duration (reads high for dispatches < 0.3 ms).
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    name = re.sub(r"^void ", "", name.replace("_ZN3m3d", ""))
    m = re.match(r"(?:m3d::)?([A-Za-z0-9_]+(?:<[0-9]+>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    d = Path(sys.argv[1])
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    stats = {}
    for f in d.glob("**/*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                           total_ns=float(r["TotalDurationNs"]), pct=float(r["Percentage"]))
    ctr = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in d.glob("**/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                dur[k].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    res = {}
    for k in sorted(set(stats) | set(ctr), key=lambda x: -stats.get(x, {}).get("total_ns", 0)):
        e = dict(stats.get(k, {}))
        c = {n: sum(v) / len(v) for n, v in ctr.get(k, {}).items()}
        e["counters_per_launch"] = c
        if "FETCH_SIZE" in c:
            e["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
            e["fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "fetch_bytes_corrected" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        if "GRBM_GUI_ACTIVE" in c and dur.get(k):
            e["eff_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / (sum(dur[k]) / len(dur[k]))
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
            e["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        res[k] = e
    for k, e in res.items():
        c = e["counters_per_launch"]
        print(f"{k:28s} calls={e.get('calls', '-'):>5} avg={e.get('avg_ns', 0)/1e3:9.2f}us "
              f"pct={e.get('pct', 0):5.1f} clk={e.get('eff_clock_ghz', 0):4.2f}GHz "
              + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
    if out_json:
        Path(out_json).write_text(json.dumps({"source": str(d), "kernels": res}, indent=1))


if __name__ == "__main__":
    main()
