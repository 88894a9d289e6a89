#!/usr/bin/env python3
"""Wall-time breakdown of Ply()'s full-cloud normals stage (ply.py:66 EstimateNormals on the
full-resolution cloud, radius 2v, max_nn 30) on a generated 180k-vertex scan: upload, cloud
pack, grid, neighbourhoods + normals, download."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import prep, synth
from m3d.core import Cloud


def lap(t0, name, out):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out[name] = round((t - t0) * 1e3, 3)
    return t


def main():
    v, _ = synth.surface_mesh(300, 600, seed=1)
    pts = v.astype(np.float32).astype(np.float64)
    for rep in range(3):
        out = {}
        torch.cuda.synchronize()
        t = time.perf_counter()
        c = Cloud(pts)
        t = lap(t, "cloud_create", out)
        nrm = prep.estimate_normals(c, 0.6, 30)
        t = lap(t, "estimate_normals(total)", out)
        idx, d2, cnt = prep.hybrid_search(c, 0.6, 30)
        t = lap(t, "hybrid_search+download", out)
        print(rep, len(pts), out, "mean neighbours", float(cnt.mean()))


if __name__ == "__main__":
    main()
