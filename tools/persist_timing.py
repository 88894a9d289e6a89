#!/usr/bin/env python3
"""cfg1 grid ICP loop: the persistent one-launch loop against the two-launch loop (graph replay).
Events around whole runs of `it + 1` evaluations, best of `reps`; µs per evaluation.
Usage: python tools/persist_timing.py [iters] [reps]   (M3D_PERSIST_LANES = 1 | 2 in the env)"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import synth
from m3d.core import Cloud, IcpLoop

it = int(sys.argv[1]) if len(sys.argv) > 1 else 50
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.cuda.set_device(0)
for ns in (100_000, 20_000):
    src, tgt, nrm, _ = synth.icp_pair(ns, 100_000, seed=0)
    s, t = Cloud(src), Cloud(tgt, nrm)
    out = {}
    for persist in (True, False):
        lp = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=it, nn="grid",
                     persist=persist)
        for _ in range(3):
            lp.reset(np.eye(4))
            lp.steps(it + 1)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            lp.reset(np.eye(4))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lp.steps(it + 1)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / (it + 1))
        r = lp.result()
        out[persist] = (best, r.transformation.copy(), r.fitness)
        del lp
    same = np.array_equal(out[True][1], out[False][1]) and out[True][2] == out[False][2]
    print(f"ns={ns} lanes={os.environ.get('M3D_PERSIST_LANES', '2')}: persistent {out[True][0]:.2f} us/eval, "
          f"two-launch (graph) {out[False][0]:.2f} us/eval, same bits: {same}", flush=True)
