"""Cold cfg1 (--n 1000000: cfg3) setup timing (bench.py bench_cold's stages, more repetitions): fresh device clouds,
then the ICP loop object (grids, Morton source copy, fp16 tiles, target records), per NN method.
Prints one line per method: median ms of clouds / loop_create over --reps runs after one warm run.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-matching_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--tag", default="")
    ap.add_argument("--n", type=int, default=100000, help="points per cloud (cfg3: 1000000)")
    ap.add_argument("--nns", default="grid,brute")
    a = ap.parse_args()
    import numpy as np
    import torch
    from pathlib import Path

    from m3d import _lib, synth

    if os.environ.get("AB_LIB"):  # time another build of the library (tools/ab_build.sh)
        _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
    from m3d.core import Cloud, IcpLoop

    src, tgt, nrm, _ = synth.icp_pair(a.n, a.n, seed=0)
    r = 0.4 * 0.3

    def once(nn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc, tc = Cloud(src), Cloud(tgt, nrm)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        lp = IcpLoop(sc, tc, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=50, nn=nn)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        lp.reset(np.eye(4))
        lp.steps(51)
        res = lp.result()
        t3 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, res.transformation

    for nn in a.nns.split(","):
        once(nn)
        runs = [once(nn) for _ in range(a.reps)]
        T = runs[0][3]
        same = all(np.array_equal(x[3], T) for x in runs)
        med = [float(np.median([x[k] for x in runs])) for k in range(3)]
        print(f"{a.tag} {nn}: clouds {med[0]:.3f} ms, loop_create {med[1]:.3f} ms, "
              f"iterations {med[2]:.3f} ms, T identical across runs {same}, T[0,3] {T[0, 3]!r}", flush=True)


if __name__ == "__main__":
    main()
