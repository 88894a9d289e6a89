#!/usr/bin/env python3
"""Short, fixed workload for rocprofv3 runs (kernel trace / PMC counters).

ICP: cfg1 geometry (100k↔100k), `--icp-iters` iterations from identity, brute-force NN and
then the uniform-grid NN (`--nn brute|grid|both`).
RANSAC: cfg2 geometry (Nc = 1e5), `--hyps` native hypotheses, no early stop.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-matching_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--icp-iters", type=int, default=5)
    ap.add_argument("--hyps", type=int, default=20_000)
    ap.add_argument("--skip-ransac", action="store_true")
    ap.add_argument("--skip-icp", action="store_true")
    ap.add_argument("--nn", default="both", choices=["brute", "grid", "both"])
    a = ap.parse_args()
    import numpy as np
    import torch

    from m3d import _lib, synth
    from m3d.core import Cloud, CorrSet, IcpLoop, RansacParams

    torch.cuda.set_device(0)
    if not a.skip_icp:
        src, tgt, nrm, _ = synth.icp_pair(a.n, seed=0)
        sc, tc = Cloud(src), Cloud(tgt, nrm)
        for nn in (["brute", "grid"] if a.nn == "both" else [a.nn]):
            loop = IcpLoop(sc, tc, 0.12, relative_fitness=-1, relative_rmse=-1,
                           max_iteration=a.icp_iters, nn=nn)
            loop.reset(np.eye(4))
            for _ in range(a.icp_iters + 1):
                loop.step()
            r = loop.result()
            print("icp", nn, r.fitness, r.iterations)
    if not a.skip_ransac:
        s, t, c, _ = synth.ransac_pair(a.n, seed=42)
        cs = CorrSet(s, t, c)
        out = cs.run(RansacParams(max_iter=a.hyps, seed=42, thr=0.45, mode=_lib.SCORE_NORM,
                                  early_stop=False))
        print("ransac", out.fitness, out.iterations)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
