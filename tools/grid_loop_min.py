"""Minimal cfg1 grid ICP loop for kernel A/B under rocprofv3: 100k ↔ 100k, 50 iterations × 6."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    import numpy as np
    import torch

    from m3d import synth
    from m3d.core import Cloud, IcpLoop

    src, tgt, nrm, _ = synth.icp_pair(100_000, 100_000, seed=0)
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=50, nn="grid", persist=False)
    import time
    ts = []
    for _ in range(6):
        lp.reset(np.eye(4))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lp.steps(50)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3 / 50)
    print(f"grid loop us per iteration: median {np.median(ts[1:]) * 1e3:.2f} (all {[round(t * 1e3, 1) for t in ts]})",
          flush=True)


if __name__ == "__main__":
    main()
