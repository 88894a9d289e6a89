#!/usr/bin/env python3
"""Per-iteration cost of the cfg1 ICP loop under different host drivers (experiment).

Python step() loop vs the native m3d_icp_steps loop, with and without the library's
per-kernel HIP event timers, for the brute-force and the grid NN."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-matching_amd"))

import numpy as np
import torch

from m3d import synth
from m3d.core import Cloud, IcpLoop


def main():
    torch.cuda.set_device(0)
    src, tgt, nrm, _ = synth.icp_pair(100_000, seed=0)
    sc, tc = Cloud(src), Cloud(tgt, nrm)
    iters = 50
    for nn in ("grid", "brute"):
        loop = IcpLoop(sc, tc, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=iters, nn=nn)
        for native in (False, True):
            for events in (False, True):
                ctx = sc.ctx
                ctx.profile(events)
                def run():
                    loop.reset(np.eye(4))
                    if native:
                        loop.steps(iters + 1)
                    else:
                        for _ in range(iters + 1):
                            loop.step()
                run()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                el = (time.perf_counter() - t0) / 5
                ctx.profile(False)
                print(f"{nn:5s} native={native!s:5s} events={events!s:5s} "
                      f"{el / (iters + 1) * 1e6:8.1f} us/iter  {5 * iters / (el * 5):9.1f} it/s", flush=True)


if __name__ == "__main__":
    main()
