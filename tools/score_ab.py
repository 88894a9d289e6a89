#!/usr/bin/env python3
"""Scoring A/B on one device: counts + time of m3d_ransac_score at cfg2 geometry, and the number
of pairs re-evaluated in fp64.  Run twice (M3D_SCORE_MFMA=1 / 0) and compare the printed lines."""
import os
import sys
import time
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-matching_amd"))


def main():
    import numpy as np
    import torch

    from m3d import _lib, synth
    from m3d.core import CorrSet, context

    torch.cuda.set_device(0)
    nc = int(os.environ.get("NC", "100000"))
    H = int(os.environ.get("H", "10000"))
    src, tgt, corr, _ = synth.ransac_pair(nc, seed=42)
    cs = CorrSet(src, tgt, corr)
    T, _ = cs.kabsch3(H, seed=42)
    ctx = context()
    for rep in range(3):
        s0 = ctx.stats()[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        counts = cs.score(T, 0.45, _lib.SCORE_NORM)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s1 = ctx.stats()[0]
    c = counts.cpu().numpy()
    print(f"{os.environ.get('AB_TAG', '')} mfma={os.environ.get('M3D_SCORE_MFMA', '1')} mg={os.environ.get('M3D_SCORE_MG', '2')} nc={nc} H={H} ms={dt * 1e3:.3f} "
          f"sum={int(c.sum())} mean_fit={c.mean() / nc:.4f} rechecked={int(s1 - s0)} "
          f"crc={zlib.crc32(c.tobytes()):08x}")
    np.save(f"gpurun_out/counts_{os.environ.get('M3D_SCORE_MFMA', '1')}{os.environ.get('AB_TAG', '')}.npy", c)


if __name__ == "__main__":
    main()
