#!/usr/bin/env python3
"""RANSAC loop throughput (cfg2: Nc = 1e5, 1e5 hypotheses, no early stop) against the device
batch size (hypotheses per kabsch3 → score → select round)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import torch

from m3d import _lib, synth
from m3d.core import CorrSet, RansacParams

src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
cs = CorrSet(src, tgt, corr)
for B in (10_000, 20_000, 25_000, 50_000, 100_000):
    p = RansacParams(max_iter=100_000, seed=42, thr=0.45, mode=_lib.SCORE_NORM, early_stop=False, batch=B)
    cs.run(p)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        out = cs.run(p)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 5
    print(f"batch {B:>6}: {el * 1e3:.3f} ms per 1e5 hypotheses = {1e5 / el:.4g} hyp/s (best {out.best_count})")
