#!/usr/bin/env python3
"""cfg2 RANSAC run time (Nc = 1e5, 1e5 hypotheses, no early stop) under the variants the bench
and tools/ransac_batch.py differ in: synchronous run vs run_async, the threshold literal."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import torch

from m3d import _lib, synth
from m3d.core import RESULT_WORDS, CorrSet, RansacParams

src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
cs = CorrSet(src, tgt, corr)
res = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
for rep in range(2):
    for thr in (0.45, 0.3 * 1.5):
        p = RansacParams(max_iter=100_000, seed=42, thr=thr, mode=_lib.SCORE_NORM, early_stop=False)
        for mode in ("run", "async"):
            f = (lambda: cs.run(p)) if mode == "run" else (lambda: cs.run_async(p, res))
            f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / 5
            print(f"rep {rep} thr {thr!r:>20} {mode:5s}: {el * 1e3:.3f} ms per run = {1e5 / el:.4g} hyp/s")
