#!/usr/bin/env python3
"""cfg2 scoring-kernel timing (AB_LIB=path: another build of libm3d.so, e.g. the pricing builds of
tools/ab_build.sh -DM3D_SCORE_PRICE=1|2): the a4 run at Nc = 1e5, H = 1e5 (bench cfg2), library
HIP events around every score_mfma_kernel launch; prints ms per launch and a crc of the counts.
Usage: python tools/score_timing.py [runs]"""
import os
import sys
import zlib
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib, synth

if os.environ.get("AB_LIB"):
    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d.core import RESULT_WORDS, CorrSet, RansacParams, context, ptr, stream_handle
import ctypes

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
ctx = context()
src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
cs = CorrSet(src, tgt, corr)
H = 100_000
counts = torch.zeros(H, dtype=torch.int32, device="cuda")
buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
p = RansacParams(max_iter=H, seed=42, thr=0.45, mode=_lib.SCORE_NORM, early_stop=False).to_c()


def run():
    ctx.check(ctx.lib.m3d_ransac_run_async(ctx.h, cs.h, ctypes.byref(p), None, ptr(counts), ptr(buf),
                                           stream_handle()), "run")


for _ in range(5):
    run()
torch.cuda.synchronize()
ctx.profile(True)
ctx.profile_read(_lib.KERNEL_SCORE)
for _ in range(runs):
    run()
ms, n = ctx.profile_read(_lib.KERNEL_SCORE)
ctx.profile(False)
c = counts.cpu().numpy()
print(f"{os.environ.get('AB_LIB', 'libm3d.so')}: score_mfma_kernel {ms / n:.4f} ms per launch ({n} launches), "
      f"counts crc {zlib.crc32(c.tobytes()):08x}", flush=True)
