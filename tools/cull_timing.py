"""RANSAC tile culling A/B (ransac.hip cull_classify_kernel): bench.py's cfg2 batches — Nc = 1e5
(noise 0, evaluate_inlier_ratio's norm comparator) and the noise_ratio 2.0 set (Nc = 3e5, the
squared comparator) — one 1e5-hypothesis run each, culling on / off alternating; median ms per run,
the share of (group, tile) blocks skipped, and whether the outcomes agree.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    import numpy as np
    import torch

    from m3d import _lib, synth
    from m3d.core import RESULT_WORDS, CorrSet, RansacOutcome, RansacParams
    from matcher.ransac import inject_noise

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
    np.random.seed(3)
    c3 = inject_noise(np.asarray(corr), len(src), len(tgt), 2.0)
    thr = 0.45
    H = 100_000
    for name, c, t, mode in (("n1e5", corr, thr, _lib.SCORE_NORM), ("n3e5", c3, thr * thr, _lib.SCORE_SQUARED)):
        cs = CorrSet(src, tgt, c)
        p = RansacParams(max_iter=H, seed=42, thr=t, mode=mode, early_stop=False)
        buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
        res = {}
        for cull in (1, 0, 1, 0):
            os.environ["M3D_SCORE_CULL"] = str(cull)
            for _ in range(3):
                cs.run_async(p, buf)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                cs.run_async(p, buf)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            out = RansacOutcome.from_device(buf, cs.nc)
            skip = 0.0
            if cull:  # the skip share from one extra run with the classifier's counters on
                os.environ["M3D_CULL_STATS"] = "1"
                torch.cuda.synchronize()
                s0 = cs.ctx.stats()
                cs.run_async(p, buf)
                torch.cuda.synchronize()
                s1 = cs.ctx.stats()
                del os.environ["M3D_CULL_STATS"]
                skip = (s1[4] - s0[4]) / max(s1[5] - s0[5], 1)
            res.setdefault(cull, []).append((float(np.median(ts)), skip, out.best_index, out.best_count))
        print(f"{name}: culled {[(round(a, 3), round(b, 3)) for a, b, _, _ in res[1]]} ms/skip, "
              f"unculled {[round(a, 3) for a, _, _, _ in res[0]]} ms; same winner "
              f"{res[1][0][2:] == res[0][0][2:]} {res[1][0][2:]}", flush=True)
        del cs


if __name__ == "__main__":
    main()
