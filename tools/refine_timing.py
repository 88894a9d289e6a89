"""Where the drop-in refine_registration's time goes (bench.py cfg1_cold.refine_registration_ms):
content keys, the two device clouds, m3d_icp_run (loop create + iterations + result), the
correspondence-set fetch — each stage synchronised and timed separately, median over --reps
calls after one warm call.  Prints one line of stage medians and the iteration count.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-matching_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    import numpy as np
    import torch

    from m3d import cache, synth
    from m3d.core import Cloud, corr_pairs, icp
    from matcher.icp import refine_registration
    from ply import Ply

    src, tgt, nrm, _ = synth.icp_pair(100000, 100000, seed=0)
    jdev = torch.from_numpy(np.arange(len(src), dtype=np.int32)).cuda()

    def staged():
        cache.clear()
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        keys = cache._content_keys([src, tgt, nrm])
        t.append(time.perf_counter())
        sc, tc = Cloud(src), Cloud(tgt, nrm)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        out = icp(sc, tc, 0.12, init=np.eye(4), with_correspondences=False)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        out2 = icp(sc, tc, 0.12, init=np.eye(4), with_correspondences=True)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        corr_pairs(sc.ctx, jdev, len(src))
        t.append(time.perf_counter())
        assert len(keys) == 3
        return [(t[k + 1] - t[k]) * 1e3 for k in range(5)], out.iterations, out2

    def whole():
        cache.clear()
        pa, pb = Ply.from_arrays(src), Ply.from_arrays(tgt, nrm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = refine_registration(pa, pb, np.eye(4), 0.3)
        return (time.perf_counter() - t0) * 1e3, res

    staged()
    whole()
    st = [staged() for _ in range(a.reps)]
    wh = [whole() for _ in range(a.reps)]
    med = np.median(np.array([s[0] for s in st]), axis=0)
    print(f"refine stages ms: keys {med[0]:.3f}  clouds {med[1]:.3f}  icp_run(no corr) {med[2]:.3f}  "
          f"icp_run(+corr fetch) {med[3]:.3f}  corr_pairs alone {med[4]:.3f}  iterations {st[0][1]}", flush=True)
    print(f"refine_registration ms: {np.median([w[0] for w in wh]):.3f} (fitness {wh[0][1].fitness:.5f})",
          flush=True)


if __name__ == "__main__":
    main()
