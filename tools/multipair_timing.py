"""refine_registration over a stream of distinct pairs (cfg1 size), as a caller registering many
scans would: each call uploads two new clouds, and once the cache is full (8 objects) inserting
them evicts — destroys — older ones inside the call.  Median ms per call over the evicting calls,
next to the cold call with the cache cleared outside the timed region (bench cfg1_cold)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    import numpy as np
    import torch

    from m3d import cache, synth
    from matcher.icp import refine_registration
    from ply import Ply

    pairs = []
    for k in range(14):
        s, t, n, _ = synth.icp_pair(100_000, 100_000, seed=100 + k)
        pairs.append((Ply.from_arrays(s), Ply.from_arrays(t, normals=n)))
    refine_registration(pairs[0][0], pairs[0][1], np.eye(4), 0.3)
    cache.clear()
    torch.cuda.synchronize()
    ts = []
    for k in range(1, 14):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        refine_registration(pairs[k][0], pairs[k][1], np.eye(4), 0.3)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    cold = []
    for k in range(1, 6):
        cache.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        refine_registration(pairs[k][0], pairs[k][1], np.eye(4), 0.3)
        torch.cuda.synchronize()
        cold.append((time.perf_counter() - t0) * 1e3)
    print(f"per-call ms over distinct pairs: {[round(t, 2) for t in ts]}", flush=True)
    print(f"evicting calls (5..13) median {np.median(ts[4:]):.3f} ms; cold with the cache cleared outside "
          f"the timing median {np.median(cold):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
