"""Debug probe of the grid NN deferral (run with the M3D_DEBUG_GUARDS build and M3D_GRID_HEAVY=8):
one loop stepped with a sync after every step, then two loops interleaved as in
tests/test_gpu_icp.py::test_graph_replay_matches_enqueued_steps."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    import numpy as np
    import torch

    from m3d import synth
    from m3d.core import Cloud, IcpLoop

    src, tgt, nrm, _ = synth.icp_pair(30000, seed=13)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=80, nn="grid", persist=False)
    T0 = synth.random_rigid(5, rot_range=0.02, trans_range=0.03)
    a = IcpLoop(s, t, 0.12, **kw)
    a.reset(T0)
    for k in range(4):
        print(f"--- one loop, step {k}", flush=True)
        a.step()
        torch.cuda.synchronize()
    b = IcpLoop(s, t, 0.12, **kw)
    for lp in (a, b):
        lp.reset(T0)
    torch.cuda.synchronize()
    for k in range(3):
        print(f"--- a.step {k}", flush=True)
        a.step()
        torch.cuda.synchronize()
    for k in range(3):
        print(f"--- b.step {k}", flush=True)
        b.step()
        torch.cuda.synchronize()
    print("--- a.steps(6)", flush=True)
    a.steps(6)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
