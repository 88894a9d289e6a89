"""Per-iteration trace of cfg4's refine ICP (the tools/cfg4_refine_timing.py pair, grid NN,
two-launch loop): each step timed alone with HIP events, next to what the NN had to do at that
step's transform (scipy cKDTree on the host): sources with a target within r, the mean / max
number of targets within r, the fp32 near-ties (runner-up within 1e-5 of the best distance).
"""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    import numpy as np
    import torch
    from scipy.spatial import cKDTree

    from m3d import plyio, synth
    from m3d import _lib
    from m3d.core import Cloud, IcpLoop, context
    from matcher.ransac import global_registration
    from ply import Ply

    T = synth.random_rigid(31, rot_range=0.5, trans_range=0.5)
    with tempfile.TemporaryDirectory() as d:
        nl = 300
        v_s, f_s = synth.surface_mesh(nl, 2 * nl, seed=1)
        v_t, f_t = synth.surface_mesh(int(nl * 1.1), int(nl * 2.2), seed=2)
        plyio.write_stl(f"{d}/src.stl", synth.apply(np.linalg.inv(T), v_s), f_s)
        plyio.write_stl(f"{d}/tgt.stl", v_t, f_t)
        plyio.convert_stl_to_ply(f"{d}/src.stl", f"{d}/src.ply")
        plyio.convert_stl_to_ply(f"{d}/tgt.stl", f"{d}/tgt.ply")
        np.random.seed(0)
        src, tgt = Ply(f"{d}/src.ply", 0.3), Ply(f"{d}/tgt.ply", 0.3)
        coarse = global_registration(src, tgt, 0.3, iteration=30)
    sp = np.asarray(src.pcd.points)
    tp, tn = np.asarray(tgt.pcd.points), np.asarray(tgt.pcd.normals)
    r = 0.12
    kt = cKDTree(tp)
    loop = IcpLoop(Cloud(sp), Cloud(tp, tn), r, nn="grid")
    ctx = context()
    ctx.profile(True)
    loop.reset(coarse.transformation)
    Tk = np.array(coarse.transformation, dtype=np.float64)
    print(f"points {len(sp)} / {len(tp)}; coarse fitness {coarse.fitness:.4f}", flush=True)
    for k in range(31):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        loop.step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        nn_ms, _ = ctx.profile_read(_lib.KERNEL_NN)
        t_ms, _ = ctx.profile_read(_lib.KERNEL_TERMS)
        x = synth.apply(Tk, sp)
        dd, _ = kt.query(x, k=2, distance_upper_bound=r)
        has = np.isfinite(dd[:, 0])
        ball = kt.query_ball_point(x, r, return_length=True)
        ok = np.isfinite(dd[:, 1])
        ties = int((dd[ok, 1] - dd[ok, 0] < 1e-5).sum())
        res = loop.result()
        print(f"step {k:2d}: {ms * 1e3:7.1f} us (nn {nn_ms * 1e3:6.1f}, terms {t_ms * 1e3:6.1f})  with-nn {has.mean():.4f}  ball mean {ball.mean():6.1f} "
              f"max {ball.max():5d} >500 {(ball > 500).sum():4d}  ties {ties:4d}  "
              f"fitness {res.fitness:.5f} rmse {res.inlier_rmse:.5f} it {res.iterations} conv {res.converged}",
              flush=True)
        Tk = res.transformation
        if res.converged:
            break


if __name__ == "__main__":
    main()
