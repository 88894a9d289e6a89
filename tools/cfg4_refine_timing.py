"""cfg4's cold refine_registration (bench.py bench_cfg4: generated STL scans → Ply(0.3) → RANSAC →
refine) split into stages: content keys, clouds, m3d_icp_run (with M3D_RUN_PROF=1 /
M3D_CREATE_PROF=1 for its own stages), median over --reps cold calls (cache cleared each time).
"""
import argparse
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]
if os.environ.get("AB_LIB"):  # time another build of libm3d.so (tools/ab_build.sh)
    from pathlib import Path

    from m3d import _lib

    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mesh", type=int, default=300)
    a = ap.parse_args()
    import numpy as np
    import torch

    from m3d import cache, plyio, synth
    from m3d.core import Cloud, icp
    from matcher.icp import refine_registration
    from matcher.ransac import global_registration
    from ply import Ply

    T = synth.random_rigid(31, rot_range=0.5, trans_range=0.5)
    with tempfile.TemporaryDirectory() as d:
        nl = a.mesh
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
        print(f"points {len(sp)} / {len(tp)}, dtypes {sp.dtype} {tp.dtype} {tn.dtype}, "
              f"contiguous {sp.flags.c_contiguous} {tp.flags.c_contiguous} {tn.flags.c_contiguous}", flush=True)
        rows = []
        sc = tc = out = None
        for _ in range(a.reps + 1):
            del sc, tc, out  # the previous clouds' hipFree outside the timed stages
            cache.clear()
            torch.cuda.synchronize()
            t = [time.perf_counter()]
            keys = cache._content_keys([sp, tp, tn])
            t.append(time.perf_counter())
            sc, tc = Cloud(sp), Cloud(tp, tn)
            torch.cuda.synchronize()
            t.append(time.perf_counter())
            out = icp(sc, tc, 0.12, init=coarse.transformation)
            torch.cuda.synchronize()
            t.append(time.perf_counter())
            cache.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = refine_registration(src, tgt, coarse.transformation, 0.3)
            t.append(t0)
            t.append(time.perf_counter())
            rows.append([(t[1] - t[0]) * 1e3, (t[2] - t[1]) * 1e3, (t[3] - t[2]) * 1e3, (t[5] - t[4]) * 1e3,
                         out.iterations])
        m = np.median(np.array(rows[1:]), axis=0)
        print(f"cfg4 cold refine stages ms: keys {m[0]:.3f} clouds {m[1]:.3f} icp_run {m[2]:.3f} "
              f"(iterations {int(m[4])}); refine_registration {m[3]:.3f}", flush=True)


if __name__ == "__main__":
    main()
