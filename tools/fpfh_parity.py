#!/usr/bin/env python3
"""FPFH parity, measured: the device FPFH against the CPU restatement
(oracle/prep_oracle.py, glibc acos/atan2) on
  (a) the FPFH test cloud of tests/test_gpu_prep.py (2,500 points, radius-0.8 normals), and
  (b) cfg4's generated scans (bench.py bench_cfg4: two tessellations of the synthetic surface →
      binary STL → PLY → voxel 0.3 → normals (0.6, 30) → FPFH (1.5, 100)),
then what a differing row changes downstream: the a5 correspondences (mutual filter, ransac.py:85)
and the a6 outcome (RegistrationRANSACBasedOnCorrespondence with the reference's checkers,
ransac.py:20-59) computed from the device features and from the oracle features.
Both FPFHs take the same points and the same (device) normals, so only the FPFH differs.
Prints one JSON line per cloud."""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "3d-matching_amd"), str(ROOT / "oracle")]
import numpy as np

import prep_oracle as P
from m3d import _lib

if os.environ.get("AB_LIB"):  # another build of libm3d.so (tools/ab_build.sh)
    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d import plyio, prep, synth


def compare(name, pts, nrm, radius, max_nn=100, down_pair=None):
    t0 = time.perf_counter()
    got = prep.compute_fpfh(pts, nrm, radius, max_nn)
    ref = P.compute_fpfh(pts, nrm, radius, max_nn)
    exact = np.all(got == ref, axis=1)
    close = np.all(np.abs(got - ref) <= 1e-12 * np.maximum(1.0, np.abs(ref)), axis=1)
    out = {"cloud": name, "points": len(pts), "rows_bit_exact": int(exact.sum()),
           "rows_within_1e-12": int(close.sum()), "rows_differing_1e-12": int((~close).sum()),
           "max_abs_diff": float(np.abs(got - ref).max()), "oracle_s": round(time.perf_counter() - t0, 1)}
    return got, ref, out


def main():
    res = []
    # (a) the unit-test cloud
    pts, _ = synth.surface_points(2500, seed=5)
    nrm = P.estimate_normals(pts, 0.8, 30)
    _, _, o = compare("test_gpu_prep (2500 pts, normals r=0.8)", pts, nrm, 2.0)
    res.append(o)
    print(json.dumps(o), flush=True)
    # (b) cfg4 scans (bench.py bench_cfg4 geometry, mesh 300 rings)
    T = synth.random_rigid(31, rot_range=0.5, trans_range=0.5)
    nl = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    with tempfile.TemporaryDirectory() as d:
        v_s, f_s = synth.surface_mesh(nl, 2 * nl, seed=1)
        v_t, f_t = synth.surface_mesh(int(nl * 1.1), int(nl * 2.2), seed=2)
        plyio.write_stl(f"{d}/src.stl", synth.apply(np.linalg.inv(T), v_s), f_s)
        plyio.write_stl(f"{d}/tgt.stl", v_t, f_t)
        feats = {}
        for side in ("src", "tgt"):
            plyio.convert_stl_to_ply(f"{d}/{side}.stl", f"{d}/{side}.ply")
            p, n = plyio.read_ply(f"{d}/{side}.ply")
            down, down_prev = prep.voxel_down_sample(p, 0.3, normals=n)
            down = down.cpu().numpy() if hasattr(down, "cpu") else np.asarray(down)
            down_prev = None if down_prev is None else (down_prev.cpu().numpy() if hasattr(down_prev, "cpu")
                                                        else np.asarray(down_prev))
            dn = prep.estimate_normals(down, 0.6, 30, normals=down_prev)
            got, ref, o = compare(f"cfg4 {side} scan (voxel 0.3)", down, dn, 1.5)
            feats[side] = (down, got, ref)
            res.append(o)
            print(json.dumps(o), flush=True)
        (sp, fs_dev, fs_orc), (tp, ft_dev, ft_orc) = feats["src"], feats["tgt"]
        c_dev = prep.feature_correspondences(fs_dev, ft_dev, True)
        c_orc = prep.feature_correspondences(fs_orc, ft_orc, True)
        sd, so = {tuple(x) for x in c_dev.tolist()}, {tuple(x) for x in c_orc.tolist()}
        down_out = {"a5_correspondences_device": len(c_dev), "a5_correspondences_oracle_features": len(c_orc),
                    "a5_pairs_only_device": len(sd - so), "a5_pairs_only_oracle": len(so - sd),
                    "a5_identical": bool(np.array_equal(c_dev, c_orc))}
        kw = dict(edge_length=0.9, distance=0.45, confidence=0.999, seed=0)
        for it in (30, 30000):
            a = prep.ransac_on_correspondences(sp, tp, c_dev, 0.45, max_iteration=it, **kw)
            b = prep.ransac_on_correspondences(sp, tp, c_orc, 0.45, max_iteration=it, **kw)
            down_out[f"a6_iter{it}"] = {
                "device": [a.best_index, a.validations, a.fitness, a.inlier_rmse],
                "oracle_features": [b.best_index, b.validations, b.fitness, b.inlier_rmse],
                "identical": bool(a.best_index == b.best_index and a.validations == b.validations
                                  and a.fitness == b.fitness and np.array_equal(a.transformation, b.transformation))}
        print(json.dumps(down_out), flush=True)


if __name__ == "__main__":
    main()
