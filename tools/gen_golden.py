"""Generate golden vectors from the REFERENCE's own numpy code (build container only).

Imports ``/root/reference/src/matcher/ransac.py`` with ``tools/oracle_stub`` standing in for the
absent open3d wheel and records what the reference computes:

* tests/golden/ransac_5k_points.npz  — 5k-pt synthetic pair (cfg0 geometry), clean identity
  correspondences and a noise_ratio=2.0 set made by the reference's own
  ``compute_feature_correspondences`` (ransac.py:62-101; the stubbed FPFH matcher returns the
  identity pairs, the outlier injection :88-99 is the reference's code).
* tests/golden/ransac_5k_seed{0,1,42}.npz — for each correspondence set, 1000 successive
  ``compute_step_transformation`` calls after ``np.random.seed(s)``: the sampled rows (captured by
  replaying the RNG state), the 4×4 results, ``evaluate_inlier_ratio`` (voxel 0.3) and
  ``evaluate_inlier_ratio_fast`` (thr² = (0.3·1.5)²) of each.
* tests/golden/crash_kats.npz — the edge cases of test_ransac_crash.py:82-294 with asserted
  outputs (minimal/collinear/coplanar/duplicate/zero-correspondence/large-transform).
* tests/golden/loop_trajectory.npz — the step-RANSAC loop of _visualize_matcher.py:394-450
  driven by the reference's a1 + a3 (best index, best fitness, stop iteration, fitness stream).
* tests/golden/ransac_cfg2.npz — cfg2 scale (benchmark_ransac.py:105-113 at Nc = 1e5): bench.py's
  pair (m3d.synth.ransac_pair(1e5, seed=42), pinned by a SHA-256 of its arrays) and the
  reference's noise_ratio 2.0 set on it (Nc = 3e5); for np.random.seed 42 and 7, 200 successive
  compute_step_transformation calls (rows, 4×4) with their evaluate_inlier_ratio and
  evaluate_inlier_ratio_fast counts (100 calls on the noisy set).  Only the rows, transforms and
  counts are stored (the pair is regenerated from its seed).

Run:  python tools/gen_golden.py [--only cfg2]   (skips cleanly when /root/reference is absent)
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
REF_SRC = Path("/root/reference/src")
OUT = ROOT / "tests" / "golden"


class _Pts:
    def __init__(self, pts):
        self.points = pts


class MockPly:
    """Duck type of test_ransac_crash.py:92-96 (only ``pcd_down.points`` is read by a1/a2)."""

    def __init__(self, pts):
        self.pcd_down = _Pts(np.asarray(pts, dtype=np.float64))
        self.pcd = self.pcd_down
        self.pcd_fpfh = None


def main() -> int:
    if not REF_SRC.exists():
        print("reference not present; nothing to do")
        return 0
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path[:0] = [str(ROOT / "tools" / "oracle_stub"), str(REF_SRC), str(ROOT / "3d-matching_amd")]
    from matcher import ransac as ref  # the reference module
    from open3d.pipelines import registration as stubreg
    from m3d import synth

    OUT.mkdir(parents=True, exist_ok=True)
    gen_cfg2(ref, stubreg, synth)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "cfg2":
        return 0

    # ---------------- G1: 5k pair ----------------
    n = 5000
    src, tgt, corr_clean, T_true = synth.ransac_pair(n, seed=0, noise_ratio=0.0)
    stubreg.set_feature_correspondences(corr_clean)
    np.random.seed(7)
    corr_noise = np.asarray(ref.compute_feature_correspondences(MockPly(src), MockPly(tgt),
                                                                noise_ratio=2.0), dtype=np.int32)
    np.random.seed(11)
    corr_mid = np.asarray(ref.compute_feature_correspondences(MockPly(src), MockPly(tgt),
                                                              noise_ratio=0.6), dtype=np.int32)
    np.savez_compressed(OUT / "ransac_5k_points.npz", src=src, tgt=tgt, corr_clean=corr_clean,
                        corr_noise=corr_noise, corr_mid=corr_mid, T_true=T_true, voxel=0.3)
    S, Tg = MockPly(src), MockPly(tgt)
    voxel = 0.3
    thr_sq = (voxel * 1.5) * (voxel * 1.5)
    H = 1000
    for seed in (0, 1, 42):
        rec = {}
        for name, corr in (("clean", corr_clean), ("noise", corr_noise)):
            p_src = src[corr[:, 0]]
            p_tgt = tgt[corr[:, 1]]
            np.random.seed(seed)
            tri = np.empty((H, 3), dtype=np.int32)
            Ts = np.empty((H, 4, 4))
            slow = np.empty(H)
            fast = np.empty(H)
            for h in range(H):
                st = np.random.get_state()
                res = ref.compute_step_transformation(S, Tg, corr)
                after = np.random.get_state()
                np.random.set_state(st)
                tri[h] = np.random.choice(len(corr), 3, replace=False)
                chk = np.random.get_state()
                assert chk[2] == after[2] and np.array_equal(chk[1], after[1])
                Ts[h] = res.transformation
                slow[h] = ref.evaluate_inlier_ratio(S, Tg, corr, res.transformation, voxel)
                fast[h] = ref.evaluate_inlier_ratio_fast(p_src, p_tgt, res.transformation, thr_sq)
            rec[f"{name}_triples"] = tri
            rec[f"{name}_T"] = Ts
            rec[f"{name}_ratio_slow"] = slow
            rec[f"{name}_ratio_fast"] = fast
            rec[f"{name}_count_slow"] = np.rint(slow * len(corr)).astype(np.int64)
            rec[f"{name}_count_fast"] = np.rint(fast * len(corr)).astype(np.int64)
        np.savez_compressed(OUT / f"ransac_5k_seed{seed}.npz", thr_sq=thr_sq, voxel=voxel, **rec)

    # ---------------- G2: crash KATs (test_ransac_crash.py) ----------------
    kat = {}
    c3 = np.array([[0, 0], [1, 1], [2, 2]], dtype=np.int32)
    mins_src, mins_tgt, mins_T = [], [], []
    for s in range(10):
        np.random.seed(100 + s)
        a = np.random.rand(3, 3)                       # create_minimal_point_cloud(3) :36
        b = np.random.rand(3, 3)
        np.random.seed(200 + s)
        r = ref.compute_step_transformation(MockPly(a), MockPly(b), c3)
        mins_src.append(a); mins_tgt.append(b); mins_T.append(r.transformation)
    kat["minimal_src"] = np.array(mins_src)
    kat["minimal_tgt"] = np.array(mins_tgt)
    kat["minimal_T"] = np.array(mins_T)
    col = np.array([[0, 0, i] for i in range(10)], dtype=float)          # :50
    np.random.seed(5)
    kat["collinear_pts"] = col
    kat["collinear_T"] = ref.compute_step_transformation(MockPly(col), MockPly(col), c3).transformation
    np.random.seed(6)
    cop_a = np.random.rand(10, 3); cop_a[:, 2] = 0.0                      # :63-64
    cop_b = np.random.rand(10, 3); cop_b[:, 2] = 0.0
    np.random.seed(8)
    kat["coplanar_src"], kat["coplanar_tgt"] = cop_a, cop_b
    kat["coplanar_T"] = ref.compute_step_transformation(MockPly(cop_a), MockPly(cop_b), c3).transformation
    np.random.seed(8)
    kat["coplanar_self_T"] = ref.compute_step_transformation(MockPly(cop_a), MockPly(cop_a), c3).transformation
    dup = np.array([[1, 1, 1]] * 10, dtype=float)                         # :77
    np.random.seed(9)
    kat["duplicate_pts"] = dup
    kat["duplicate_T"] = ref.compute_step_transformation(MockPly(dup), MockPly(dup), c3).transformation
    z = np.zeros((0, 2), dtype=np.int32)
    ten = np.random.rand(10, 3)
    kat["zero_corr_ratio"] = ref.evaluate_inlier_ratio(MockPly(ten), MockPly(ten), z, np.eye(4), 0.3)
    kat["two_corr_T"] = ref.compute_step_transformation(MockPly(ten), MockPly(ten), c3[:2]).transformation
    large = np.eye(4)                                                     # :283-285
    large[:3, :3] *= 1000.0
    large[:3, 3] = [1000, 1000, 1000]
    kat["large_T"] = large
    kat["large_ratio_clean"] = ref.evaluate_inlier_ratio(S, Tg, corr_clean, large, 0.3)
    kat["identity_ratio_clean"] = ref.evaluate_inlier_ratio(S, Tg, corr_clean, np.eye(4), 0.3)
    kat["true_ratio_clean"] = ref.evaluate_inlier_ratio(S, Tg, corr_clean, T_true, 0.3)
    kat["true_ratio_noise"] = ref.evaluate_inlier_ratio(S, Tg, corr_noise, T_true, 0.3)
    np.savez_compressed(OUT / "crash_kats.npz", **kat)

    # ---------------- G3: step-RANSAC loop trajectory ----------------
    traj = {}
    for name, corr, max_iter, seed in (("clean", corr_clean, 500, 42), ("noise", corr_noise, 300, 3),
                                       ("mid", corr_mid, 400, 5)):
        p_src = src[corr[:, 0]]
        p_tgt = tgt[corr[:, 1]]
        np.random.seed(seed)
        best_fit, best_idx, it, fits = -1.0, -1, 0, []
        stop = max_iter
        while it < max_iter:                               # _visualize_matcher.py:394
            it += 1
            res = ref.compute_step_transformation(S, Tg, corr)
            w = ref.evaluate_inlier_ratio_fast(p_src, p_tgt, res.transformation, thr_sq)
            fits.append(w)
            if best_idx < 0 or w > best_fit:               # :426-429
                best_idx, best_fit = it - 1, w
            if best_fit > 0.5:                             # :432
                req = int(np.log(1 - 0.99) / np.log(1 - best_fit ** 3)) if best_fit >= 0.01 else max_iter
                if it >= req:
                    stop = it
                    break
        traj[f"{name}_seed"] = seed
        traj[f"{name}_max_iter"] = max_iter
        traj[f"{name}_best_index"] = best_idx
        traj[f"{name}_best_fitness"] = best_fit
        traj[f"{name}_iterations"] = stop
        traj[f"{name}_fitness"] = np.array(fits)
    np.savez_compressed(OUT / "loop_trajectory.npz", **traj)
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)
    return 0


def pair_digest(*arrays) -> str:
    import hashlib

    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str((a.dtype.str, a.shape)).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def replay_calls(ref, S, Tg, corr, seed, H, voxel):
    """H successive reference a1 calls after np.random.seed(seed): rows, 4×4, a2 and a3 counts."""
    src, tgt = S.pcd_down.points, Tg.pcd_down.points
    p_src, p_tgt = src[corr[:, 0]], tgt[corr[:, 1]]
    thr_sq = (voxel * 1.5) * (voxel * 1.5)
    np.random.seed(seed)
    tri = np.empty((H, 3), dtype=np.int32)
    Ts = np.empty((H, 4, 4))
    slow = np.empty(H, dtype=np.int64)
    fast = np.empty(H, dtype=np.int64)
    for h in range(H):
        st = np.random.get_state()
        res = ref.compute_step_transformation(S, Tg, corr)
        after = np.random.get_state()
        np.random.set_state(st)
        tri[h] = np.random.choice(len(corr), 3, replace=False)
        chk = np.random.get_state()
        assert chk[2] == after[2] and np.array_equal(chk[1], after[1])
        Ts[h] = res.transformation
        slow[h] = int(np.rint(ref.evaluate_inlier_ratio(S, Tg, corr, res.transformation, voxel) * len(corr)))
        fast[h] = int(np.rint(ref.evaluate_inlier_ratio_fast(p_src, p_tgt, res.transformation, thr_sq) * len(corr)))
    return tri, Ts, slow, fast


def gen_cfg2(ref, stubreg, synth):
    n = 100_000
    src, tgt, corr, _ = synth.ransac_pair(n, seed=42)
    S, Tg = MockPly(src), MockPly(tgt)
    stubreg.set_feature_correspondences(corr)
    np.random.seed(3)
    corr_noise = np.asarray(ref.compute_feature_correspondences(S, Tg, noise_ratio=2.0), dtype=np.int32)
    rec = dict(n=n, pair_seed=42, voxel=0.3, digest=pair_digest(src, tgt, corr),
               noise_seed=3, noise_digest=pair_digest(corr_noise))
    for seed in (42, 7):
        tri, Ts, slow, fast = replay_calls(ref, S, Tg, corr, seed, 200, 0.3)
        rec.update({f"s{seed}_triples": tri, f"s{seed}_T": Ts, f"s{seed}_count_slow": slow,
                    f"s{seed}_count_fast": fast})
    tri, Ts, slow, fast = replay_calls(ref, S, Tg, corr_noise, 42, 100, 0.3)
    rec.update(noise_triples=tri, noise_T=Ts, noise_count_slow=slow, noise_count_fast=fast)
    np.savez_compressed(OUT / "ransac_cfg2.npz", **rec)
    print("ransac_cfg2.npz", (OUT / "ransac_cfg2.npz").stat().st_size)


if __name__ == "__main__":
    raise SystemExit(main())
