#!/usr/bin/env python3
"""Round-4 verdict item 5 (RANSAC scoring, exact block culling) priced on the CPU before building it.

For bench.py's cfg2 pair (Nc = 1e5 noise 0, and the noise_ratio 2.0 set, Nc = 3e5) and 2048
hypotheses of the counter sampler (seed 42): correspondences sorted into 32-row tiles by a Morton
key of p (or of (p, q) jointly), per tile the centres c_p, c_q, ρ_p = max |p − c_p| and
e = max |R0 (p − c_p) − (q − c_q)| with R0 the Kabsch rotation of the whole set.  For hypothesis
(R, t) every row of a tile satisfies | |d_i| − |d_c| | ≤ ‖R − R0‖_F ρ_p + e (d_c the residual of the
tile centre), so a tile is decided without per-row work when |d_c| ± that bound stays on one side
of the threshold.  The MFMA screen scores 32 hypotheses × 32 rows per instruction, so a block can
be skipped only when all 32 hypotheses of its group are decided for that tile — the second rate
printed.  Result (this container): noise 0: 77 % of (hypothesis, tile) pairs decided but 0.3 % of
(32-hypothesis group, tile) blocks; noise 2.0: 22–61 % / 0–6 %.  Not built.
Usage: python tools/ransac_cull_sim.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "3d-matching_amd")]
import numpy as np  # noqa: E402

import ransac_oracle as O  # noqa: E402
from m3d import synth  # noqa: E402
from matcher.ransac import inject_noise  # noqa: E402


def morton(x, bits=10):
    lo, hi = x.min(0), x.max(0)
    c = ((x - lo) / (hi - lo + 1e-12) * (2 ** bits - 1)).astype(np.int64)
    key = np.zeros(len(x), np.int64)
    for b in range(bits):
        for k in range(x.shape[1]):
            key |= ((c[:, k] >> b) & 1) << (b * x.shape[1] + k)
    return key


def analyze(src, tgt, corr, name, H=2048, tile=32, sort="p", thr=0.45):
    p, q = src[corr[:, 0]], tgt[corr[:, 1]]
    cs, ct = p.mean(0), q.mean(0)
    pc, qc = p - cs, q - ct
    U, _, Vt = np.linalg.svd(pc.T @ qc)
    R0 = Vt.T @ U.T
    if np.linalg.det(R0) < 0:
        Vt[2] *= -1
        R0 = Vt.T @ U.T
    o = np.argsort(morton(pc) if sort == "p" else morton(np.c_[pc, qc]), kind="stable")
    pc, qc = pc[o], qc[o]
    nt = len(pc) // tile
    P, Q = pc[:nt * tile].reshape(nt, tile, 3), qc[:nt * tile].reshape(nt, tile, 3)
    cp, cq = P.mean(1), Q.mean(1)
    dp, dq = P - cp[:, None], Q - cq[:, None]
    rho = np.linalg.norm(dp, axis=2).max(1)
    e = np.linalg.norm(dp @ R0.T - dq, axis=2).max(1)
    tri = O.native_triples(42, 0, H, len(corr))
    dec = np.zeros((H, nt), bool)
    for h in range(H):
        T, _ = O.kabsch3(p[tri[h]], q[tri[h]])
        R, t = T[:3, :3], T[:3, 3]
        d = np.linalg.norm(cp @ R.T + (R @ cs + t - ct) - cq, axis=1)
        r = np.linalg.norm(R - R0) * rho + e + 1e-4
        dec[h] = (d + r < thr) | (d - r > thr)
    grp = dec.reshape(H // 32, 32, nt).all(1)
    print(f"{name} sort={sort}: (hypothesis, tile) decided {dec.mean():.3f}; "
          f"(32-hypothesis group, tile) decided {grp.mean():.3f}")


def main():
    src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
    analyze(src, tgt, corr, "Nc=1e5 noise 0", sort="p")
    analyze(src, tgt, corr, "Nc=1e5 noise 0", sort="pq")
    np.random.seed(3)
    c3 = inject_noise(np.asarray(corr), len(src), len(tgt), 2.0)
    analyze(src, tgt, c3, "Nc=3e5 noise 2.0", sort="p")
    analyze(src, tgt, c3, "Nc=3e5 noise 2.0", sort="pq")


if __name__ == "__main__":
    main()
