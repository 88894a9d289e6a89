"""Determinism / parity probe of the cfg2 bench batch (tests/test_gpu_ransac.py
test_cfg2_bench_batch_exact): runs the 1e5-hypothesis batch several times in one process,
compares the runs with each other and with the reference's golden counts, and re-scores every
mismatching hypothesis one at a time (the device's own transform through m3d_ransac_score, and the
oracle's transform) to tell a batch-kernel fault from a transform difference.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd"), os.path.join(HERE, "..", "tests"),
                os.path.join(HERE, "..", "oracle")]


def main():
    import numpy as np
    import torch

    import ransac_oracle as O
    from golden_pairs import cfg2_pair
    from m3d import _lib
    from m3d.core import CorrSet
    from test_gpu_ransac import THR, _run_batch

    gdir = os.path.join(HERE, "..", "tests", "golden")

    def golden(name):
        return np.load(os.path.join(gdir, name))

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    g, src, tgt, corr, noise = cfg2_pair(golden)
    full = golden("ransac_cfg2_full.npz")
    H = int(full["h"])
    for key, c, thr, mode in (("n3e5", noise, THR * THR, _lib.SCORE_SQUARED), ("n1e5", corr, THR, _lib.SCORE_NORM)):
        cs = CorrSet(src, tgt, c)
        want = full[f"batch_{key}_count"].astype(np.int64)
        free = full[f"batch_{key}_band"] == 0
        runs = [_run_batch(cs, H, thr, mode)[0] for _ in range(reps)]
        same = [int((runs[k] != runs[0]).sum()) for k in range(reps)]
        bad = np.nonzero(free & (runs[0] != want))[0]
        print(f"{key}: runs differing from run 0 in {same} hypotheses; run 0 vs golden (free) {len(bad)} mismatches",
              flush=True)
        for k in range(reps):
            bk = np.nonzero(free & (runs[k] != want))[0]
            print(f"  run {k}: mismatches {bk[:12].tolist()}", flush=True)
        allbad = sorted(set(np.nonzero((np.stack(runs) != want[None]).any(0) & free)[0].tolist()))
        if allbad:
            T, st = cs.kabsch3(H, seed=42)
            Td = T.cpu().numpy()[allbad]
            one = cs.score(Td, thr, mode).cpu().numpy()
            pp, qq = src[c[:, 0]], tgt[c[:, 1]]
            tri = O.native_triples(42, 0, H, len(c))
            To = np.stack([O.kabsch3(pp[tri[h]], qq[tri[h]])[0] for h in allbad])
            oo = cs.score(To, thr, mode).cpu().numpy()
            for j, h in enumerate(allbad[:20]):
                print(f"  hyp {h}: golden {want[h]} runs {[int(r[h]) for r in runs]} rescored(dev T) {one[j]} "
                      f"rescored(oracle T) {oo[j]} status {int(st.cpu().numpy()[h])} |dT| "
                      f"{np.abs(Td[j] - To[j]).max():.2e}", flush=True)
        del cs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
