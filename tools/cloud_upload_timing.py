"""Where cfg4's cloud creation goes (180k / 218k points, as tools/cfg4_refine_timing.py):
m3d Cloud from host arrays vs from device tensors (no upload), against torch's own pageable and
pinned H2D copies of the same arrays; median ms over --reps."""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-matching_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--ns", type=int, default=180002)
    ap.add_argument("--nt", type=int, default=217802)
    a = ap.parse_args()
    import numpy as np
    import torch

    from m3d.core import Cloud

    rng = np.random.default_rng(0)
    sp = rng.normal(size=(a.ns, 3))
    tp, tn = rng.normal(size=(a.nt, 3)), rng.normal(size=(a.nt, 3))

    def med(fn):
        ts = []
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            keep = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            del keep
        return float(np.median(ts[1:]))

    dev = [torch.from_numpy(x).cuda() for x in (sp, tp, tn)]
    pin = [torch.from_numpy(x).pin_memory() for x in (sp, tp, tn)]
    rows = {
        "m3d host src": med(lambda: Cloud(sp)),
        "m3d host tgt+nrm": med(lambda: Cloud(tp, tn)),
        "m3d host both": med(lambda: (Cloud(sp), Cloud(tp, tn))),
        "m3d device both": med(lambda: (Cloud(dev[0]), Cloud(dev[1], dev[2]))),
        "m3d device src": med(lambda: Cloud(dev[0])),
        "torch empty 2 blocks (alloc)": med(lambda: (torch.empty(a.ns * 7, dtype=torch.float64, device="cuda"),
                                                    torch.empty(a.nt * 10, dtype=torch.float64, device="cuda"))),
        "torch pageable H2D (3 arrays)": med(lambda: [torch.from_numpy(x).cuda() for x in (sp, tp, tn)]),
        "torch pinned H2D (3 arrays)": med(lambda: [x.cuda(non_blocking=True) for x in pin]),
        "torch pageable H2D src only": med(lambda: torch.from_numpy(sp).cuda()),
    }
    mb = (sp.nbytes + tp.nbytes + tn.nbytes) / 1e6
    print(f"arrays {mb:.1f} MB", flush=True)
    for k, v in rows.items():
        print(f"{k:32s} {v:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
