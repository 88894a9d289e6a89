"""Fixture data rebuilt from committed golden files (tests/golden/) — test helpers."""
import numpy as np

import ransac_oracle as O


def cfg2_pair(golden):
    """bench.py's cfg2 pair regenerated from its seed, checked against the digest the generator
    recorded, and the reference's noise_ratio 2.0 set (ransac.py:88-99) rebuilt by the oracle."""
    import hashlib

    from m3d import synth

    g = golden("ransac_cfg2.npz")

    def digest(*arrays):
        h = hashlib.sha256()
        for a in arrays:
            a = np.ascontiguousarray(a)
            h.update(str((a.dtype.str, a.shape)).encode())
            h.update(a.tobytes())
        return h.hexdigest()

    src, tgt, corr, _ = synth.ransac_pair(int(g["n"]), seed=int(g["pair_seed"]))
    assert digest(src, tgt, corr) == str(g["digest"])
    np.random.seed(int(g["noise_seed"]))
    noise = np.asarray(O.inject_noise_legacy(corr, len(src), len(tgt), 2.0), np.int32)
    assert digest(noise) == str(g["noise_digest"])
    return g, src, tgt, corr, noise
