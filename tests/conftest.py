"""Shared pytest setup: markers and import paths.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors, host logic, C-ABI symbol checks.
``-m gpu`` runs on an MI355X and calls the HIP path through the C ABI (libm3d.so).
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "3d-matching_amd"
for p in (str(PKG), str(ROOT / "oracle"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP path through libm3d.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # the C-ABI / host-code tests load libm3d.so: build it in-tree first when a fresh checkout
    # has none (hipcc cross-compiles gfx950 without a GPU; __graft_entry__.build() does the same)
    lib = PKG / "m3d" / "libm3d.so"
    if not lib.exists() and os.environ.get("M3D_NO_AUTOBUILD") != "1":
        import subprocess

        subprocess.run(["make", "-C", str(PKG / "csrc"), "-j", str(min(8, os.cpu_count() or 1))],
                       check=False, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def pts5k(golden):
    return golden("ransac_5k_points.npz")
