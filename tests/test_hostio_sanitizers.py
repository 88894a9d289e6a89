"""Host code under sanitizers ("optional -fsanitize=address on the host C++").

csrc/hostio.cpp — the C-ABI's ASCII parser/formatter, STL vertex merge and the content-key hash
pool — is plain C++, so it is compiled here with g++ twice, with AddressSanitizer + UBSan and with
ThreadSanitizer, together with tests/sanitize/hostio_driver.cpp, which feeds every entry point
random and adversarial inputs (round trips against strtod, malformed blocks, buffer-overrun
guards, concurrent content keys).  No GPU involved; skipped if g++ is absent."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = [ROOT / "3d-matching_amd/csrc/hostio.cpp", ROOT / "tests/sanitize/hostio_driver.cpp"]


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_hostio_under_sanitizers(tmp_path, san):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / f"hostio_{san.split(',')[0]}"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", "-pthread", "-I", str(ROOT / "include"), *map(str, SRC),
           "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, M3D_HOST_THREADS="8", ASAN_OPTIONS="detect_leaks=0",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "0 failed checks" in r.stdout
