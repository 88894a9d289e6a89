"""The 128-bit content keys of the drop-in's cache (m3d.cache "content" policy; csrc/hostio.cpp
m3d_content_keys): XXH64 and XXH3-128 known answers, determinism, and that any one-byte edit of a buffer —
in place, at chunk boundaries, first or last byte — gives a new key (the property that makes the
cache exact for the reference's per-call API, ransac.py:195-236)."""
import ctypes as C

import numpy as np
import pytest

from m3d import _lib, cache


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


def test_xxh64_known_answers(lib):
    # the published XXH64 test vectors (seed 0)
    for text, want in ((b"", 0xEF46DB3751D8E999), (b"a", 0xD24EC4F1A98C6E5B), (b"abc", 0x44BC2CF5AD770999),
                       (b"Nobody inspects the spammish repetition", 0xFBCEA83C8A378BF1)):
        buf = C.create_string_buffer(text, len(text))
        assert lib.m3d_debug_xxh64(buf, len(text), 0) == want, text


def _keys(lib, arrays):
    n = len(arrays)
    bufs = (C.c_void_p * n)(*[a.ctypes.data for a in arrays])
    lens = (C.c_size_t * n)(*[a.nbytes for a in arrays])
    out = (C.c_uint64 * (2 * n))()
    assert lib.m3d_content_keys(bufs, lens, n, out) == 0
    return [(out[2 * i], out[2 * i + 1]) for i in range(n)]


def test_content_keys_exact(lib):
    rng = np.random.default_rng(0)
    a = rng.random((100_000, 3))
    b = a.copy()
    c = rng.integers(0, 1 << 20, (100_000, 2)).astype(np.int32)
    k = _keys(lib, [a, b, c])
    assert k[0] == k[1] and k[0] != k[2]                  # content, not identity
    assert _keys(lib, [c, a]) == [k[2], k[0]]             # per buffer, order-free
    raw = a.view(np.uint8).reshape(-1)
    for pos in (0, 1, 65535, 65536, 65537, 131071, raw.size // 2, raw.size - 1):
        old = raw[pos]
        raw[pos] ^= 0x01                                   # in place: same pointer, same shape
        assert _keys(lib, [a])[0] != k[0], pos
        raw[pos] = old
    assert _keys(lib, [a])[0] == k[0]
    assert _keys(lib, [a[:-1]])[0] != k[0]                 # length is part of the key
    # repeated batches from the pool agree with each other
    for _ in range(20):
        assert _keys(lib, [a, b, c]) == k


def test_cache_sees_in_place_edits():
    """corr_key under the content policy: an in-place edit of any of the three arrays changes
    the key (so the cached correspondence set is never stale)."""
    rng = np.random.default_rng(1)
    s, t = rng.random((50_000, 3)), rng.random((50_000, 3))
    c = rng.integers(0, 50_000, (50_000, 2)).astype(np.int32)
    k0 = cache.corr_key(s, t, c)
    assert cache.corr_key(s, t, c) == k0
    s[12_345, 2] = np.nextafter(s[12_345, 2], 9.0)
    k1 = cache.corr_key(s, t, c)
    assert k1 != k0
    c[49_999, 0] ^= 1
    assert cache.corr_key(s, t, c) not in (k0, k1)


def test_xxh3_128_known_answers(lib):
    """The content keys' chunk hash is XXH3-128 (long-input path, default secret, seed 0): equal to
    the xxhash package's xxh3_128 for lengths across the stripe / block / last-stripe boundaries."""
    import xxhash

    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 300_000, dtype=np.uint8)
    out = (C.c_uint64 * 2)()
    for n in (241, 255, 256, 257, 1023, 1024, 1025, 1088, 4096, 65536, 65536 + 17, 131072, 299_999):
        buf = np.ascontiguousarray(data[:n])
        assert lib.m3d_debug_xxh3_128(buf.ctypes.data, n, out) == 0
        want = xxhash.xxh3_128_intdigest(buf.tobytes())
        assert (out[1] << 64 | out[0]) == want, n
    assert lib.m3d_debug_xxh3_128(data.ctypes.data, 240, out) != 0  # short inputs: not this path


def test_content_keys_use_both_halves(lib):
    """Both 64-bit halves of a key depend on every chunk: a one-byte edit in any chunk changes
    the low AND the high word (round 3's keys chained 64-bit chunk digests; now each chunk has a
    128-bit digest), including a short tail that joins the previous chunk."""
    rng = np.random.default_rng(7)
    for nbytes in (100, 240, 241, 300_000, 65536 * 4 + 100, 65536 * 4 + 300):
        a = rng.integers(0, 256, nbytes, dtype=np.uint8)
        k0 = _keys(lib, [a])[0]
        for pos in sorted({0, nbytes // 2, nbytes - 1, min(nbytes - 1, 65536 * 4 + 50)}):
            a[pos] ^= 0x80
            k1 = _keys(lib, [a])[0]
            a[pos] ^= 0x80
            assert k1[0] != k0[0] and k1[1] != k0[1], (nbytes, pos)
    # equal prefixes of different lengths (zero padding must not collide with real zeros)
    z = np.zeros(300, np.uint8)
    assert _keys(lib, [z[:100]])[0] != _keys(lib, [z[:101]])[0]
    assert _keys(lib, [np.zeros(0, np.uint8)])[0] != _keys(lib, [z[:1]])[0]


def test_xxh3_128_sse2_kernel_known_answers():
    """The SSE2 block kernel (hosts without AVX2; forced by M3D_XXH3_SSE2) gives the same answers."""
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import ctypes as C, sys
sys.path[:0] = [sys.argv[1]]
import numpy as np, xxhash
from m3d import _lib
lib = _lib.load()
data = np.random.default_rng(5).integers(0, 256, 200_000, dtype=np.uint8)
out = (C.c_uint64 * 2)()
for n in (241, 1024, 1025, 65536 + 17, 199_999):
    assert lib.m3d_debug_xxh3_128(data.ctypes.data, n, out) == 0
    assert (out[1] << 64 | out[0]) == xxhash.xxh3_128_intdigest(data[:n].tobytes()), n
print("ok")
'''
    import os

    env = dict(os.environ, M3D_XXH3_SSE2="1")
    pkg = str(Path(__file__).resolve().parents[1] / "3d-matching_amd")
    r = subprocess.run([sys.executable, "-c", code, pkg], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
