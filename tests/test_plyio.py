"""PLY / STL I/O (m3d.plyio): round trips and hand-written files of every supported layout.

Reference readers (Open3D read_point_cloud, trimesh) are not installed — parity unpinned; the
files here are written byte by byte from the PLY/STL specifications.
"""
import struct

import numpy as np
import pytest

from m3d import plyio


@pytest.mark.parametrize("binary", [False, True])
@pytest.mark.parametrize("dtype", ["double", "float"])
@pytest.mark.parametrize("with_normals", [False, True])
def test_round_trip(tmp_path, binary, dtype, with_normals):
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(257, 3)) * 10
    nrm = rng.normal(size=(257, 3)) if with_normals else None
    p = tmp_path / "a.ply"
    plyio.write_ply(p, pts, nrm, binary=binary, dtype=dtype)
    got, gn = plyio.read_ply(p)
    cast = np.float64 if dtype == "double" else np.float32
    # binary float → the float32 value; ASCII values parse as double (as rply/strtod do), so a
    # printed float32 re-rounds to that float32
    np.testing.assert_array_equal(got.astype(cast), pts.astype(cast))
    if with_normals:
        np.testing.assert_array_equal(gn.astype(cast), nrm.astype(cast))
    else:
        assert gn is None


def test_big_endian_with_extra_props_and_faces(tmp_path):
    pts = np.array([[1.5, -2.0, 3.25], [0.0, 1.0, 2.0], [4.0, 5.0, 6.0]])
    head = ("ply\nformat binary_big_endian 1.0\ncomment made by hand\n"
            "element vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
            "property uchar red\nproperty uchar green\nproperty uchar blue\n"
            "element face 1\nproperty list uchar int vertex_indices\nend_header\n").encode()
    body = b"".join(struct.pack(">fffBBB", *p, 1, 2, 3) for p in pts)
    body += struct.pack(">Biii", 3, 0, 1, 2)
    (tmp_path / "b.ply").write_bytes(head + body)
    got, nrm = plyio.read_ply(tmp_path / "b.ply")
    np.testing.assert_array_equal(got, pts)
    assert nrm is None


def test_element_before_vertices_is_skipped(tmp_path):
    head = ("ply\nformat binary_little_endian 1.0\nelement camera 2\nproperty list uchar float k\n"
            "property int id\nelement vertex 2\nproperty double x\nproperty double y\n"
            "property double z\nproperty double nx\nproperty double ny\nproperty double nz\n"
            "end_header\n").encode()
    body = struct.pack("<Bffi", 2, 1.0, 2.0, 7) + struct.pack("<Bi", 0, 8)
    body += struct.pack("<6d", 1, 2, 3, 0, 0, 1) + struct.pack("<6d", 4, 5, 6, 1, 0, 0)
    (tmp_path / "c.ply").write_bytes(head + body)
    pts, nrm = plyio.read_ply(tmp_path / "c.ply")
    np.testing.assert_array_equal(pts, [[1, 2, 3], [4, 5, 6]])
    np.testing.assert_array_equal(nrm, [[0, 0, 1], [1, 0, 0]])


def test_ascii_int_coordinates_and_blank_lines(tmp_path):
    text = ("ply\nformat ascii 1.0\nelement vertex 3\nproperty int x\nproperty int y\n"
            "property int z\nelement face 0\nproperty list uchar int vertex_indices\nend_header\n"
            "1 2 3\n\n4 5 6\n7 8 9\n")
    (tmp_path / "d.ply").write_text(text)
    pts, _ = plyio.read_ply(tmp_path / "d.ply")
    np.testing.assert_array_equal(pts, np.arange(1, 10).reshape(3, 3))


@pytest.mark.parametrize("text,err", [
    ("plx\n", "magic"),
    ("ply\nformat ascii 1.0\nelement face 0\nend_header\n", "no vertex"),
    ("ply\nformat binary_little_endian 1.0\nelement vertex 5\nproperty float x\nproperty float y\n"
     "property float z\nend_header\n", "truncated"),
    ("ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\nend_header\n1\n", "x/y/z"),
])
def test_malformed_files_raise(tmp_path, text, err):
    (tmp_path / "e.ply").write_bytes(text.encode())
    with pytest.raises(plyio.PlyError, match=err):
        plyio.read_ply(tmp_path / "e.ply")


def _tetra():
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float64)
    f = np.array([[0, 2, 1], [0, 1, 3], [0, 3, 2], [1, 2, 3]])
    return v, f


def test_binary_stl_merges_shared_vertices(tmp_path):
    v, f = _tetra()
    raw = b"\0" * 80 + struct.pack("<I", len(f))
    for tri in f:
        raw += struct.pack("<3f", 0, 0, 0) + struct.pack("<9f", *v[tri].ravel()) + b"\0\0"
    (tmp_path / "t.stl").write_bytes(raw)
    verts, faces = plyio.read_stl(tmp_path / "t.stl")
    assert len(verts) == 4
    np.testing.assert_array_equal(verts[faces], v[f])       # faces reference the merged vertices
    np.testing.assert_array_equal(verts, v[[0, 2, 1, 3]])   # first-occurrence order


def test_ascii_stl_and_convert(tmp_path):
    v, f = _tetra()
    lines = ["solid t"]
    for tri in f:
        lines += ["facet normal 0 0 0", "outer loop"] + [f"vertex {a} {b} {c}" for a, b, c in v[tri]]
        lines += ["endloop", "endfacet"]
    lines.append("endsolid t")
    (tmp_path / "t.stl").write_text("\n".join(lines))
    n = plyio.convert_stl_to_ply(tmp_path / "t.stl", tmp_path / "t.ply")
    assert n == 4
    pts, _ = plyio.read_ply(tmp_path / "t.ply")
    assert sorted(map(tuple, pts)) == sorted(map(tuple, v))


def test_ply_class_checks_like_reference(tmp_path):
    from ply import Ply

    with pytest.raises(FileNotFoundError):
        Ply(tmp_path / "missing.ply")
    (tmp_path / "x.txt").write_text("x")
    with pytest.raises(TypeError):
        Ply(tmp_path / "x.txt")


@pytest.mark.parametrize("binary", [True, False])
def test_stl_writer_round_trip_on_generated_mesh(tmp_path, binary):
    """m3d.synth.surface_mesh → write_stl → read_stl: a closed mesh (every edge in two faces),
    vertices merged back exactly (float32 STL payload), faces preserved."""
    from m3d import synth

    v, f = synth.surface_mesh(20, 40, seed=4)
    e = np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1)
    assert set(np.unique(np.unique(e, axis=0, return_counts=True)[1])) == {2}
    plyio.write_stl(tmp_path / "m.stl", v, f, binary=binary)
    vv, ff = plyio.read_stl(tmp_path / "m.stl")
    v32 = v.astype(np.float32).astype(np.float64)
    if binary:
        np.testing.assert_array_equal(vv, v32)
    else:  # ASCII holds 9 significant digits of each float32 coordinate
        np.testing.assert_allclose(vv, v32, rtol=1e-8, atol=1e-12)
    np.testing.assert_array_equal(ff, f)
    assert plyio.convert_stl_to_ply(tmp_path / "m.stl", tmp_path / "m.ply") == len(v)
    np.testing.assert_array_equal(plyio.read_ply(tmp_path / "m.ply")[0], vv)


def test_native_ascii_parser_equals_numpy():
    """csrc/hostio.cpp (m3d_parse_ascii_rows): the doubles numpy's own parser returns, on
    extreme magnitudes, integers, signed zeros, tabs, CRLF, blank lines and trailing spaces."""
    import ctypes as C

    from m3d import _lib

    lib = _lib.load()
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.normal(size=600) * 10.0 ** rng.integers(-300, 300, 600),
                           [0.0, -0.0, 1.0, -7.0, 5e-324, 1.7976931348623157e308, 0.1, 1 / 3]])
    vals = vals[: len(vals) // 3 * 3].reshape(-1, 3)
    lines = []
    for k, row in enumerate(vals):
        sep = "\t" if k % 5 == 0 else " "
        txt = sep.join(repr(float(v)) if k % 2 else f"{v:.17g}" for v in row)
        lines.append(txt + ("  " if k % 7 == 0 else "") + ("\r\n" if k % 3 == 0 else "\n"))
        if k % 11 == 0:
            lines.append("\n")
    buf = "".join(lines).encode() + b"trailing element data\n"
    out = np.empty_like(vals)
    used = C.c_size_t(0)
    assert lib.m3d_parse_ascii_rows(buf, len(buf), len(vals), 3,
                                    out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(used)) == 0
    exp = np.loadtxt([l for l in lines if l.strip()], dtype=np.float64)
    np.testing.assert_array_equal(out.view(np.uint64), exp.view(np.uint64))  # bit for bit
    assert buf[used.value:] == b"trailing element data\n"
    # short input, extra tokens and non-numbers are refused (plyio then uses numpy)
    for bad, rows in ((b"1 2 3\n", 2), (b"1 2 3 4\n", 1), (b"1 2 x\n", 1), (b"+1 2 3\n", 1)):
        assert lib.m3d_parse_ascii_rows(bad, len(bad), rows, 3, out.ctypes.data_as(C.POINTER(C.c_double)),
                                        C.byref(used)) != 0


def test_native_ascii_writer_round_trips_and_plus_sign_fallback(tmp_path):
    rng = np.random.default_rng(4)
    pts = rng.normal(size=(1000, 3)) * 10.0 ** rng.integers(-200, 200, (1000, 1))
    pts[0] = [-0.0, 5e-324, 1.7976931348623157e308]
    p = tmp_path / "w.ply"
    plyio.write_ply(p, pts, binary=False, dtype="double")
    got, _ = plyio.read_ply(p)
    np.testing.assert_array_equal(got.view(np.uint64), pts.view(np.uint64))
    # a file the native parser refuses ('+' signs) still reads through numpy
    q = tmp_path / "plus.ply"
    q.write_text("ply\nformat ascii 1.0\nelement vertex 2\nproperty double x\nproperty double y\n"
                 "property double z\nend_header\n+1.5 2 3\n4 +5e1 6\n")
    got, _ = plyio.read_ply(q)
    np.testing.assert_array_equal(got, [[1.5, 2, 3], [4, 50, 6]])


def test_native_vertex_merge_equals_numpy_merge():
    """csrc/hostio.cpp m3d_merge_vertices = plyio._merge_numpy: first-occurrence order, exact
    equality with -0.0 ≡ +0.0, on shared corners, duplicates and signed zeros."""
    from m3d import synth

    v, f = synth.surface_mesh(40, 80, seed=5)
    corners = v[f].reshape(-1, 3).astype(np.float32).astype(np.float64)
    corners[::97] = [-0.0, 0.0, 1.0]
    corners[1::101] = [0.0, -0.0, 1.0]
    ref_v, ref_f = plyio._merge_numpy(corners)
    import ctypes as C

    uniq = np.empty_like(corners)
    inv = np.empty(len(corners), np.int32)
    m = C.c_int64(0)
    P = C.POINTER(C.c_double)
    assert plyio._text_lib().m3d_merge_vertices(corners.ctypes.data_as(P), len(corners), uniq.ctypes.data_as(P),
                                                inv.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(m)) == 0
    np.testing.assert_array_equal(uniq[: m.value], ref_v)
    np.testing.assert_array_equal(inv.reshape(-1, 3), ref_f)


@pytest.mark.parametrize("n,k", [(12, 3), (300000, 100000), (200001, 7)])
def test_native_vertex_merge_table_growth(n, k):
    """The merge table starts at n / 4 slots and doubles at half load: mostly-unique inputs
    (several doublings), few-unique inputs and tiny inputs all equal the numpy merge."""
    import ctypes as C

    rng = np.random.default_rng(n)
    base = rng.integers(-50, 50, size=(k, 3)).astype(np.float64) * 0.5
    base[rng.random(k) < 0.1, 0] = -0.0
    flat = np.ascontiguousarray(base[rng.integers(0, k, n)])
    uniq = np.empty_like(flat)
    inv = np.empty(n, np.int32)
    m = C.c_int64(0)
    P = C.POINTER(C.c_double)
    assert plyio._text_lib().m3d_merge_vertices(flat.ctypes.data_as(P), n, uniq.ctypes.data_as(P),
                                                inv.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(m)) == 0
    ref_v, ref_f = plyio._merge_numpy(flat)
    np.testing.assert_array_equal(uniq[: m.value], ref_v)
    np.testing.assert_array_equal(inv, ref_f.reshape(-1))


def test_native_ascii_parser_large_input():
    """A multi-megabyte vertex block: the same doubles, blank lines and CRLF anywhere, the rows
    stop exactly at the declared count even when numeric rows (faces) follow, and errors deep
    inside or a short block are reported."""
    import ctypes as C

    from m3d import _lib

    lib = _lib.load()
    rng = np.random.default_rng(11)
    n = 60000
    vals = rng.normal(size=(n, 3)) * 10.0 ** rng.integers(-5, 5, (n, 1))
    lines = []
    for k, row in enumerate(vals):
        lines.append(" ".join(repr(float(v)) for v in row) + ("\r\n" if k % 3 == 0 else "\n"))
        if k % 97 == 0:
            lines.append(" \t\n")
    faces = "".join(f"3 {k} {k + 1} {k + 2}\n" for k in range(500))
    buf = "".join(lines).encode() + faces.encode()
    assert len(buf) > 1 << 20
    out = np.empty_like(vals)
    used = C.c_size_t(0)
    P = C.POINTER(C.c_double)
    assert lib.m3d_parse_ascii_rows(buf, len(buf), n, 3, out.ctypes.data_as(P), C.byref(used)) == 0
    np.testing.assert_array_equal(out, vals)
    assert buf[used.value:] == faces.encode()
    # a bad row deep inside, and a declared count beyond the rows present, are refused
    bad = bytearray(buf)
    pos = len(buf) * 2 // 3
    pos = buf.index(b"\n", pos) + 1
    bad[pos:pos + 1] = b"x"
    assert lib.m3d_parse_ascii_rows(bytes(bad), len(bad), n, 3, out.ctypes.data_as(P), C.byref(used)) != 0
    short = "".join(lines).encode()
    assert lib.m3d_parse_ascii_rows(short, len(short), n + 1, 3, out.ctypes.data_as(P), C.byref(used)) != 0


def test_native_ascii_parser_fast_path_exact():
    """hostio.cpp's fast decimal path (≤ 19 significant digits, |exponent| ≤ 27, one x87
    extended operation, results near a double halfway point sent to std::from_chars) returns the
    correctly rounded double: random values in the formats point files use, exact ties between
    two doubles, 19 / 20-digit mantissas, signed zeros and exponent spellings — bit for bit
    against Python's float() (correctly rounded), on a block large enough for the threaded path."""
    import ctypes as C

    from m3d import _lib

    lib = _lib.load()
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-10, 10, 40000), rng.normal(size=20000) * 10.0 ** rng.integers(-12, 12, 20000),
                        rng.uniform(-5, 5, 20000).astype(np.float32).astype(np.float64)])
    fmts = ["{!r}", "{:.17g}", "{:.16g}", "{:.15g}", "{:.9g}", "{:.6f}", "{:.3e}", "{:.12E}"]
    toks = [fmts[k % len(fmts)].format(float(v)) for k, v in enumerate(x)]
    toks += ["9007199254740993e1", "9007199254740993", "9007199254740995e-1", "4503599627370497.5",
             "1234567890123456789", "12345678901234567890", "0.1234567890123456789", "-0.0", "0.000",
             ".5", "5.", "1e5", "1E+05", "2.5e-27", "2.5e27", "7e-28", "7e28", "123456789012345678e-27"]
    toks += toks[-18:] * 2
    toks = toks[: len(toks) // 3 * 3]
    buf = ("\n".join(" ".join(toks[i:i + 3]) for i in range(0, len(toks), 3)) + "\n").encode()
    rows = len(toks) // 3
    out = np.empty((rows, 3))
    used = C.c_size_t(0)
    assert lib.m3d_parse_ascii_rows(buf, len(buf), rows, 3, out.ctypes.data_as(C.POINTER(C.c_double)),
                                    C.byref(used)) == 0
    exp = np.array([float(t) for t in toks]).reshape(-1, 3)
    np.testing.assert_array_equal(out.view(np.uint64), exp.view(np.uint64))


def test_native_ascii_writer_threaded_equals_serial():
    """Blocks past 32k numbers are formatted on several threads: the text equals the serial
    formatting of the same rows piece by piece, and reads back bit for bit."""
    import ctypes as C

    from m3d import _lib

    lib = _lib.load()
    rng = np.random.default_rng(8)
    data = rng.normal(size=(50001, 3)) * 10.0 ** rng.integers(-30, 30, (50001, 1))
    P = C.POINTER(C.c_double)

    def fmt(block):
        block = np.ascontiguousarray(block)
        buf = C.create_string_buffer(block.size * 25 + 64)
        n = C.c_size_t(0)
        assert lib.m3d_format_ascii_rows(block.ctypes.data_as(P), len(block), block.shape[1], buf,
                                         len(buf), C.byref(n)) == 0
        return buf.raw[: n.value]

    whole = fmt(data)
    pieces = b"".join(fmt(data[i:i + 5000]) for i in range(0, len(data), 5000))  # serial each
    assert whole == pieces
    back = np.array(whole.split(), dtype=np.float64).reshape(-1, 3)
    np.testing.assert_array_equal(back.view(np.uint64), data.view(np.uint64))


def test_text_paths_without_the_library(tmp_path, monkeypatch):
    """No loadable libm3d (no build, no HIP/RCCL runtime): ASCII PLY read / write and the STL
    vertex merge take their numpy paths and give the same values as the library's."""
    rng = np.random.default_rng(5)
    pts = rng.normal(size=(300, 3)) * 7
    nrm = rng.normal(size=(300, 3))
    with_lib = tmp_path / "lib.ply"
    plyio.write_ply(with_lib, pts, nrm, binary=False)
    ref = plyio.read_ply(with_lib)
    tri = rng.normal(size=(40, 3))
    faces = rng.integers(0, 40, (90, 3))
    plyio.write_stl(tmp_path / "m.stl", tri, faces, binary=True)
    ref_stl = plyio.read_stl(tmp_path / "m.stl")

    monkeypatch.setattr(plyio, "_text_lib", lambda: None)
    no_lib = tmp_path / "nolib.ply"
    plyio.write_ply(no_lib, pts, nrm, binary=False)
    assert no_lib.read_bytes() == with_lib.read_bytes()   # shortest round-trip text both ways
    for path in (with_lib, no_lib):
        got = plyio.read_ply(path)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
    got_stl = plyio.read_stl(tmp_path / "m.stl")
    np.testing.assert_array_equal(got_stl[0], ref_stl[0])
    np.testing.assert_array_equal(got_stl[1], ref_stl[1])
