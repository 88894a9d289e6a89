"""PLY / STL point I/O (host side, feeds cfg4).

Replaces the two readers the reference path touches:

* ``o3d.io.read_point_cloud(path)`` for ``.ply`` (``src/ply/ply.py:80``): vertex positions
  ``x y z`` and, when present, normals ``nx ny nz``.  Formats: ``ascii 1.0``,
  ``binary_little_endian 1.0``, ``binary_big_endian 1.0``; every PLY scalar type
  (``char/int8 … double/float64``) for any vertex property; list properties and other elements
  (faces, edges) are parsed only as far as needed to skip them.
* ``convert_stl-ply.py`` (trimesh 4.11.1, not installed — parity unpinned): STL (binary or
  ASCII) → unique vertices → ASCII PLY point cloud.  Vertices are merged on exact equality and
  kept in first-occurrence order (trimesh merges within 1e-8; scans never differ by less).

Readers return fp64 arrays (N×3) — the reference converts to ``Vector3dVector`` (fp64).
Binary payloads are decoded with one numpy structured-dtype view, so a 1M-point file reads in
milliseconds.
"""

from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


class PlyError(ValueError):
    pass


def _parse_header(f):
    first = f.readline()
    if first.strip() != b"ply":
        raise PlyError("not a PLY file (missing 'ply' magic)")
    fmt = None
    elements = []  # [name, count, [(prop, type) | (prop, ('list', count_type, item_type))]]
    while True:
        line = f.readline()
        if not line:
            raise PlyError("PLY header has no end_header")
        tok = line.decode("ascii", "replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
            if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
                raise PlyError(f"unsupported PLY format {fmt!r}")
        elif tok[0] == "element":
            elements.append([tok[1], int(tok[2]), []])
        elif tok[0] == "property":
            if not elements:
                raise PlyError("property before element")
            if tok[1] == "list":
                elements[-1][2].append((tok[4], ("list", _ptype(tok[2]), _ptype(tok[3]))))
            else:
                elements[-1][2].append((tok[2], _ptype(tok[1])))
        elif tok[0] == "end_header":
            break
    if fmt is None:
        raise PlyError("PLY header has no format line")
    return fmt, elements


def _ptype(name):
    try:
        return _PLY_TYPES[name]
    except KeyError:
        raise PlyError(f"unknown PLY property type {name!r}") from None


def _skip_binary_element(f, count, props, endian):
    if all(not isinstance(t, tuple) for _, t in props):
        f.seek(count * sum(np.dtype(t).itemsize for _, t in props), 1)
        return
    for _ in range(count):  # list properties: variable length rows
        for _, t in props:
            if isinstance(t, tuple):
                n = int(np.frombuffer(f.read(np.dtype(t[1]).itemsize), endian + t[1])[0])
                f.seek(n * np.dtype(t[2]).itemsize, 1)
            else:
                f.seek(np.dtype(t).itemsize, 1)


def read_ply(path):
    """Read vertices of a PLY file → ``(points N×3 f64, normals N×3 f64 or None)``."""
    path = Path(path)
    with open(path, "rb") as f:
        fmt, elements = _parse_header(f)
        endian = {"binary_little_endian": "<", "binary_big_endian": ">"}.get(fmt, "")
        for name, count, props in elements:
            if name == "vertex":
                names = [p for p, _ in props]
                if not all(k in names for k in ("x", "y", "z")):
                    raise PlyError("vertex element has no x/y/z properties")
                if fmt == "ascii":
                    cols = _read_ascii_vertices(f, count, props)
                    if names[:3] == ["x", "y", "z"] and "_rows" in cols:
                        # x, y, z lead the rows: the points are a view of the parsed block (its
                        # first three columns; no copy when that is all the block holds)
                        rows = cols["_rows"]
                        pts = rows if rows.shape[1] == 3 else np.ascontiguousarray(rows[:, :3])
                        nrm = None
                        if all(k in names for k in ("nx", "ny", "nz")):
                            nrm = np.stack([cols["nx"], cols["ny"], cols["nz"]], axis=1)
                        return pts, nrm
                else:
                    if any(isinstance(t, tuple) for _, t in props):
                        raise PlyError("list properties in the vertex element are not supported")
                    dt = np.dtype([(p, endian + t) for p, t in props])
                    raw = f.read(dt.itemsize * count)
                    if len(raw) != dt.itemsize * count:
                        raise PlyError("PLY file truncated in the vertex element")
                    arr = np.frombuffer(raw, dt)
                    cols = {p: arr[p] for p in names}
                pts = np.stack([cols["x"], cols["y"], cols["z"]], axis=1).astype(np.float64)
                nrm = None
                if all(k in names for k in ("nx", "ny", "nz")):
                    nrm = np.stack([cols["nx"], cols["ny"], cols["nz"]], axis=1).astype(np.float64)
                return pts, nrm
            # an element before the vertices: skip it
            if fmt == "ascii":
                for _ in range(count):
                    f.readline()
            else:
                _skip_binary_element(f, count, props, endian)
    raise PlyError("PLY file has no vertex element")


def _text_lib():
    """libm3d's host text routines, or None when the library cannot be loaded (no build, no
    HIP/RCCL runtime): the numpy paths beside each call site give the same values."""
    try:
        from . import _lib

        return _lib.load()
    except (ImportError, OSError):
        return None


def _read_ascii_vertices(f, count, props):
    if any(isinstance(t, tuple) for _, t in props):
        raise PlyError("list properties in the vertex element are not supported")
    # fast path: the library's parser over the rest of the file (csrc/hostio.cpp), the same
    # correctly rounded doubles as numpy's; anything unusual falls back to numpy.  (A mapped
    # file instead of the read copy measured slower on the GPU box: 3.5 vs 2.0 ms at 180k rows.)
    pos = f.tell()
    rest = f.read()
    out = np.empty((count, len(props)), np.float64)
    used = C.c_size_t(0)
    lib = _text_lib()
    rc = -1 if lib is None else lib.m3d_parse_ascii_rows(
        rest, len(rest), count, len(props), out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(used))
    if rc == 0:
        f.seek(pos + used.value)
        cols = {p: out[:, k] for k, (p, _) in enumerate(props)}
        cols["_rows"] = out
        return cols
    f.seek(pos)
    rows = []
    while len(rows) < count:
        line = f.readline()
        if not line:
            raise PlyError("PLY file truncated in the vertex element")
        if line.strip():
            rows.append(line)
    if any(isinstance(t, tuple) for _, t in props):
        raise PlyError("list properties in the vertex element are not supported")
    data = np.loadtxt(rows, dtype=np.float64, ndmin=2) if count else np.zeros((0, len(props)))
    if data.shape[1] < len(props):
        raise PlyError("ASCII vertex rows shorter than the declared properties")
    return {p: data[:, k] for k, (p, _) in enumerate(props)}


def write_ply(path, points, normals=None, binary: bool = False, dtype="double"):
    """Write a PLY point cloud (x y z [nx ny nz]); ``dtype`` "double" or "float"."""
    pts = np.asarray(points, np.float64).reshape(-1, 3)
    cols = [pts]
    names = ["x", "y", "z"]
    if normals is not None:
        cols.append(np.asarray(normals, np.float64).reshape(-1, 3))
        names += ["nx", "ny", "nz"]
    data = np.concatenate(cols, axis=1)
    np_t = {"double": "f8", "float": "f4"}[dtype]
    head = ["ply", f"format {'binary_little_endian' if binary else 'ascii'} 1.0",
            f"element vertex {len(pts)}"] + [f"property {dtype} {n}" for n in names] + ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        if binary:
            f.write(np.ascontiguousarray(data.astype("<" + np_t)).tobytes())
        elif dtype == "double" and _text_lib() is None:
            # shortest round-trip text per number, as the library writes it (Python's repr)
            f.write("".join(" ".join(map(repr, row)) + "\n" for row in data.tolist()).encode("ascii"))
        elif dtype == "double":  # shortest round-trip text per number (csrc/hostio.cpp)
            data = np.ascontiguousarray(data)
            cap = 32 * data.size + 1
            buf = np.empty(cap, np.uint8)
            n = C.c_size_t(0)
            rc = _text_lib().m3d_format_ascii_rows(data.ctypes.data_as(C.POINTER(C.c_double)), len(data),
                                                   data.shape[1], buf.ctypes.data, cap, C.byref(n))
            if rc != 0:
                raise PlyError("ASCII formatting failed")
            f.write(memoryview(buf[:n.value]))
        else:
            np.savetxt(f, data.astype(np_t), fmt="%.9g")


_STL_VERTEX = re.compile(rb"vertex\s+(\S+)\s+(\S+)\s+(\S+)")


def read_stl(path):
    """Read an STL mesh → ``(vertices V×3 f64 unique, faces F×3 int64)``."""
    raw = Path(path).read_bytes()
    tri = None
    if len(raw) >= 84:
        n = int(np.frombuffer(raw[80:84], "<u4")[0])
        if len(raw) == 84 + 50 * n:  # binary: exact size match
            rec = np.frombuffer(raw[84:], np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)),
                                                    ("a", "<u2")]), count=n)
            tri = rec["v"].astype(np.float64)
    if tri is None:
        if not raw.lstrip().startswith(b"solid"):
            raise ValueError(f"{path}: neither binary nor ASCII STL")
        v = np.array(_STL_VERTEX.findall(raw), dtype=np.float64)
        if len(v) % 3:
            raise ValueError(f"{path}: ASCII STL vertex count is not a multiple of 3")
        tri = v.reshape(-1, 3, 3)
    flat = np.ascontiguousarray(tri.reshape(-1, 3), dtype=np.float64)
    # exact-equality merge in first-occurrence order: one hash pass in the library
    # (csrc/hostio.cpp m3d_merge_vertices); the numpy sort below is the same merge
    uniq = np.empty_like(flat)
    inv = np.empty(len(flat), np.int32)
    m = C.c_int64(0)
    P = C.POINTER(C.c_double)
    lib = _text_lib()
    if lib is not None and lib.m3d_merge_vertices(flat.ctypes.data_as(P), len(flat), uniq.ctypes.data_as(P),
                                      inv.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(m)) == 0:
        return uniq[: m.value].copy(), inv.astype(np.int64).reshape(-1, 3)
    return _merge_numpy(flat)


def _merge_numpy(flat):
    """Exact-equality merge on the raw bytes of each (x, y, z) (one 1-D sort of 24-byte keys);
    +0.0 and -0.0 differ in bytes, so they are canonicalised first."""
    flat = flat + 0.0
    key = flat.view(np.dtype((np.void, 24))).ravel()
    _, first, inverse = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")     # unique vertices in first-occurrence order
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    verts = flat[first[order]]
    faces = rank[inverse.reshape(-1)].reshape(-1, 3)
    return verts, faces


def convert_stl_to_ply(stl_path, ply_path):
    """convert_stl-ply.py: STL mesh vertices → ASCII PLY point cloud."""
    verts, _ = read_stl(stl_path)
    write_ply(ply_path, verts, binary=False, dtype="double")
    return len(verts)


def write_stl(path, vertices, faces, binary: bool = True):
    """Write a triangle mesh as STL (binary little-endian or ASCII), facet normals from the
    vertex winding.  Test/benchmark fixtures only: the reference reads STL, never writes it."""
    v = np.asarray(vertices, np.float64).reshape(-1, 3)
    f = np.asarray(faces, np.int64).reshape(-1, 3)
    tri = v[f].astype(np.float32).astype(np.float64)  # STL stores float32 coordinates
    n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    n = np.divide(n, ln, out=np.zeros_like(n), where=ln > 0)
    if binary:
        rec = np.zeros(len(f), np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
        rec["n"] = n
        rec["v"] = tri
        with open(path, "wb") as fh:
            fh.write(b"m3d synthetic mesh".ljust(80, b" "))
            fh.write(np.array([len(f)], "<u4").tobytes())
            fh.write(rec.tobytes())
        return
    with open(path, "w") as fh:
        fh.write("solid m3d\n")
        for k in range(len(f)):
            fh.write(f"facet normal {n[k, 0]:.9g} {n[k, 1]:.9g} {n[k, 2]:.9g}\n outer loop\n")
            for j in range(3):
                fh.write(f"  vertex {tri[k, j, 0]:.9g} {tri[k, j, 1]:.9g} {tri[k, j, 2]:.9g}\n")
            fh.write(" endloop\nendfacet\n")
        fh.write("endsolid m3d\n")
