"""Synthetic point-cloud pairs with a known rigid transform.

The reference ships no data (`3d_data/.gitignore:1-2`), so every config runs on synthetic clouds:

* points sampled on a closed, asymmetric, star-shaped surface of extent ~10 units (so the
  reference's voxel size 0.3, RANSAC threshold 1.5·v and ICP radius 0.4·v are meaningful);
* analytic outward normals (the reference estimates them with Open3D, `ply.py:123-135`);
* a random rigid pose drawn with the recipe of `_visualize_matcher.py:294-323`
  (angles U(±π/6) per axis composed ``Rz @ Ry @ Rx``, translation U(±0.1), rotation about the
  cloud centre);
* Gaussian point noise N(0, 0.05²) as `ply.py:59-62` adds to ``pcd_down``;
* outlier correspondences injected with the recipe of `ransac.py:88-99`.

Everything is seeded through ``numpy.random.default_rng`` so fixtures are reproducible.
"""

from __future__ import annotations

import numpy as np

R0 = 5.0          # mean radius -> extent ~10 units
ALPHA = 0.3       # bump amplitude


def _bump(u: np.ndarray):
    """g(u) and its gradient (treating g as a function on R^3 evaluated at unit u)."""
    ux, uy, uz = u[:, 0], u[:, 1], u[:, 2]
    s = 3.0 * ux + 2.0 * uy - uz
    g = 0.3 * ux * uy + 0.2 * uz ** 3 + 0.15 * np.sin(s)
    c = 0.15 * np.cos(s)
    grad = np.stack([0.3 * uy + 3.0 * c, 0.3 * ux + 2.0 * c, 0.6 * uz ** 2 - c], axis=1)
    return g, grad


def surface_points(n: int, seed: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Sample ``n`` points (N×3 float64) and unit outward normals on the synthetic surface.

    Surface: |x| = r(x/|x|),  r(u) = R0 (1 + ALPHA g(u)).  Implicit F(x) = |x| - r(x/|x|),
    grad F = u - (R0 ALPHA / |x|) (I - u u^T) grad g(u).
    """
    rng = np.random.default_rng(seed)
    u = rng.standard_normal((n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    g, dg = _bump(u)
    r = R0 * (1.0 + ALPHA * g)
    pts = u * r[:, None]
    tang = dg - np.sum(dg * u, axis=1, keepdims=True) * u
    nrm = u - (R0 * ALPHA / r)[:, None] * tang
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    return pts, nrm


def euler_zyx(angles) -> np.ndarray:
    """R = Rz(a2) @ Ry(a1) @ Rx(a0) — the composition of `_visualize_matcher.py:305-315`."""
    a0, a1, a2 = angles
    rx = np.array([[1, 0, 0], [0, np.cos(a0), -np.sin(a0)], [0, np.sin(a0), np.cos(a0)]])
    ry = np.array([[np.cos(a1), 0, np.sin(a1)], [0, 1, 0], [-np.sin(a1), 0, np.cos(a1)]])
    rz = np.array([[np.cos(a2), -np.sin(a2), 0], [np.sin(a2), np.cos(a2), 0], [0, 0, 1]])
    return rz @ ry @ rx


def random_rigid(seed: int, center=None, rot_range=np.pi / 6, trans_range=0.1) -> np.ndarray:
    """Random 4×4 rigid transform rotating about ``center`` (`_visualize_matcher.py:294-323`)."""
    rng = np.random.default_rng(seed)
    rot = euler_zyx(rng.uniform(-rot_range, rot_range, 3))
    trans = rng.uniform(-trans_range, trans_range, 3)
    c = np.zeros(3) if center is None else np.asarray(center, dtype=np.float64)
    T = np.eye(4)
    T[:3, :3] = rot
    T[:3, 3] = -rot @ c + c + trans
    return T


def apply(T: np.ndarray, pts: np.ndarray) -> np.ndarray:
    return pts @ T[:3, :3].T + T[:3, 3]


def inject_outliers(corr: np.ndarray, n_src: int, n_tgt: int, noise_ratio: float,
                    rng: np.random.Generator) -> np.ndarray:
    """Outlier injection recipe of `ransac.py:88-99` on a seeded Generator."""
    corr = np.asarray(corr, dtype=np.int32).reshape(-1, 2)
    n_noise = int(len(corr) * noise_ratio)
    if noise_ratio <= 0 or n_noise <= 0:
        return corr
    noise = np.stack((rng.integers(0, n_src, n_noise), rng.integers(0, n_tgt, n_noise)), axis=1)
    out = np.vstack((corr, noise)).astype(np.int32)
    rng.shuffle(out)
    return out


def ransac_pair(n: int, seed: int = 0, noise_sigma: float = 0.05, noise_ratio: float = 0.0):
    """RANSAC workload (cfg0/cfg2): source cloud, target = T·source + noise, identity pairs.

    Returns ``(src, tgt, corr, T_true)``; ``corr`` is int32 Nc×2 with Nc = n·(1+noise_ratio).
    """
    src, _ = surface_points(n, seed)
    T = random_rigid(seed + 1, center=src.mean(axis=0))
    rng = np.random.default_rng(seed + 2)
    tgt = apply(T, src) + noise_sigma * rng.standard_normal(src.shape)
    src = src + noise_sigma * rng.standard_normal(src.shape)
    corr = np.stack([np.arange(n), np.arange(n)], axis=1).astype(np.int32)
    corr = inject_outliers(corr, n, n, noise_ratio, rng)
    return src, tgt, corr, T


def icp_pair(ns: int, nt: int | None = None, seed: int = 0):
    """ICP workload (cfg1/cfg3): two independent samplings of the same surface.

    target = surface sample (with analytic normals); source = another sample mapped by T_true^-1,
    so the registration source→target is T_true.  Returns ``(src, tgt, tgt_normals, T_true)``.
    """
    nt = ns if nt is None else nt
    tgt, tgt_n = surface_points(nt, seed)
    src_world, _ = surface_points(ns, seed + 100)
    T = random_rigid(seed + 1, center=tgt.mean(axis=0), rot_range=np.pi / 60, trans_range=0.05)
    Tinv = np.linalg.inv(T)
    src = apply(Tinv, src_world)
    return src, tgt, tgt_n, T


_CUSPS = (((0.3, 0.8, 0.5), 0.2, 0.05), ((-0.7, 0.2, 0.6), 0.12, 0.03),
          ((0.5, -0.6, 0.6), 0.15, 0.04), ((0.1, 0.1, -1.0), 0.08, 0.08))


def surface_mesh(n_lat: int, n_lon: int, seed: int = 0):
    """Triangle mesh of the synthetic surface (a scan stand-in for cfg4's STL input).

    A UV-sphere tessellation (``n_lat`` rings × ``n_lon`` segments plus the two poles) whose
    directions are first rotated by a seeded random rotation — two seeds give two different
    tessellations (vertex sets) of the same surface, like two scans — then mapped onto
    |x| = r(x/|x|) with four extra cusps (Gaussian lobes of height 0.08–0.2·R0 in fixed
    directions) so that no rotation maps the shape close onto itself — the tooth-like scan the
    reference's cfg4 registers; ``surface_points`` stays cusp-free (the goldens use it).
    Returns ``(vertices V×3 f64, faces F×3 int64)``.
    """
    rng = np.random.default_rng(seed)
    q = rng.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    Rg = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    th = np.pi * (np.arange(1, n_lat + 1) / (n_lat + 1))
    ph = 2.0 * np.pi * np.arange(n_lon) / n_lon
    st, ct = np.sin(th)[:, None], np.cos(th)[:, None]
    ring = np.stack([st * np.cos(ph)[None, :], st * np.sin(ph)[None, :], np.broadcast_to(ct, (n_lat, n_lon))],
                    axis=2).reshape(-1, 3)
    u = np.vstack([[0.0, 0.0, 1.0], ring, [0.0, 0.0, -1.0]]) @ Rg.T
    g, _ = _bump(u)
    cusp = np.zeros(len(u))
    for d, hgt, w in _CUSPS:
        d = np.asarray(d, np.float64) / np.linalg.norm(d)
        cusp += hgt * np.exp(-np.sum((u - d) ** 2, axis=1) / w)
    verts = u * (R0 * (1.0 + ALPHA * g + cusp))[:, None]
    idx = 1 + np.arange(n_lat * n_lon).reshape(n_lat, n_lon)
    nxt = np.roll(idx, -1, axis=1)
    faces = [np.stack([np.zeros(n_lon, np.int64), idx[0], nxt[0]], axis=1)]
    a, b, c, d = idx[:-1], nxt[:-1], idx[1:], nxt[1:]
    faces.append(np.stack([a, c, b], axis=2).reshape(-1, 3))
    faces.append(np.stack([b, c, d], axis=2).reshape(-1, 3))
    south = len(verts) - 1
    faces.append(np.stack([np.full(n_lon, south, np.int64), nxt[-1], idx[-1]], axis=1))
    return verts, np.vstack(faces).astype(np.int64)
