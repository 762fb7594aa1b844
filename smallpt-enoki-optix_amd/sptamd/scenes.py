"""Deterministic synthetic scenes (the reference's assets are absent).

* ``mitsuba_synth`` — stand-in for the hard-coded ``mitsuba.obj``
  (main.cpp:365): a material-preview-like object at the origin (an outer
  shell with a cut-away window, an inner sphere, an equatorial ring and a
  base) on a finite ground plane, smooth per-vertex normals with their own
  ``vn`` index stream, five ``usemtl`` materials.  Framed by the reference
  camera (main.cpp:383).  ~250k triangles at detail=1.
* ``cornell_spheres`` — smallpt's Cornell box (walls as quads, the two
  spheres and the ceiling light tessellated) for the ray-compaction stress
  configuration.
* ``smallpt_analytic`` — the same box with smallpt's own analytic spheres:
  a mirror ball, a glass ball and the big light sphere (SPT_MAT_* kinds).
* ``city_synth`` — a ~10M-triangle procedural "San-Miguel-class" scene for
  the large-scene configuration.

All generators return a mesh dict with the arrays spt_scene_create takes:
pos (V,3) f32, pos_tri (T,3) i32, nrm (N,3) f32, nrm_tri (T,3) i32,
mat_id (T,) i32 (obj material index + 1, main.cpp:185), kd (M,3) f32.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional

import numpy as np

from . import _lib


class _Builder:
    def __init__(self):
        self.pos: List[np.ndarray] = []
        self.nrm: List[np.ndarray] = []
        self.pt: List[np.ndarray] = []
        self.nt: List[np.ndarray] = []
        self.mat: List[np.ndarray] = []
        self.nv = 0
        self.nn = 0
        self.mtl_names: List[str] = []
        self.kd: List[tuple] = []
        self.ke: List[tuple] = []

    def material(self, name: str, kd, ke=(0.0, 0.0, 0.0)) -> int:
        self.mtl_names.append(name)
        self.kd.append(tuple(float(x) for x in kd))
        self.ke.append(tuple(float(x) for x in ke))
        return len(self.mtl_names)  # obj index + 1

    def add(self, pos, nrm, pt, nt, mat: int):
        pos = np.asarray(pos, np.float32).reshape(-1, 3)
        nrm = np.asarray(nrm, np.float32).reshape(-1, 3)
        pt = np.asarray(pt, np.int64).reshape(-1, 3)
        nt = np.asarray(nt, np.int64).reshape(-1, 3)
        self.pos.append(pos)
        self.nrm.append(nrm)
        self.pt.append((pt + self.nv).astype(np.int32))
        self.nt.append((nt + self.nn).astype(np.int32))
        self.mat.append(np.full(pt.shape[0], mat, np.int32))
        self.nv += pos.shape[0]
        self.nn += nrm.shape[0]

    def mesh(self) -> Dict[str, np.ndarray]:
        kd = np.array([(1.0, 1.0, 1.0)] + self.kd, np.float32)
        ke = np.array([(0.0, 0.0, 0.0)] + self.ke, np.float32)
        return dict(pos=np.concatenate(self.pos), nrm=np.concatenate(self.nrm), pos_tri=np.concatenate(self.pt),
                    nrm_tri=np.concatenate(self.nt), mat_id=np.concatenate(self.mat), kd=kd, ke=ke,
                    mtl_names=list(self.mtl_names))


def _grid_tris(nu: int, nv: int, wrap_u: bool):
    """Two triangles per (u, v) cell of a (nu [+1]) x (nv+1) vertex grid."""
    cols = nu if wrap_u else nu + 1
    u = np.arange(nu)
    v = np.arange(nv)
    uu, vv = np.meshgrid(u, v, indexing="ij")
    u1 = (uu + 1) % cols if wrap_u else uu + 1
    a = vv * cols + uu
    b = vv * cols + u1
    c = (vv + 1) * cols + u1
    d = (vv + 1) * cols + uu
    t = np.stack([np.stack([a, b, c], -1), np.stack([a, c, d], -1)], 2)
    return t.reshape(-1, 3), (uu.reshape(-1), vv.reshape(-1))


def _sphere(center, r, nlon, nlat, keep=None, flip=False):
    lon = np.arange(nlon) * (2 * math.pi / nlon)
    lat = np.linspace(-math.pi / 2, math.pi / 2, nlat + 1)
    lo, la = np.meshgrid(lon, lat, indexing="xy")
    n = np.stack([np.cos(la) * np.cos(lo), np.sin(la), np.cos(la) * np.sin(lo)], -1).reshape(-1, 3)
    p = np.asarray(center, np.float64) + r * n
    tris, (cu, cv) = _grid_tris(nlon, nlat, wrap_u=True)
    if keep is not None:
        cell_lon = (cu + 0.5) * (2 * math.pi / nlon)
        cell_lat = -math.pi / 2 + (cv.repeat(1) + 0.5) * (math.pi / nlat)
        m = keep(np.repeat(cell_lon, 2), np.repeat(cell_lat, 2))
        tris = tris[m]
    if flip:
        tris = tris[:, [0, 2, 1]]
        n = -n
    # degenerate pole triangles are kept (zero area: the watertight test rejects them)
    return p, n, tris


def _bottom_cap(center, r, theta_max, nseg, nring):
    """Spherical cap around the -y pole of a sphere (polar angle <= theta_max),
    outward normals."""
    th = np.linspace(0.0, theta_max, nring + 1)[1:]
    a = np.arange(nseg) * (2 * math.pi / nseg)
    tt, aa = np.meshgrid(th, a, indexing="ij")
    n = np.stack([np.sin(tt) * np.cos(aa), -np.cos(tt), np.sin(tt) * np.sin(aa)], -1).reshape(-1, 3)
    n = np.concatenate([[[0.0, -1.0, 0.0]], n])
    p = np.asarray(center, np.float64) + r * n
    fan = np.stack([np.zeros(nseg, np.int64), 1 + np.arange(nseg), 1 + (np.arange(nseg) + 1) % nseg], -1)
    rings, _ = _grid_tris(nseg, nring - 1, wrap_u=True)
    return p, n, np.concatenate([fan, rings + 1])


def _torus(center, R, r, nu, nv):
    u = np.arange(nu) * (2 * math.pi / nu)
    v = np.arange(nv) * (2 * math.pi / nv)
    uu, vv = np.meshgrid(u, v, indexing="xy")
    cx, cz = np.cos(uu), np.sin(uu)
    n = np.stack([np.cos(vv) * cx, np.sin(vv), np.cos(vv) * cz], -1).reshape(-1, 3)
    ring = np.stack([R * cx, np.zeros_like(cx), R * cz], -1).reshape(-1, 3)
    p = np.asarray(center, np.float64) + ring + r * n
    t, _ = _grid_tris(nu, nv, wrap_u=True)
    # wrap v as well
    t = np.where(t >= nu * nv, t - nu * nv, t)
    return p, n, t


def _cylinder(center, r, y0, y1, nseg):
    a = np.arange(nseg) * (2 * math.pi / nseg)
    ring = np.stack([np.cos(a), np.zeros_like(a), np.sin(a)], -1)
    p = np.concatenate([np.asarray(center) + r * ring + [0, y0, 0], np.asarray(center) + r * ring + [0, y1, 0]])
    n = np.concatenate([ring, ring])
    t, _ = _grid_tris(nseg, 1, wrap_u=True)
    # top cap (fan) with an up normal
    ctr = np.asarray(center, np.float64) + [0, y1, 0]
    cap_p = np.concatenate([[ctr], np.asarray(center) + r * ring + [0, y1, 0]])
    cap_t = np.stack([np.zeros(nseg, np.int64), 1 + (np.arange(nseg) + 1) % nseg, 1 + np.arange(nseg)], -1)
    return (p, n, t), (cap_p, np.array([[0.0, 1.0, 0.0]]), cap_t)


def _quad_grid(corner, eu, ev, nu, nv, normal):
    u = np.linspace(0, 1, nu + 1)
    v = np.linspace(0, 1, nv + 1)
    vv, uu = np.meshgrid(v, u, indexing="ij")
    p = np.asarray(corner, np.float64) + uu[..., None] * np.asarray(eu) + vv[..., None] * np.asarray(ev)
    t, _ = _grid_tris(nu, nv, wrap_u=False)
    return p.reshape(-1, 3), np.asarray(normal, np.float64).reshape(1, 3), t


def mitsuba_synth(detail: float = 1.0) -> Dict[str, np.ndarray]:
    """Stand-in for mitsuba.obj (main.cpp:365).  detail scales tessellation."""
    b = _Builder()
    m_ground = b.material("ground", (0.8, 0.8, 0.8))
    m_shell = b.material("shell", (0.9, 0.3, 0.2))
    m_inner = b.material("inner", (0.2, 0.2, 0.8))
    m_ring = b.material("ring", (0.9, 0.9, 0.3))
    m_base = b.material("base", (0.4, 0.4, 0.4))
    s = lambda n: max(4, int(round(n * detail)))  # noqa: E731
    # ground plane y = -1, 20 x 20 units, normal shared through one vn
    p, n, t = _quad_grid((-10.0, -1.0, 10.0), (20.0, 0.0, 0.0), (0.0, 0.0, -20.0), s(80), s(80), (0, 1, 0))
    b.add(p, n, t, np.zeros_like(t), m_ground)
    # outer shell, radius 1, with a window cut out toward the camera (+z, upper half)
    def keep(lon, lat):
        d_lon = np.abs(((lon - math.pi / 2) + math.pi) % (2 * math.pi) - math.pi)
        return ~((d_lon < math.radians(55)) & (lat > math.radians(-10)) & (lat < math.radians(60)))
    p, n, t = _sphere((0.0, 0.0, 0.0), 1.0, s(400), s(200), keep=keep)
    b.add(p, n, t, t, m_shell)
    # inner sphere
    p, n, t = _sphere((0.0, 0.0, 0.0), 0.75, s(200), s(100))
    b.add(p, n, t, t, m_inner)
    # equatorial ring
    p, n, t = _torus((0.0, 0.0, 0.0), 1.06, 0.06, s(384), s(48))
    b.add(p, n, t, t, m_ring)
    # base (cylinder + cap) between the ground and the shell
    (p, n, t), (cp, cn, ct) = _cylinder((0.0, 0.0, 0.0), 0.55, -1.0, -0.82, s(128))
    b.add(p, n, t, t, m_base)
    b.add(cp, cn, ct, np.zeros_like(ct), m_base)
    return b.mesh()


def cornell_spheres(detail: float = 1.0) -> Dict[str, np.ndarray]:
    """smallpt's Cornell box in smallpt units scaled by 1/100 (walls as quads,
    the mirror/glass spheres made diffuse, ceiling light as a small cap with
    Ke = 12 like smallpt's light sphere; the open front acts as smallpt's black
    front wall when rendered with env = 0).  Render with smallpt_materials().
    Camera: cornell_camera()."""
    b = _Builder()
    m_left = b.material("left", (0.75, 0.25, 0.25))
    m_right = b.material("right", (0.25, 0.25, 0.75))
    m_white = b.material("white", (0.75, 0.75, 0.75))
    m_sph = b.material("sphere", (0.999, 0.999, 0.999))
    m_light = b.material("light", (0.0, 0.0, 0.0), (12.0, 12.0, 12.0))
    s = lambda n: max(4, int(round(n * detail)))  # noqa: E731
    # smallpt's walls are planes (1e5 spheres) and its camera rays start 1.4
    # units in (cam.o + d * 140): the side walls, floor and ceiling run out to
    # z = 2.9 (just short of the camera) so every camera ray enters the box.
    x0, x1, y0, y1, z0, z1 = 0.01, 0.99, 0.0, 0.816, 0.0, 2.9
    walls = [
        ((x0, y0, z0), (0, 0, z1 - z0), (0, y1 - y0, 0), (1, 0, 0), m_left),      # left
        ((x1, y0, z0), (0, y1 - y0, 0), (0, 0, z1 - z0), (-1, 0, 0), m_right),    # right
        ((x0, y0, z0), (0, y1 - y0, 0), (x1 - x0, 0, 0), (0, 0, 1), m_white),     # back
        ((x0, y0, z0), (x1 - x0, 0, 0), (0, 0, z1 - z0), (0, 1, 0), m_white),     # floor
        ((x0, y1, z0), (0, 0, z1 - z0), (x1 - x0, 0, 0), (0, -1, 0), m_white),    # ceiling
    ]
    for corner, eu, ev, nrm, m in walls:
        p, n, t = _quad_grid(corner, eu, ev, s(8), s(8), nrm)
        b.add(p, n, t, np.zeros_like(t), m)
    for c in ((0.27, 0.165, 0.47), (0.73, 0.165, 0.78)):
        p, n, t = _sphere(c, 0.165, s(192), s(96))
        b.add(p, n, t, t, m_sph)
    # smallpt: Sphere(600, Vec(50, 681.6 - .27, 81.6), Vec(12, 12, 12)) — only
    # the part below the ceiling (a disk of radius ~0.18) is visible.
    p, n, t = _bottom_cap((0.5, 6.816 - 0.0027, 0.816), 6.0, math.radians(2.5), s(64), s(8))
    b.add(p, n, t, t, m_light)
    return b.mesh()


def smallpt_analytic(detail: float = 1.0) -> Dict[str, np.ndarray]:
    """smallpt's scene as smallpt has it (scaled by 1/100): the Cornell walls as
    triangle quads (cornell_spheres' walls), and the mirror ball, the glass
    ball and the 600-radius light as analytic spheres (spt_scene_set_spheres)
    with SPT_MAT_MIRROR / SPT_MAT_GLASS / diffuse-emitting materials
    (spt_scene_set_material_kinds).  Render with smallpt_materials(), env = 0,
    cornell_camera().  Extra keys: spheres (3, 4), sphere_mat (3,), kinds."""
    b = _Builder()
    m_left = b.material("left", (0.75, 0.25, 0.25))
    m_right = b.material("right", (0.25, 0.25, 0.75))
    m_white = b.material("white", (0.75, 0.75, 0.75))
    m_mirror = b.material("mirror", (0.999, 0.999, 0.999))
    m_glass = b.material("glass", (0.999, 0.999, 0.999))
    m_light = b.material("light", (0.0, 0.0, 0.0), (12.0, 12.0, 12.0))
    s = lambda n: max(1, int(round(n * detail)))  # noqa: E731
    x0, x1, y0, y1, z0, z1 = 0.01, 0.99, 0.0, 0.816, 0.0, 2.9
    walls = [
        ((x0, y0, z0), (0, 0, z1 - z0), (0, y1 - y0, 0), (1, 0, 0), m_left),
        ((x1, y0, z0), (0, y1 - y0, 0), (0, 0, z1 - z0), (-1, 0, 0), m_right),
        ((x0, y0, z0), (0, y1 - y0, 0), (x1 - x0, 0, 0), (0, 0, 1), m_white),
        ((x0, y0, z0), (x1 - x0, 0, 0), (0, 0, z1 - z0), (0, 1, 0), m_white),
        ((x0, y1, z0), (0, 0, z1 - z0), (x1 - x0, 0, 0), (0, -1, 0), m_white),
    ]
    for corner, eu, ev, nrm, m in walls:
        p, n, t = _quad_grid(corner, eu, ev, s(8), s(8), nrm)
        b.add(p, n, t, np.zeros_like(t), m)
    mesh = b.mesh()
    # smallpt: Sphere(16.5, (27, 16.5, 47), SPEC), Sphere(16.5, (73, 16.5, 78), REFR),
    # Sphere(600, (50, 681.6 - .27, 81.6), e = 12) — in the same 1/100 units
    mesh["spheres"] = np.array([[0.27, 0.165, 0.47, 0.165], [0.73, 0.165, 0.78, 0.165],
                                [0.5, 6.816 - 0.0027, 0.816, 6.0]], np.float32)
    mesh["sphere_mat"] = np.array([m_mirror, m_glass, m_light], np.int32)
    kinds = np.zeros(mesh["kd"].shape[0], np.uint32)
    kinds[m_mirror] = _lib.SPT_MAT_MIRROR
    kinds[m_glass] = _lib.SPT_MAT_GLASS
    mesh["kinds"] = kinds
    return mesh


def smallpt_materials(mesh: Dict[str, np.ndarray]):
    """(albedo, emission) tables for smallpt-style shading: Kd as albedo and Ke
    as emission (the reference itself renders albedo 1, no emitters)."""
    ke = mesh.get("ke")
    return mesh["kd"], (ke if ke is not None else np.zeros_like(mesh["kd"]))


def cornell_camera() -> dict:
    """smallpt: Ray cam(Vec(50,52,295.6), Vec(0,-0.042612,-1).norm()), 0.5135 fov scale."""
    from_ = np.array([0.5, 0.52, 2.956])
    d = np.array([0.0, -0.042612, -1.0])
    d = d / np.linalg.norm(d)
    fov = 2.0 * math.atan(0.5135)
    return dict(look_from=tuple(from_), look_at=tuple(from_ + d), up=(0.0, 1.0, 0.0), lens_radius=0.0,
                focal_dist=1.0, fov_y=float(np.float32(fov)), film_size_y=0.035)


def city_synth(target_tris: int = 10_000_000, seed: int = 7) -> Dict[str, np.ndarray]:
    """~target_tris procedural 'San-Miguel-class' scene: a courtyard of
    tessellated boxes, columns and foliage spheres on a ground plane."""
    rng = np.random.default_rng(seed)
    b = _Builder()
    m_ground = b.material("ground", (0.7, 0.7, 0.7))
    m_wall = b.material("wall", (0.8, 0.7, 0.6))
    m_leaf = b.material("leaf", (0.2, 0.6, 0.2))
    p, n, t = _quad_grid((-12.0, -1.0, 12.0), (24.0, 0.0, 0.0), (0.0, 0.0, -24.0), 200, 200, (0, 1, 0))
    b.add(p, n, t, np.zeros_like(t), m_ground)
    total = t.shape[0]
    # foliage spheres carry most of the triangles
    per_sphere = 2 * 64 * 32
    nsph = max(1, (target_tris - total) // per_sphere)
    centers = np.stack([rng.uniform(-10, 10, nsph), rng.uniform(-0.8, 4.0, nsph), rng.uniform(-10, 6, nsph)], -1)
    radii = rng.uniform(0.05, 0.35, nsph)
    lon = np.arange(64) * (2 * math.pi / 64)
    lat = np.linspace(-math.pi / 2, math.pi / 2, 33)
    lo, la = np.meshgrid(lon, lat, indexing="xy")
    unit = np.stack([np.cos(la) * np.cos(lo), np.sin(la), np.cos(la) * np.sin(lo)], -1).reshape(-1, 3)
    tris, _ = _grid_tris(64, 32, wrap_u=True)
    nv = unit.shape[0]
    pos = (centers[:, None, :] + radii[:, None, None] * unit[None]).reshape(-1, 3)
    nrm = np.tile(unit, (nsph, 1))
    pt = (tris[None] + (np.arange(nsph) * nv)[:, None, None]).reshape(-1, 3)
    b.add(pos, nrm, pt, pt, m_leaf)
    # a ring of columns (low tessellation)
    for k in range(24):
        a = 2 * math.pi * k / 24
        (cp, cn, ct), _ = _cylinder((9 * math.cos(a), 0.0, 9 * math.sin(a)), 0.3, -1.0, 5.0, 32)
        b.add(cp, cn, ct, ct, m_wall)
    return b.mesh()


def city_camera() -> dict:
    """A courtyard view for city_synth (San Miguel comes with its own pbrt camera)."""
    return dict(look_from=(-6.0, 2.5, 8.0), look_at=(2.0, 0.5, -4.0), up=(0.0, 1.0, 0.0), lens_radius=0.0,
                focal_dist=1.0, fov_y=0.9, film_size_y=0.035)


def with_planar_uv(mesh: Dict[str, np.ndarray], scale: float = 0.3, offset=(0.5, 0.5)) -> Dict[str, np.ndarray]:
    """A copy of mesh with per-vertex texcoords from a planar projection
    (u = x * scale + offset, v = z * scale + offset), tc_tri = pos_tri — for
    the textured-material tests (the generated stand-ins carry no vt)."""
    m = dict(mesh)
    p = np.asarray(mesh["pos"], np.float32)
    m["tc"] = np.stack([p[:, 0] * np.float32(scale) + np.float32(offset[0]),
                        p[:, 2] * np.float32(scale) + np.float32(offset[1])], 1).astype(np.float32)
    m["tc_tri"] = np.asarray(mesh["pos_tri"], np.int32).copy()
    return m


def checker(w: int, h: int, a=(0.9, 0.8, 0.2), b=(0.2, 0.4, 0.9), cell: int = 1) -> np.ndarray:
    """(h, w, 3) float32 checkerboard image."""
    y, x = np.mgrid[0:h, 0:w]
    sel = ((x // cell + y // cell) % 2 == 0)[..., None]
    return np.where(sel, np.float32(a), np.float32(b)).astype(np.float32)


def write_obj(path: str, mesh: Dict[str, np.ndarray], mtl: str = None) -> None:
    """Write mesh as OBJ (+ .mtl) using v / vn / f v//vn and usemtl groups."""
    mtl = mtl or os.path.splitext(path)[0] + ".mtl"
    names = mesh.get("mtl_names") or [f"m{i}" for i in range(len(mesh["kd"]) - 1)]
    with open(mtl, "w") as f:
        for i, nm in enumerate(names):
            kd = mesh["kd"][i + 1]
            f.write(f"newmtl {nm}\nKd {kd[0]:.6g} {kd[1]:.6g} {kd[2]:.6g}\n")
            ke = mesh["ke"][i + 1] if mesh.get("ke") is not None else (0.0, 0.0, 0.0)
            if any(float(x) != 0.0 for x in ke):
                f.write(f"Ke {ke[0]:.6g} {ke[1]:.6g} {ke[2]:.6g}\n")
            f.write("\n")
    pos, nrm = mesh["pos"], mesh["nrm"]
    pt, nt, mat = mesh["pos_tri"], mesh["nrm_tri"], mesh["mat_id"]
    with open(path, "w") as f:
        f.write(f"# generated by sptamd.scenes\nmtllib {os.path.basename(mtl)}\n")
        f.write("".join("v %.9g %.9g %.9g\n" % tuple(r) for r in pos.tolist()))
        f.write("".join("vn %.9g %.9g %.9g\n" % tuple(r) for r in nrm.tolist()))
        # faces grouped by runs of equal material
        change = np.flatnonzero(np.diff(mat)) + 1
        starts = np.concatenate([[0], change])
        ends = np.concatenate([change, [len(mat)]])
        pt1 = (pt + 1).tolist()
        nt1 = (nt + 1).tolist()
        for s, e in zip(starts.tolist(), ends.tolist()):
            m = int(mat[s])
            f.write(f"usemtl {names[m - 1]}\n" if m > 0 else "usemtl __none__\n")
            f.write("".join("f %d//%d %d//%d %d//%d\n" % (a[0], b[0], a[1], b[1], a[2], b[2])
                            for a, b in zip(pt1[s:e], nt1[s:e])))


def _np_copy(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype).copy()


def _mesh_from_c(m) -> Dict[str, np.ndarray]:
    out = dict(
        pos_tri=_np_copy(m.pos_tri, 3 * m.ntri, np.int32).reshape(-1, 3),
        pos=_np_copy(m.pos, 3 * m.nvert, np.float32).reshape(-1, 3),
        nrm_tri=_np_copy(m.nrm_tri, 3 * m.ntri, np.int32).reshape(-1, 3),
        nrm=_np_copy(m.nrm, 3 * m.nnrm, np.float32).reshape(-1, 3),
        tc_tri=_np_copy(m.tc_tri, 3 * m.ntri, np.int32).reshape(-1, 3),
        tc=_np_copy(m.tc, 2 * m.ntc, np.float32).reshape(-1, 2),
        mat_id=_np_copy(m.mat_id, m.ntri, np.int32),
        kd=_np_copy(m.kd, 3 * m.nmat, np.float32).reshape(-1, 3),
        ke=_np_copy(m.ke, 3 * m.nmat, np.float32).reshape(-1, 3),
    )
    if out["tc"].size == 0:
        out["tc"] = None
        out["tc_tri"] = None
    return out


def load_obj(path: str) -> Dict[str, np.ndarray]:
    """load_meshes (main.cpp:141-251) through the C ABI's OBJ reader."""
    m = _lib.Mesh()
    _lib.check(_lib.lib.spt_obj_load(path.encode(), ctypes.byref(m)), f"spt_obj_load({path})")
    try:
        return _mesh_from_c(m)
    finally:
        _lib.lib.spt_mesh_free(ctypes.byref(m))


def load_pbrt(path: str):
    """pbrt-v3 scene through the C ABI's reader (spt_pbrt_load).  Returns
    (mesh dict as load_obj's, info dict: camera (make_params form) or None,
    xres, yres, env or None, shapes, shapes_skipped, instances)."""
    m = _lib.Mesh()
    info = _lib.PbrtInfo()
    _lib.check(_lib.lib.spt_pbrt_load(path.encode(), ctypes.byref(m), ctypes.byref(info)), f"spt_pbrt_load({path})")
    try:
        mesh = _mesh_from_c(m)
    finally:
        _lib.lib.spt_mesh_free(ctypes.byref(m))
    return mesh, pbrt_info_from_c(info)


def pbrt_info_from_c(info: "_lib.PbrtInfo") -> dict:
    """spt_pbrt_info -> load_pbrt's info dict."""
    c = info.camera
    cam = dict(look_from=tuple(c.look_from), look_at=tuple(c.look_at), up=tuple(c.up), lens_radius=c.lens_radius,
               focal_dist=c.focal_dist, fov_y=c.fov_y, film_size_y=c.film_size_y) if info.has_camera else None
    return dict(camera=cam, fov_deg=info.fov_deg, xres=info.xres, yres=info.yres,
                env=tuple(info.env) if info.has_env else None, shapes=info.shapes,
                shapes_skipped=info.shapes_skipped, instances=info.instances)


def pbrt_info_to_c(d: dict) -> "_lib.PbrtInfo":
    """load_pbrt's info dict -> spt_pbrt_info (the scene cache's extra bytes,
    shared with spt_render_cli --save-cache)."""
    info = _lib.PbrtInfo()
    cam = d.get("camera")
    if cam is not None:
        info.has_camera = 1
        for k in ("look_from", "look_at", "up"):
            getattr(info.camera, k)[:] = [float(x) for x in cam[k]]
        for k in ("lens_radius", "focal_dist", "fov_y", "film_size_y"):
            setattr(info.camera, k, cam[k])
    info.fov_deg, info.xres, info.yres = d.get("fov_deg", 90.0), d.get("xres", 640), d.get("yres", 480)
    if d.get("env") is not None:
        info.has_env = 1
        info.env[:] = [float(x) for x in d["env"]]
    info.shapes, info.shapes_skipped, info.instances = d.get("shapes", 0), d.get("shapes_skipped", 0), \
        d.get("instances", 0)
    return info


def _write_ply(path: str, pos: np.ndarray, nrm: Optional[np.ndarray], tris: np.ndarray, binary: bool = True) -> None:
    """Triangle PLY: float x y z (nx ny nz), uchar/int vertex_indices lists."""
    nv, nt = len(pos), len(tris)
    props = ["x", "y", "z"] + (["nx", "ny", "nz"] if nrm is not None else [])
    hdr = ["ply", "format binary_little_endian 1.0" if binary else "format ascii 1.0",
           f"element vertex {nv}"] + [f"property float {p}" for p in props] + [
           f"element face {nt}", "property list uchar int vertex_indices", "end_header"]
    verts = np.ascontiguousarray(np.hstack([pos, nrm]) if nrm is not None else pos, dtype="<f4")
    with open(path, "wb") as f:
        f.write(("\n".join(hdr) + "\n").encode())
        if binary:
            f.write(verts.tobytes())
            face = np.zeros(nt, dtype=[("n", "u1"), ("i", "<i4", (3,))])
            face["n"] = 3
            face["i"] = tris
            f.write(face.tobytes())
        else:
            for v in verts:
                f.write((" ".join(repr(float(x)) for x in v) + "\n").encode())
            for t in tris:
                f.write(f"3 {t[0]} {t[1]} {t[2]}\n".encode())


def write_pbrt(path: str, mesh: Dict[str, np.ndarray], camera: Optional[dict] = None, width: int = 1024,
               height: int = 1024, binary: bool = True) -> None:
    """Write mesh as a pbrt-v3 scene: one "plymesh" per run of equal material
    (triangle order kept), named matte materials with the mesh's Kd, diffuse
    area lights for its Ke, LookAt + perspective camera."""
    import math
    base = os.path.splitext(path)[0]
    stem = os.path.basename(base)
    pos = np.asarray(mesh["pos"], np.float32).reshape(-1, 3)
    pt = np.asarray(mesh["pos_tri"], np.int64).reshape(-1, 3)
    nrm = mesh.get("nrm")
    nt = mesh.get("nrm_tri")
    has_n = nrm is not None and nt is not None and len(nrm) > 0
    if has_n:
        nrm = np.asarray(nrm, np.float32).reshape(-1, 3)
        nt = np.asarray(nt, np.int64).reshape(-1, 3)
        has_n = bool(np.all(nt >= 0))
    mat = np.asarray(mesh.get("mat_id", np.zeros(len(pt), np.int32)), np.int64)
    kd = np.asarray(mesh.get("kd", np.ones((1, 3))), np.float32).reshape(-1, 3)
    ke = mesh.get("ke")
    ke = np.zeros_like(kd) if ke is None else np.asarray(ke, np.float32).reshape(-1, 3)
    cam = camera or dict(look_from=(0.0, 3.03, 5.0), look_at=(0.0, 0.03, 0.0), up=(0.0, 1.0, 0.0),
                         fov_y=40.0 / 180.0 * math.pi)
    fov = float(cam["fov_y"]) * 180.0 / math.pi
    if width < height:  # pbrt's fov spans the shorter axis
        fov = 2.0 * math.degrees(math.atan(math.tan(0.5 * float(cam["fov_y"])) * width / height))
    lines = ["# written by sptamd.scenes.write_pbrt",
             "LookAt " + " ".join(f"{float(x)!r}" for x in (*cam["look_from"], *cam["look_at"], *cam["up"])),
             f'Camera "perspective" "float fov" [ {fov!r} ]',
             f'Film "image" "integer xresolution" [ {width} ] "integer yresolution" [ {height} ]',
             "WorldBegin"]
    for i in range(1, len(kd)):
        lines.append(f'MakeNamedMaterial "m{i}" "string type" "matte" '
                     f'"rgb Kd" [ {float(kd[i][0])!r} {float(kd[i][1])!r} {float(kd[i][2])!r} ]')
    change = np.flatnonzero(mat[1:] != mat[:-1]) + 1
    starts = np.concatenate([[0], change]).astype(np.int64)
    ends = np.concatenate([change, [len(mat)]]).astype(np.int64)
    for k, (s, e) in enumerate(zip(starts.tolist(), ends.tolist())):
        m = int(mat[s]) if len(mat) else 0
        # per-vertex (position, normal) pairs of this run
        if has_n:  # unique (position, normal) pairs, as one int64 key each
            key = pt[s:e].reshape(-1) * np.int64(len(nrm)) + nt[s:e].reshape(-1)
            uniq, inv = np.unique(key, return_inverse=True)
            vp, vn = pos[uniq // len(nrm)], nrm[uniq % len(nrm)]
        else:
            uniq, inv = np.unique(pt[s:e].reshape(-1), return_inverse=True)
            vp, vn = pos[uniq], None
        ply = f"{stem}_{k}.ply"
        _write_ply(os.path.join(os.path.dirname(path) or ".", ply), vp, vn, inv.reshape(-1, 3).astype(np.int32),
                   binary=binary)
        lines.append("AttributeBegin")
        if m > 0:
            lines.append(f'  NamedMaterial "m{m}"')
            if m < len(ke) and np.any(ke[m] != 0):
                lines.append(f'  AreaLightSource "diffuse" "rgb L" '
                             f'[ {float(ke[m][0])!r} {float(ke[m][1])!r} {float(ke[m][2])!r} ]')
        lines.append(f'  Shape "plymesh" "string filename" "{ply}"')
        lines.append("AttributeEnd")
    lines.append("WorldEnd")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def scene_pbrt(name: str, detail: float = 1.0) -> str:
    """Path of a generated pbrt-v3 scene (+ PLY files), generated once into
    build/scenes/.  city_synth: detail x 10M triangles, 1920 x 1080 film."""
    d = os.path.join(SCENE_DIR, f"{name}_d{detail:g}_pbrt")
    path = os.path.join(d, f"{name}.pbrt")
    if not os.path.exists(path):
        tmp = d + f".tmp{os.getpid()}"
        os.makedirs(tmp, exist_ok=True)
        out = os.path.join(tmp, f"{name}.pbrt")
        if name == "city_synth":
            write_pbrt(out, city_synth(int(10_000_000 * detail)), camera=city_camera(), width=1920, height=1080)
        else:
            gen = {"mitsuba_synth": mitsuba_synth, "cornell_spheres": cornell_spheres}[name]
            write_pbrt(out, gen(detail), camera=cornell_camera() if name == "cornell_spheres" else None)
        try:
            os.replace(tmp, d)
        except OSError:  # another process won
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)
    return path


SCENE_DIR = os.path.join(_lib.REPO_ROOT, "build", "scenes")


def scene_obj(name: str, detail: float = 1.0) -> str:
    """Path of a generated OBJ, generating it once into build/scenes/."""
    os.makedirs(SCENE_DIR, exist_ok=True)
    path = os.path.join(SCENE_DIR, f"{name}_d{detail:g}.obj")
    if not os.path.exists(path):
        gen = {"mitsuba_synth": mitsuba_synth, "cornell_spheres": cornell_spheres}[name]
        tmp = path + f".tmp{os.getpid()}"
        write_obj(tmp, gen(detail), mtl=os.path.splitext(path)[0] + ".mtl")
        os.replace(tmp, path)
    return path
