"""ctypes wrapper of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product (smallpt-enoki-optix_amd/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of the same oracle (tools/sanitize.sh's ASan build)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")
PCG32_DEFAULT_STATE = 0x853C49E6748FEA9B


class OracleParams(ctypes.Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("spp", c_int32), ("max_depth", c_int32),
                ("look_from", c_float * 3), ("look_at", c_float * 3), ("up", c_float * 3),
                ("lens_radius", c_float), ("focal_dist", c_float), ("fov_y", c_float), ("film_size_y", c_float),
                ("rng_order", c_int32), ("rr_start_depth", c_int32), ("env", c_float * 3),
                ("rng_initstate", c_uint64)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


# oracle.c header: one unpinned arithmetic choice each, and all four at once
VARIANTS = ("sincos", "rsqrt", "fma", "tri", "all", "tex1x1", "enoki")


def _load(path=LIB_PATH):
    if not os.path.exists(path):
        build()
    lib = ctypes.CDLL(path)
    vp = c_void_p
    lib.oracle_scene_create.restype = vp
    lib.oracle_scene_create.argtypes = [vp, vp, c_int64, c_int64, vp, vp, c_int64, vp, vp, c_int32, c_int32]
    lib.oracle_scene_destroy.argtypes = [vp]
    lib.oracle_scene_set_emission.argtypes = [vp, vp, c_int32]
    lib.oracle_scene_set_texcoords.argtypes = [vp, vp, vp, c_int64]
    lib.oracle_scene_set_texture.argtypes = [vp, c_int32, vp, c_int32, c_int32]
    lib.oracle_scene_set_spheres.argtypes = [vp, vp, vp, c_int32]
    lib.oracle_scene_set_material_kinds.argtypes = [vp, vp, c_int32]
    lib.oracle_texture_eval.argtypes = [vp, c_int32, c_int32, c_float, c_float, vp]
    lib.oracle_intersect.argtypes = [vp] + [vp] * 8 + [vp, c_uint32] + [vp] * 4 + [c_int64, c_int32, c_int32]
    lib.oracle_render.restype = c_int32
    lib.oracle_render.argtypes = [vp, POINTER(OracleParams), vp, c_int32, vp, c_int32, POINTER(c_uint64)]
    lib.oracle_pcg32_seq.argtypes = [c_uint64, c_uint64, vp, c_int32]
    lib.oracle_pcg32_floats.argtypes = [c_uint64, c_uint64, vp, c_int32]
    lib.oracle_camera_ray.argtypes = [POINTER(OracleParams), c_int32, c_int32, vp, vp, vp, vp]
    lib.oracle_sincos.argtypes = [c_float, POINTER(c_float), POINTER(c_float)]
    lib.oracle_cosine_hemisphere.argtypes = [c_float, c_float, vp]
    lib.oracle_disk_from_square.argtypes = [c_float, c_float, vp]
    lib.oracle_frame_to_world.argtypes = [vp, vp, vp]
    lib.oracle_trace_sample.restype = c_int32
    lib.oracle_trace_sample.argtypes = [vp, POINTER(OracleParams), c_int32, c_int32, c_int32, vp, vp, vp, vp]
    return lib


lib = _load()
_variants = {}


def variant(name: str):
    """liboracle_alt_<name>.so: the oracle with one arithmetic choice swapped
    (VARIANTS); pass it as OracleScene(..., lib=variant(name))."""
    if name not in VARIANTS:
        raise ValueError(f"unknown oracle variant {name!r}; one of {VARIANTS}")
    if name not in _variants:
        _variants[name] = _load(os.path.join(HERE, "build", f"liboracle_alt_{name}.so"))
    return _variants[name]


def _p(a):
    return None if a is None else a.ctypes.data


def reference_params(width=512, height=512, spp=100, max_depth=2, camera=None, rng_order=0,
                     rr_start_depth=1, env=(1.0, 1.0, 1.0), rng_initstate=PCG32_DEFAULT_STATE) -> OracleParams:
    """Defaults = main.cpp:357-383."""
    p = OracleParams()
    p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
    if camera is None:
        camera = dict(look_from=(0.0, 3.03, 5.0), look_at=(0.0, 0.03, 0.0), up=(0.0, 1.0, 0.0), lens_radius=0.0,
                      focal_dist=1.0, fov_y=float(np.float32(np.float32(40.0) / np.float32(180.0))
                                                  * np.float32(np.pi)), film_size_y=0.035)
    p.look_from[:] = list(camera["look_from"])
    p.look_at[:] = list(camera["look_at"])
    p.up[:] = list(camera["up"])
    p.lens_radius = camera["lens_radius"]
    p.focal_dist = camera["focal_dist"]
    p.fov_y = camera["fov_y"]
    p.film_size_y = camera["film_size_y"]
    p.rng_order = rng_order
    p.rr_start_depth = rr_start_depth
    p.env[:] = list(env)
    p.rng_initstate = rng_initstate
    return p


class OracleScene:
    def __init__(self, mesh: dict, use_bvh: bool = True, albedo=None, emission=None, lib=None, textures=None,
                 spheres=None, sphere_mat=None, kinds=None):
        """textures: {material id: (H, W, 3) float32 image} (ImageTexture, main.cpp:34-80).
        spheres: (n, 4) float32 (cx, cy, cz, r) with sphere_mat (n,) material ids —
        smallpt's analytic spheres after the triangles; kinds: per-material
        SPT_MAT_* (0 diffuse, 1 mirror, 2 glass).  Defaults come from the mesh
        dict's "spheres" / "sphere_mat" / "kinds" keys."""
        self.lib = lib if lib is not None else globals()["lib"]
        lib = self.lib
        self.pt = np.ascontiguousarray(mesh["pos_tri"], dtype=np.int32)
        self.pos = np.ascontiguousarray(mesh["pos"], dtype=np.float32)
        self.nt = None if mesh.get("nrm_tri") is None else np.ascontiguousarray(mesh["nrm_tri"], dtype=np.int32)
        self.nrm = None if mesh.get("nrm") is None else np.ascontiguousarray(mesh["nrm"], dtype=np.float32)
        self.mat = None if mesh.get("mat_id") is None else np.ascontiguousarray(mesh["mat_id"], dtype=np.int32)
        alb = albedo if albedo is not None else mesh.get("albedo")
        self.alb = None if alb is None else np.ascontiguousarray(alb, dtype=np.float32).reshape(-1, 3)
        ntri = self.pt.size // 3
        self.h = lib.oracle_scene_create(_p(self.pt), _p(self.pos), self.pos.size // 3, ntri, _p(self.nt),
                                         _p(self.nrm), 0 if self.nrm is None else self.nrm.size // 3,
                                         _p(self.mat), _p(self.alb), 0 if self.alb is None else self.alb.shape[0],
                                         1 if use_bvh else 0)
        emi = emission if emission is not None else mesh.get("emission")
        self.emi = None if emi is None else np.ascontiguousarray(emi, dtype=np.float32).reshape(-1, 3)
        if self.emi is not None:
            lib.oracle_scene_set_emission(self.h, _p(self.emi), self.emi.shape[0])
        if mesh.get("tc_tri") is not None and mesh.get("tc") is not None:
            self.tt = np.ascontiguousarray(mesh["tc_tri"], dtype=np.int32)
            self.tc = np.ascontiguousarray(mesh["tc"], dtype=np.float32)
            lib.oracle_scene_set_texcoords(self.h, _p(self.tt), _p(self.tc), self.tc.size // 2)
        sph = spheres if spheres is not None else mesh.get("spheres")
        if sph is not None and len(sph):
            self.sph = np.ascontiguousarray(sph, dtype=np.float32).reshape(-1, 4)
            sm = sphere_mat if sphere_mat is not None else mesh.get("sphere_mat")
            self.sph_mat = (np.zeros(self.sph.shape[0], np.int32) if sm is None
                            else np.ascontiguousarray(sm, dtype=np.int32).reshape(-1))
            lib.oracle_scene_set_spheres(self.h, _p(self.sph), _p(self.sph_mat), self.sph.shape[0])
        kd = kinds if kinds is not None else mesh.get("kinds")
        if kd is not None and len(kd):
            self.kinds = np.ascontiguousarray(kd, dtype=np.uint32).reshape(-1)
            lib.oracle_scene_set_material_kinds(self.h, _p(self.kinds), self.kinds.size)
        self.tex = {}
        for mat, img in (textures or {}).items():
            img = np.ascontiguousarray(img, dtype=np.float32)
            self.tex[mat] = img
            lib.oracle_scene_set_texture(self.h, int(mat), _p(img), img.shape[1], img.shape[0])

    def __del__(self):
        if getattr(self, "h", None) and getattr(self, "lib", None) is not None:  # (module teardown at exit)
            self.lib.oracle_scene_destroy(self.h)
            self.h = None

    def intersect(self, o, d, tmin=None, tmax=None, mask=None, closest=True, nthreads=8, init=None):
        o = np.ascontiguousarray(o, dtype=np.float32).reshape(3, -1)
        d = np.ascontiguousarray(d, dtype=np.float32).reshape(3, -1)
        n = o.shape[1]
        tmin = np.full(n, 0.001, np.float32) if tmin is None else np.ascontiguousarray(tmin, dtype=np.float32)
        tmax = np.full(n, 1e20, np.float32) if tmax is None else np.ascontiguousarray(tmax, dtype=np.float32)
        if mask is None:
            mask = np.ones(1, np.uint8)
        mask = np.ascontiguousarray(mask, dtype=np.uint8).reshape(-1)
        if init is None:
            tri = np.full(n, -1, np.int32)
            t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        else:
            tri, t, u, v = (np.array(x, copy=True) for x in init)
        self.lib.oracle_intersect(self.h, _p(o[0]), _p(o[1]), _p(o[2]), _p(d[0]), _p(d[1]), _p(d[2]), _p(tmin), _p(tmax),
                             _p(mask), mask.size, _p(tri), _p(t), _p(u), _p(v), n, 1 if closest else 0, nthreads)
        return tri, t, u, v

    def render(self, params: OracleParams, rows=None, nthreads=8):
        rows = np.arange(params.height, dtype=np.int32) if rows is None else np.ascontiguousarray(rows, np.int32)
        film = np.zeros((3, rows.size, params.width), np.float32)
        casts = c_uint64(0)
        rc = self.lib.oracle_render(self.h, ctypes.byref(params), _p(rows), rows.size, _p(film), nthreads,
                               ctypes.byref(casts))
        if rc != 0:
            raise RuntimeError(f"oracle_render failed: {rc}")
        return film, int(casts.value)


def texture_eval(img, u: float, v: float) -> np.ndarray:
    """ImageTexture::eval (main.cpp:62-76) of an (H, W, 3) image at (u, v)."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros(3, np.float32)
    lib.oracle_texture_eval(_p(img), img.shape[1], img.shape[0], u, v, _p(out))
    return out


def pcg32_seq(initstate: int, initseq: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    lib.oracle_pcg32_seq(initstate, initseq, _p(out), n)
    return out


def pcg32_floats(initstate: int, initseq: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    lib.oracle_pcg32_floats(initstate, initseq, _p(out), n)
    return out


def camera_ray(params: OracleParams, px: int, py: int, xi4):
    xi = np.ascontiguousarray(xi4, np.float32)
    o, d, basis = np.zeros(3, np.float32), np.zeros(3, np.float32), np.zeros(9, np.float32)
    lib.oracle_camera_ray(ctypes.byref(params), px, py, _p(xi), _p(o), _p(d), _p(basis))
    return o, d, basis.reshape(3, 3)


def sincos(x: float):
    s, c = c_float(), c_float()
    lib.oracle_sincos(x, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def cosine_hemisphere(xi_x: float, xi_y: float) -> np.ndarray:
    out = np.zeros(3, np.float32)
    lib.oracle_cosine_hemisphere(xi_x, xi_y, _p(out))
    return out


def disk_from_square(xi_x: float, xi_y: float) -> np.ndarray:
    out = np.zeros(2, np.float32)
    lib.oracle_disk_from_square(xi_x, xi_y, _p(out))
    return out


def frame_to_world(n, local) -> np.ndarray:
    n = np.ascontiguousarray(n, np.float32)
    local = np.ascontiguousarray(local, np.float32)
    out = np.zeros(3, np.float32)
    lib.oracle_frame_to_world(_p(n), _p(local), _p(out))
    return out
