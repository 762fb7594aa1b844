"""Python host mirror of the reference's hot-path interface, over libspt.so.

    HipBackend   <-> OptixBackend        (src/accel/optix_backend.h:164-504)
    Ray3         <-> Ray<Real3C>         (src/ray.h:5-36)
    TriangleHitInfo <-> TriangleHitInfo  (src/accel/optix_backend.h:99-134)
    Scene        <-> Scene               (src/main.cpp:286-352)
    Scene.render <-> main() render loop  (src/main.cpp:354-429)

Device memory and streams come from torch (HIP tensors); every computation
runs in the HIP kernels of libspt.so.  Errors raise SptError, as the
reference's OPTIX_CHECK / CUDA_CHECK raise std::runtime_error.
"""
from __future__ import annotations

import atexit
import ctypes
import math
import os
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import (Config, Hits, HitInfo, Rays, RenderParams, RenderStats, SceneStats, check, config_from_env,
                   env_snapshot, lib)

RAY_TMIN = 0.001  # ray.h:16
RAY_TMAX = 1e20


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> Optional[int]:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream or None


def queue_stream(device: Optional[int] = None) -> torch.cuda.ExternalStream:
    """A caller stream with a hardware queue of its own, for queued renders.

    HIP maps ordinary streams onto the process's GPU_MAX_HW_QUEUES hardware
    queues, and a stream's wait on an event blocks the whole queue it sits on.
    spt_render_async ends by making the caller stream wait for the render, so
    when the two streams renders alternate on share a queue, the next render's
    start (an event recorded on the other stream) waits behind that wait and
    the renders stop overlapping: one run in ten of a tile was ~30 % slow
    (profiles/r05_exp/caller_queues/).  A stream created with a
    CU mask gets a dedicated queue (the library's own sub-wavefront streams are
    made the same way); this one has every CU in its mask.  It is a blocking
    stream, so work on the legacy null stream waits for it.  Made through the
    HIP runtime (torch offers no CU-mask stream), wrapped for torch; it is
    destroyed at interpreter exit, after a device synchronisation, before the
    runtime's own teardown."""
    dev = torch.cuda.current_device() if device is None else device
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    hip = _hip_runtime()
    handle = ctypes.c_void_p()
    with torch.cuda.device(dev):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(handle), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise _lib.SptError("hipExtStreamCreateWithCUMask", rc, "no stream with a dedicated hardware queue")
    if not _QUEUE_STREAMS:
        atexit.register(_destroy_queue_streams)
    _QUEUE_STREAMS.append((dev, handle.value))
    return torch.cuda.ExternalStream(handle.value, device=torch.device("cuda", dev))


_QUEUE_STREAMS = []


def _hip_runtime():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return hip


def _destroy_queue_streams():
    hip = _hip_runtime()
    for dev, h in _QUEUE_STREAMS:
        with torch.cuda.device(dev):
            hip.hipStreamSynchronize(h)
            hip.hipStreamDestroy(h)
    _QUEUE_STREAMS.clear()


def _dev_f32(x, device) -> torch.Tensor:
    t = torch.as_tensor(x, dtype=torch.float32)
    return t.to(device).contiguous()


def _host_ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


@dataclass
class Ray3:
    """SoA rays (ray.h:28-31).  origin/dir: (3, N) float32 device tensors."""

    origin: torch.Tensor
    dir: torch.Tensor
    tmin: torch.Tensor
    tmax: torch.Tensor

    @staticmethod
    def make(origin, direction, tmin: float = RAY_TMIN, tmax: float = RAY_TMAX, device="cuda") -> "Ray3":
        o = _dev_f32(origin, device)
        d = _dev_f32(direction, device)
        n = o.shape[1]
        return Ray3(o, d, torch.full((n,), tmin, dtype=torch.float32, device=o.device),
                    torch.full((n,), tmax, dtype=torch.float32, device=o.device))

    def __len__(self) -> int:
        return int(self.origin.shape[1])

    def c_struct(self) -> Rays:
        return Rays(self.origin[0].data_ptr(), self.origin[1].data_ptr(), self.origin[2].data_ptr(),
                    self.dir[0].data_ptr(), self.dir[1].data_ptr(), self.dir[2].data_ptr(),
                    self.tmin.data_ptr(), self.tmax.data_ptr())


@dataclass
class TriangleHitInfo:
    """optix_backend.h:99-134; device tensors, planar (3, N) vectors."""

    tri_id: torch.Tensor
    t: torch.Tensor
    barycentric: torch.Tensor
    position: torch.Tensor
    geometry_normal: torch.Tensor
    shading_normal: torch.Tensor
    texcoord: torch.Tensor
    material_id: torch.Tensor


class HipBackend:
    """OptixBackend replacement: init / set_triangles_soup / intersect."""

    def __init__(self, config: Optional[Config] = None):
        self._scene = ctypes.c_void_p()
        self.device = None
        self.stats: dict = {}
        # spt_config: explicit base (default: the library's), with the SPT_*
        # environment variables applied over it before every call that reads it
        self.base_config = config
        self._applied = None
        self._env_key = None

    def __del__(self):
        if getattr(self, "_scene", None) and self._scene.value:
            lib.spt_scene_destroy(self._scene)
            self._scene = ctypes.c_void_p()

    # optix_backend.h:178-186
    def init(self, device: int = 0) -> None:
        check(lib.spt_init(device), "spt_init")
        self.device = torch.device("cuda", device)

    # optix_backend.h:283-364 (arrays are host arrays here; the BVH is built on the host)
    def set_triangles_soup(self, position_triplets, positions, shading_normal_triplets=None, shading_normals=None,
                           texcoord_triplets=None, texcoords=None, material_ids=None, build: int = 0) -> None:
        """build: _lib.SPT_BUILD_AUTO / SPT_BUILD_HOST_SAH / SPT_BUILD_GPU_PLOC."""
        if self.device is None:
            self.init(0)
        pt = np.ascontiguousarray(np.asarray(position_triplets, dtype=np.int32).reshape(-1))
        pos = np.ascontiguousarray(np.asarray(positions, dtype=np.float32).reshape(-1))
        nt = None if shading_normal_triplets is None else np.ascontiguousarray(
            np.asarray(shading_normal_triplets, dtype=np.int32).reshape(-1))
        nrm = None if shading_normals is None else np.ascontiguousarray(
            np.asarray(shading_normals, dtype=np.float32).reshape(-1))
        tt = None if texcoord_triplets is None else np.ascontiguousarray(
            np.asarray(texcoord_triplets, dtype=np.int32).reshape(-1))
        tc = None if texcoords is None else np.ascontiguousarray(np.asarray(texcoords, dtype=np.float32).reshape(-1))
        mat = None if material_ids is None else np.ascontiguousarray(np.asarray(material_ids, dtype=np.int32).reshape(-1))
        ntri = pt.size // 3
        if self._scene.value:
            lib.spt_scene_destroy(self._scene)
            self._scene = ctypes.c_void_p()
        cfg = config_from_env(self.base_config)
        if build:
            cfg.build = build
        check(lib.spt_scene_create_cfg(
            _host_ptr(pt), _host_ptr(pos), pos.size // 3, ntri,
            _host_ptr(nt), _host_ptr(nrm), 0 if nrm is None else nrm.size // 3,
            _host_ptr(tt), _host_ptr(tc), 0 if tc is None else tc.size // 2,
            _host_ptr(mat), ctypes.byref(cfg), ctypes.byref(self._scene)), "spt_scene_create")
        self._applied = bytes(cfg)
        self._env_key = None
        st = SceneStats()
        check(lib.spt_scene_get_stats(self._scene, ctypes.byref(st)), "spt_scene_get_stats")
        self.stats = st.as_dict()

    def set_albedo(self, albedo_rgb) -> None:
        a = np.ascontiguousarray(np.asarray(albedo_rgb, dtype=np.float32).reshape(-1, 3))
        check(lib.spt_scene_set_albedo(self._scene, a.ctypes.data, a.shape[0]), "spt_scene_set_albedo")

    def set_emission(self, emission_rgb) -> None:
        e = np.ascontiguousarray(np.asarray(emission_rgb, dtype=np.float32).reshape(-1, 3))
        check(lib.spt_scene_set_emission(self._scene, e.ctypes.data, e.shape[0]), "spt_scene_set_emission")

    def set_spheres(self, center_radius=None, material_ids=None) -> None:
        """smallpt's analytic spheres: (n, 4) (cx, cy, cz, r) float32 and n material ids; None removes them."""
        if center_radius is None or len(center_radius) == 0:
            check(lib.spt_scene_set_spheres(self._scene, None, None, 0), "spt_scene_set_spheres")
            return
        cr = np.ascontiguousarray(np.asarray(center_radius, dtype=np.float32).reshape(-1, 4))
        mat = None if material_ids is None else np.ascontiguousarray(np.asarray(material_ids, dtype=np.int32))
        check(lib.spt_scene_set_spheres(self._scene, cr.ctypes.data, _host_ptr(mat), cr.shape[0]),
              "spt_scene_set_spheres")
        self._spheres = (cr, mat)

    def set_material_kinds(self, kinds) -> None:
        """Per material _lib.SPT_MAT_DIFFUSE / _MIRROR / _GLASS."""
        k = np.ascontiguousarray(np.asarray(kinds, dtype=np.uint32).reshape(-1))
        check(lib.spt_scene_set_material_kinds(self._scene, k.ctypes.data, k.size), "spt_scene_set_material_kinds")

    def set_texture(self, material: int, image=None) -> None:
        """Material `material`'s reflectance image (ImageTexture, main.cpp:34-80):
        (H, W, 3) float32, or None to remove it."""
        if image is None:
            check(lib.spt_scene_set_texture(self._scene, material, None, 0, 0), "spt_scene_set_texture")
            return
        img = np.ascontiguousarray(np.asarray(image, dtype=np.float32))
        assert img.ndim == 3 and img.shape[2] == 3, "texture must be (H, W, 3)"
        check(lib.spt_scene_set_texture(self._scene, material, img.ctypes.data, img.shape[1], img.shape[0]),
              "spt_scene_set_texture")

    def save(self, path: str, extra: bytes = b"") -> None:
        """spt_scene_save: the committed scene (BVH, arrays, materials) + extra bytes to one file."""
        check(lib.spt_scene_save(self._scene, os.fsencode(path), extra or None, len(extra)), "spt_scene_save")

    def load(self, path: str, device: int = 0) -> bytes:
        """spt_scene_load onto `device`: no parse, no build.  Returns the file's extra bytes."""
        self.init(device)
        if self._scene.value:
            lib.spt_scene_destroy(self._scene)
            self._scene = ctypes.c_void_p()
        n, cap = ctypes.c_uint64(), 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            check(lib.spt_scene_load(os.fsencode(path), ctypes.byref(self._scene), buf, cap, ctypes.byref(n)),
                  "spt_scene_load")
            if n.value <= cap:
                break
            lib.spt_scene_destroy(self._scene)      # a larger extra than the first buffer: once more
            self._scene = ctypes.c_void_p()
            cap = n.value
        cfg = Config()
        check(lib.spt_scene_get_config(self._scene, ctypes.byref(cfg)), "spt_scene_get_config")
        if self.base_config is None:
            # the file's saved knobs are the base the SPT_* overrides apply to
            # (not the library defaults, which would silently replace them)
            self.base_config = Config.from_buffer_copy(bytes(cfg))
        self._applied = bytes(cfg)
        self._env_key = None
        st = SceneStats()
        check(lib.spt_scene_get_stats(self._scene, ctypes.byref(st)), "spt_scene_get_stats")
        self.stats = st.as_dict()
        return buf.raw[:n.value]

    @property
    def handle(self):
        return self._scene

    def sync_config(self) -> None:
        """Apply base config + SPT_* environment overrides if they changed
        (a render re-reads only the variables: ~2 us when nothing changed)."""
        snap = env_snapshot()
        key = (snap, None if self.base_config is None else bytes(self.base_config))
        if key == self._env_key and self._applied is not None:
            return
        cfg = config_from_env(self.base_config, snapshot=snap)
        if bytes(cfg) != self._applied:
            check(lib.spt_scene_set_config(self._scene, ctypes.byref(cfg)), "spt_scene_set_config")
            self._applied = bytes(cfg)
        self._env_key = key

    @property
    def config(self) -> dict:
        c = Config()
        check(lib.spt_scene_get_config(self._scene, ctypes.byref(c)), "spt_scene_get_config")
        return c.as_dict()

    def _dev_mask(self, mask, dev, stream):
        """Device uint8 copy of mask, kept alive until the launch's stream has
        consumed it (record_stream: the caching allocator will not hand the
        block to another stream's allocation before that)."""
        if mask is None:
            return None, 0, None
        m = torch.as_tensor(mask, dtype=torch.uint8).to(dev).contiguous().reshape(-1)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        m.record_stream(s)
        return m.data_ptr(), m.numel(), m

    def intersect_raw(self, rays: Ray3, mask=None, do_closest: bool = True, stream=None,
                      out: Optional[Sequence[torch.Tensor]] = None):
        """__raygen__rg semantics (wavefront_isect.cu:80-112).  Returns
        (tri_id, t, u, v); masked lanes keep `out`'s values (default -1/0)."""
        n = len(rays)
        dev = rays.origin.device
        if out is None:
            tri_id = torch.full((n,), -1, dtype=torch.int32, device=dev)
            t = torch.zeros(n, dtype=torch.float32, device=dev)
            u = torch.zeros(n, dtype=torch.float32, device=dev)
            v = torch.zeros(n, dtype=torch.float32, device=dev)
        else:
            tri_id, t, u, v = out
        self.sync_config()
        mask_ptr, mask_size, m = self._dev_mask(mask, dev, stream)
        hits = Hits(tri_id.data_ptr(), t.data_ptr(), u.data_ptr(), v.data_ptr())
        rs = rays.c_struct()
        check(lib.spt_intersect(self._scene, ctypes.byref(rs), mask_ptr, mask_size, ctypes.byref(hits), n,
                                1 if do_closest else 0, _stream_handle(stream)), "spt_intersect")
        return tri_id, t, u, v

    # optix_backend.h:422-487
    def intersect(self, rays: Ray3, mask=None, stream=None):
        tri_id, t, u, v = self.intersect_raw(rays, mask, True, stream)
        n = len(rays)
        dev = rays.origin.device
        z3 = lambda: torch.zeros((3, n), dtype=torch.float32, device=dev)  # noqa: E731
        pos, gn, sn, tc = z3(), z3(), z3(), torch.zeros((2, n), dtype=torch.float32, device=dev)
        mat = torch.zeros(n, dtype=torch.int32, device=dev)
        info = HitInfo(pos[0].data_ptr(), pos[1].data_ptr(), pos[2].data_ptr(),
                       gn[0].data_ptr(), gn[1].data_ptr(), gn[2].data_ptr(),
                       sn[0].data_ptr(), sn[1].data_ptr(), sn[2].data_ptr(),
                       tc[0].data_ptr(), tc[1].data_ptr(), mat.data_ptr())
        mask_ptr, mask_size, m = self._dev_mask(mask, dev, stream)
        rs = rays.c_struct()
        hits = Hits(tri_id.data_ptr(), t.data_ptr(), u.data_ptr(), v.data_ptr())
        check(lib.spt_hit_info_compute(self._scene, ctypes.byref(rs), ctypes.byref(hits), mask_ptr, mask_size, n,
                                       ctypes.byref(info), _stream_handle(stream)), "spt_hit_info_compute")
        active = tri_id != -1                                              # optix_backend.h:463
        if mask is not None:
            mt = torch.as_tensor(mask, dtype=torch.bool).to(dev).reshape(-1)
            active = active & (mt if mt.numel() == n else mt.expand(n))
        hit = TriangleHitInfo(tri_id, t, torch.stack([u, v]), pos, gn, sn, tc, mat)
        return hit, active


def reference_camera() -> dict:
    """ThinlensCamera at main.cpp:383."""
    return dict(look_from=(0.0, 3.03, 5.0), look_at=(0.0, 0.03, 0.0), up=(0.0, 1.0, 0.0), lens_radius=0.0,
                focal_dist=1.0, fov_y=float(np.float32(np.float32(40.0) / np.float32(180.0)) * np.float32(math.pi)),
                film_size_y=0.035)


def make_params(width: int, height: int, spp: int, max_depth: int, camera: Optional[dict] = None,
                tile_index: int = 0, tile_count: int = 1, rows_per_group: int = 1, wavefront_paths: int = 0,
                rr_start_depth: int = 1, rng_order: int = 0, env=(1.0, 1.0, 1.0), timing=False,
                rng_initstate: int = _lib.PCG32_DEFAULT_STATE, pipeline: Optional[str] = None) -> RenderParams:
    """pipeline: None (library default / SPT_FUSED), "wavefront" or "fused".
    timing: False, True (HIP events around isect launches) or "all" (every launch)."""
    p = _lib.default_params()
    p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
    cam = reference_camera() if camera is None else camera
    for k in ("look_from", "look_at", "up"):
        getattr(p.camera, k)[:] = [float(x) for x in cam[k]]
    p.camera.lens_radius = cam["lens_radius"]
    p.camera.focal_dist = cam["focal_dist"]
    p.camera.fov_y = cam["fov_y"]
    p.camera.film_size_y = cam["film_size_y"]
    p.tile_index, p.tile_count, p.rows_per_group = tile_index, tile_count, rows_per_group
    p.wavefront_paths = wavefront_paths
    p.rr_start_depth = rr_start_depth
    p.rng_order = rng_order
    p.rng_initstate = rng_initstate
    p.env[:] = [float(e) for e in env]
    p.flags = _lib.SPT_FLAG_TIMING if timing else 0     # timing="all": every launch, not only isect
    if timing == "all":
        p.flags |= _lib.SPT_FLAG_TIMING_ALL
    if pipeline == "fused":
        p.flags |= _lib.SPT_FLAG_FUSED
    elif pipeline == "wavefront":
        p.flags |= _lib.SPT_FLAG_WAVEFRONT
    elif pipeline is not None:
        raise ValueError(f"pipeline must be None, 'wavefront' or 'fused', not {pipeline!r}")
    return p


class Scene:
    """main.cpp:286-352: add_triangle_mesh / commit / intersect, plus render()."""

    def __init__(self, config: Optional[Config] = None):
        self.backend = HipBackend(config)
        self.mesh = None
        self.pbrt_info: Optional[dict] = None

    def add_triangle_mesh(self, path: str) -> None:       # main.cpp:288-310
        """An OBJ (load_meshes) or, by extension, a pbrt-v3 scene; for .pbrt
        the file's camera / film / infinite light land in self.pbrt_info."""
        from .scenes import load_obj, load_pbrt
        if path.endswith(".pbrt"):
            self.mesh, self.pbrt_info = load_pbrt(path)
        else:
            self.mesh = load_obj(path)

    def add_arrays(self, mesh: dict) -> None:
        self.mesh = mesh

    def commit(self, device: int = 0, build: int = 0) -> None:  # main.cpp:312-318
        m = self.mesh
        self.backend.init(device)
        self.backend.set_triangles_soup(m["pos_tri"], m["pos"], m.get("nrm_tri"), m.get("nrm"), m.get("tc_tri"),
                                        m.get("tc"), m.get("mat_id"), build=build)
        if m.get("albedo") is not None:
            self.backend.set_albedo(m["albedo"])
        if m.get("emission") is not None:
            self.backend.set_emission(m["emission"])
        if m.get("spheres") is not None:
            self.backend.set_spheres(m["spheres"], m.get("sphere_mat"))
        if m.get("kinds") is not None:
            self.backend.set_material_kinds(m["kinds"])

    def save(self, path: str) -> None:
        """Binary scene cache of the committed scene (spt_scene_save); pbrt_info rides
        along as the extra bytes (an spt_pbrt_info, as spt_render_cli --save-cache writes)."""
        from .scenes import pbrt_info_to_c
        self.backend.save(path, bytes(pbrt_info_to_c(self.pbrt_info)) if self.pbrt_info is not None else b"")

    @classmethod
    def load(cls, path: str, device: int = 0, config: Optional[Config] = None) -> "Scene":
        """A committed Scene from a spt_scene_save file (no parse, no BVH build); mesh stays None."""
        sc = cls(config)
        extra = sc.backend.load(path, device)
        if len(extra) == ctypes.sizeof(_lib.PbrtInfo):
            from .scenes import pbrt_info_from_c
            sc.pbrt_info = pbrt_info_from_c(_lib.PbrtInfo.from_buffer_copy(extra))
        elif extra:
            raise ValueError(f"{path}: {len(extra)} extra bytes are not an spt_pbrt_info")
        return sc

    def intersect(self, ray: Ray3, active=None):           # main.cpp:320-340
        return self.backend.intersect(ray, active)

    def render(self, params: RenderParams, film: Optional[torch.Tensor] = None, stream=None):
        """One wavefront render of params' tile.  Returns (film (3, rows, W)
        float32 on the device, stats dict)."""
        film = self._film(params, film)
        st = RenderStats()
        self.backend.sync_config()
        check(lib.spt_render(self.backend.handle, ctypes.byref(params), film.data_ptr(), ctypes.byref(st),
                             _stream_handle(stream)), "spt_render")
        return film, st.as_dict()

    def render_async(self, params: RenderParams, film: Optional[torch.Tensor] = None, stream=None):
        """spt_render_async: queue the render and return (film, ticket) without
        waiting for it; collect its stats with render_wait(ticket)."""
        film = self._film(params, film)
        ticket = ctypes.c_uint64()
        self.backend.sync_config()
        check(lib.spt_render_async(self.backend.handle, ctypes.byref(params), film.data_ptr(),
                                   _stream_handle(stream), ctypes.byref(ticket)), "spt_render_async")
        return film, ticket.value

    def render_wait(self, ticket: int) -> dict:
        """spt_render_wait: the stats dict of a queued render (waits for it)."""
        st = RenderStats()
        check(lib.spt_render_wait(self.backend.handle, ticket, ctypes.byref(st)), "spt_render_wait")
        return st.as_dict()

    def isect_busy_begin(self) -> None:
        """spt_scene_isect_busy_begin: start collecting isect launch intervals."""
        check(lib.spt_scene_isect_busy_begin(self.backend.handle), "spt_scene_isect_busy_begin")

    def kernel_busy(self, kernels: int = _lib.SPT_KERNEL_ISECT) -> Tuple[float, int]:
        """spt_scene_kernel_busy: (union of the isect / drain launch intervals
        collected since isect_busy_begin, in ms; launches), without stopping
        the collection.  kernels: a mask of _lib.SPT_KERNEL_*."""
        ms, n = ctypes.c_double(0.0), ctypes.c_uint64(0)
        check(lib.spt_scene_kernel_busy(self.backend.handle, kernels, ctypes.byref(ms), ctypes.byref(n)),
              "spt_scene_kernel_busy")
        return ms.value, n.value

    def isect_busy_end(self) -> Tuple[float, int]:
        """spt_scene_isect_busy_end: (union of the intervals collected since
        isect_busy_begin in ms, launches) across every render collected."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        check(lib.spt_scene_isect_busy_end(self.backend.handle, ctypes.byref(ms), ctypes.byref(n)),
              "spt_scene_isect_busy_end")
        return ms.value, n.value

    def _film(self, params: RenderParams, film: Optional[torch.Tensor]) -> torch.Tensor:
        rows = _lib.tile_row_count(params.height, params.tile_index, params.tile_count, params.rows_per_group)
        if film is None:
            film = torch.empty((3, rows, params.width), dtype=torch.float32, device=self.backend.device)
        assert film.is_contiguous() and film.numel() >= 3 * rows * params.width
        return film


def scene_cache_info(path: str) -> dict:
    """spt_scene_cache_info: checks a scene cache file (header, sizes, every
    section's checksum) without a device; returns its stats, config and extra size."""
    st, cfg, n = SceneStats(), Config(), ctypes.c_uint64()
    check(lib.spt_scene_cache_info(os.fsencode(path), ctypes.byref(st), ctypes.byref(cfg), ctypes.byref(n)),
          "spt_scene_cache_info")
    return {"stats": st.as_dict(), "config": cfg.as_dict(), "extra_bytes": n.value}


def write_pfm(path: str, film: np.ndarray) -> None:
    """Fimage::save_pfm via the C ABI; film: (3, H, W) float32 host array."""
    f = np.ascontiguousarray(film, dtype=np.float32)
    _, h, w = f.shape
    check(lib.spt_pfm_write(path.encode(), f[0].ctypes.data, f[1].ctypes.data, f[2].ctypes.data, w, h),
          "spt_pfm_write")
