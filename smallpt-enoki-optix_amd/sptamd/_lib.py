"""ctypes binding of include/spt.h (libspt.so, built in-tree by the Makefile).

The library is the only compute path: if it is missing, import fails loudly
(there is no CPU fallback in the product).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_uint8, c_uint32, c_uint64, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
# SPT_LIB: a variant build of the same library (A/B experiments, tools/ab.sh)
LIB_PATH = os.environ.get("SPT_LIB") or os.path.join(PKG_ROOT, "build", "libspt.so")

SPT_OK = 0
SPT_ERR_INVALID, SPT_ERR_HIP, SPT_ERR_NO_DEVICE, SPT_ERR_OOM, SPT_ERR_IO, SPT_ERR_LIMIT = 1, 2, 3, 4, 5, 6
SPT_RNG_Y_FIRST = 0
SPT_RNG_X_FIRST = 1
SPT_FLAG_TIMING = 1
SPT_FLAG_TRAVERSAL_STATS = 2
SPT_FLAG_FUSED = 4
SPT_FLAG_WAVEFRONT = 8
SPT_FLAG_TIMING_ALL = 16
PCG32_DEFAULT_STATE = 0x853C49E6748FEA9B
SPT_BUILD_AUTO, SPT_BUILD_HOST_SAH, SPT_BUILD_GPU_PLOC = 0, 1, 2

# Every function include/spt.h declares (the CPU test checks they are exported).
EXPORTED = [
    "spt_init", "spt_scene_create", "spt_scene_create_ex", "spt_scene_set_albedo", "spt_scene_set_emission", "spt_scene_get_stats",
    "spt_scene_destroy", "spt_intersect", "spt_hit_info_compute", "spt_render", "spt_render_async", "spt_render_wait",
    "spt_tile_rows", "spt_default_params", "spt_last_error", "spt_version", "spt_build_id",
    "spt_obj_load", "spt_mesh_free", "spt_pfm_write", "spt_pbrt_load",
    "spt_default_config", "spt_scene_create_cfg", "spt_scene_set_config", "spt_scene_get_config",
    "spt_bvh_build_stats", "spt_scene_set_texture", "spt_scene_set_spheres", "spt_scene_set_material_kinds",
    "spt_scene_save", "spt_scene_load", "spt_scene_cache_info",
    "spt_scene_isect_busy_begin", "spt_scene_isect_busy_end", "spt_scene_kernel_busy",
    "spt_debug_fail_workspace_alloc",
]
SPT_MAT_DIFFUSE, SPT_MAT_MIRROR, SPT_MAT_GLASS = 0, 1, 2
SPT_PIPELINE_AUTO, SPT_PIPELINE_WAVEFRONT, SPT_PIPELINE_FUSED = 0, 1, 2
SPT_WORK_AUTO, SPT_WORK_SAMPLE_MAJOR, SPT_WORK_PIXEL_MAJOR = 0, 1, 2
SPT_QUEUE_CACHE_AUTO, SPT_QUEUE_CACHE_CACHED, SPT_QUEUE_CACHE_STREAM = 0, 1, 2
SPT_KERNEL_ISECT, SPT_KERNEL_DRAIN = 1, 2


class SptError(RuntimeError):
    """Raised for a non-zero spt_status (the reference throws std::runtime_error
    from OPTIX_CHECK / CUDA_CHECK, optix_backend.h:25-66)."""

    def __init__(self, what: str, code: int, msg: str):
        super().__init__(f"{what} failed ({code}): {msg}")
        self.code = code


class Rays(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("ox", "oy", "oz", "dx", "dy", "dz", "tmin", "tmax")]


class Hits(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("tri_id", "t", "u", "v")]


class HitInfo(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("px", "py", "pz", "gnx", "gny", "gnz", "snx", "sny", "snz",
                                        "tcu", "tcv", "mat_id")]


class Camera(ctypes.Structure):
    _fields_ = [("look_from", c_float * 3), ("look_at", c_float * 3), ("up", c_float * 3),
                ("lens_radius", c_float), ("focal_dist", c_float), ("fov_y", c_float),
                ("film_size_y", c_float)]


class RenderParams(ctypes.Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("spp", c_uint32), ("max_depth", c_uint32),
                ("camera", Camera),
                ("tile_index", c_uint32), ("tile_count", c_uint32), ("rows_per_group", c_uint32),
                ("wavefront_paths", c_uint32), ("rr_start_depth", c_uint32), ("rng_order", c_uint32),
                ("rng_initstate", c_uint64), ("env", c_float * 3), ("flags", c_uint32)]


class RenderStats(ctypes.Structure):
    _fields_ = [("paths", c_uint64), ("ray_casts", c_uint64), ("continuations", c_uint64),
                ("regenerations", c_uint64), ("iterations", c_uint64),
                ("paths_in_flight", c_uint32), ("tile_rows", c_uint32),
                ("isect_ms", c_double), ("shade_ms", c_double), ("camera_ms", c_double),
                ("resolve_ms", c_double), ("total_ms", c_double),
                ("isect_nodes", c_uint64), ("isect_tris", c_uint64), ("isect_lane_steps", c_uint64),
                ("isect_wave_steps", c_uint64), ("isect_launches", c_uint64), ("streams", c_uint32),
                ("fused", c_uint32), ("isect_busy_ms", c_double),
                ("isect_max_stack", c_uint64),
                ("paths_started", c_uint64), ("paths_terminated", c_uint64), ("film_slots_unwritten", c_uint64),
                ("work_order", c_uint32), ("queue_cache", c_uint32),
                ("isect_tri_wave_steps", c_uint64), ("isect_node_wave_steps", c_uint64),
                ("isect_begin_ms", c_double), ("isect_end_ms", c_double),
                ("drained_paths", c_uint64), ("drain_launches", c_uint64), ("drained_casts", c_uint64),
                ("drain_ms", c_double), ("drain_busy_ms", c_double), ("lockstep_casts", c_uint64),
                ("fit_paths", c_uint64), ("fit_retries", c_uint64),
                ("drain_refill_idle", c_uint32)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class SceneStats(ctypes.Structure):
    _fields_ = [("ntri", c_uint64), ("nodes", c_uint64), ("leaves", c_uint64),
                ("max_depth", c_uint32), ("max_leaf", c_uint32), ("bvh_width", c_uint32), ("builder", c_uint32),
                ("device_bytes", c_uint64),
                ("build_ms", c_double), ("sah_cost", c_double)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class Config(ctypes.Structure):
    """spt_config (include/spt.h): the library's build and tuning knobs."""
    _fields_ = [("build", c_uint32), ("bvh_width", c_uint32), ("gpu_build_min_tris", c_uint64),
                ("collapse", c_uint32), ("ploc_radius", c_uint32), ("stack_slack", c_uint32),
                ("pipeline", c_uint32), ("fused_max_paths", c_uint64), ("wavefront_paths", c_uint32),
                ("streams", c_uint32), ("isect_refill_idle", c_uint32), ("isect_static_share_q8", c_uint32),
                ("isect_chunk", c_uint32), ("isect_grid_q8", c_uint32), ("xcd_remap", c_uint32),
                ("fused_refill_idle", c_uint32), ("fused_static_share_q8", c_uint32), ("fused_grid_q8", c_uint32),
                ("plane_pad", c_uint32), ("film_budget_bytes", c_uint64),
                ("public_persistent", c_uint32), ("public_refill_idle", c_uint32), ("pack_groups", c_uint32),
                ("pixel_block", c_uint32), ("work_order", c_uint32), ("queue_cache", c_uint32),
                ("drain_q8", c_uint32), ("drain_grid_q8", c_uint32), ("drain_casts", c_uint32),
                ("fit_streams", c_uint32), ("fit_paths", c_uint64), ("sub_queues", c_uint32),
                ("drain_sort", c_uint32), ("lockstep_first", c_uint32), ("fit_chunks", c_uint32),
                ("fit_bytes", c_uint64), ("drain_refill_idle", c_uint32)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class Mesh(ctypes.Structure):
    _fields_ = [("pos_tri", POINTER(c_int32)), ("pos", POINTER(c_float)), ("nvert", c_uint64), ("ntri", c_uint64),
                ("nrm_tri", POINTER(c_int32)), ("nrm", POINTER(c_float)), ("nnrm", c_uint64),
                ("tc_tri", POINTER(c_int32)), ("tc", POINTER(c_float)), ("ntc", c_uint64),
                ("mat_id", POINTER(c_int32)), ("kd", POINTER(c_float)), ("nmat", c_uint32),
                ("ke", POINTER(c_float))]


class PbrtInfo(ctypes.Structure):
    _fields_ = [("has_camera", c_uint32), ("camera", Camera), ("fov_deg", c_float), ("xres", c_uint32),
                ("yres", c_uint32), ("has_env", c_uint32), ("env", c_float * 3), ("shapes", c_uint64),
                ("shapes_skipped", c_uint64), ("instances", c_uint64)]


def _load() -> ctypes.CDLL:
    # torch ships its own HIP runtime (SONAME libamdhip64.so.7).  Load it first
    # so libspt.so binds to that one copy: loading libspt.so first would map the
    # system runtime too and put two HIP runtimes in one process.
    import torch  # noqa: F401

    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libspt.so not built at {LIB_PATH}: run `make -C smallpt-enoki-optix_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    i32, u32, u64, vp = c_int32, c_uint32, c_uint64, c_void_p
    sig = {
        "spt_init": (i32, [i32]),
        "spt_scene_create": (i32, [vp, vp, u64, u64, vp, vp, u64, vp, vp, u64, vp, POINTER(vp)]),
        "spt_scene_create_ex": (i32, [vp, vp, u64, u64, vp, vp, u64, vp, vp, u64, vp, u32, POINTER(vp)]),
        "spt_scene_set_albedo": (i32, [vp, vp, u32]),
        "spt_scene_set_emission": (i32, [vp, vp, u32]),
        "spt_scene_get_stats": (i32, [vp, POINTER(SceneStats)]),
        "spt_scene_destroy": (i32, [vp]),
        "spt_intersect": (i32, [vp, POINTER(Rays), vp, u32, POINTER(Hits), u32, i32, vp]),
        "spt_hit_info_compute": (i32, [vp, POINTER(Rays), POINTER(Hits), vp, u32, u32, POINTER(HitInfo), vp]),
        "spt_render": (i32, [vp, POINTER(RenderParams), vp, POINTER(RenderStats), vp]),
        "spt_render_async": (i32, [vp, POINTER(RenderParams), vp, vp, POINTER(u64)]),
        "spt_render_wait": (i32, [vp, u64, POINTER(RenderStats)]),
        "spt_scene_isect_busy_begin": (i32, [vp]),
        "spt_scene_isect_busy_end": (i32, [vp, POINTER(ctypes.c_double), POINTER(u64)]),
        "spt_scene_kernel_busy": (i32, [vp, u32, POINTER(ctypes.c_double), POINTER(u64)]),
        "spt_tile_rows": (u32, [u32, u32, u32, u32, vp, u32]),
        "spt_default_params": (None, [POINTER(RenderParams)]),
        "spt_last_error": (c_char_p, []),
        "spt_version": (c_char_p, []),
        "spt_build_id": (c_char_p, []),
        "spt_debug_fail_workspace_alloc": (None, [ctypes.c_int32]),
        "spt_obj_load": (i32, [c_char_p, POINTER(Mesh)]),
        "spt_mesh_free": (None, [POINTER(Mesh)]),
        "spt_pbrt_load": (i32, [c_char_p, POINTER(Mesh), POINTER(PbrtInfo)]),
        "spt_pfm_write": (i32, [c_char_p, vp, vp, vp, u32, u32]),
        "spt_default_config": (None, [POINTER(Config)]),
        "spt_scene_create_cfg": (i32, [vp, vp, u64, u64, vp, vp, u64, vp, vp, u64, vp, POINTER(Config), POINTER(vp)]),
        "spt_scene_set_config": (i32, [vp, POINTER(Config)]),
        "spt_scene_get_config": (i32, [vp, POINTER(Config)]),
        "spt_bvh_build_stats": (i32, [vp, u64, POINTER(Config), POINTER(SceneStats)]),
        "spt_scene_set_texture": (i32, [vp, u32, vp, u32, u32]),
        "spt_scene_set_spheres": (i32, [vp, vp, vp, u32]),
        "spt_scene_set_material_kinds": (i32, [vp, vp, u32]),
        "spt_scene_save": (i32, [vp, c_char_p, vp, u64]),
        "spt_scene_load": (i32, [c_char_p, POINTER(vp), vp, u64, POINTER(u64)]),
        "spt_scene_cache_info": (i32, [c_char_p, POINTER(SceneStats), POINTER(Config), POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int, what: str) -> None:
    if status != SPT_OK:
        raise SptError(what, status, lib.spt_last_error().decode(errors="replace"))


def default_params() -> RenderParams:
    p = RenderParams()
    lib.spt_default_params(ctypes.byref(p))
    return p


def default_config() -> Config:
    c = Config()
    lib.spt_default_config(ctypes.byref(c))
    return c


# SPT_* environment overrides of spt_config (the host's knobs; the library
# itself reads no environment): variable -> (field, parser)
_ENV_CONFIG = {
    "SPT_BUILD": ("build", lambda v: {"auto": 0, "host": 1, "gpu": 2}[v]),
    "SPT_BVH": ("bvh_width", int),
    "SPT_GPU_BUILD_MIN_TRIS": ("gpu_build_min_tris", int),
    "SPT_COLLAPSE": ("collapse", lambda v: {"sah": 0, "dp": 0, "greedy": 1}[v]),
    "SPT_PLOC_RADIUS": ("ploc_radius", int),
    "SPT_STACK_SLACK": ("stack_slack", int),
    "SPT_FUSED": ("pipeline", lambda v: {"0": 1, "1": 2, "2": 0, "auto": 0}[v]),
    "SPT_FUSED_MAX_PATHS": ("fused_max_paths", int),
    "SPT_WAVEFRONT_PATHS": ("wavefront_paths", int),
    "SPT_STREAMS": ("streams", int),
    "SPT_REFILL_IDLE": ("isect_refill_idle", int),
    "SPT_STATIC_SHARE_Q8": ("isect_static_share_q8", int),
    "SPT_CHUNK": ("isect_chunk", int),
    "SPT_ISECT_GRID_Q8": ("isect_grid_q8", int),
    "SPT_XCD": ("xcd_remap", int),
    "SPT_FUSED_IDLE": ("fused_refill_idle", int),
    "SPT_FUSED_STATIC_SHARE_Q8": ("fused_static_share_q8", int),
    "SPT_FUSED_GRID_Q8": ("fused_grid_q8", int),
    "SPT_PLANE_PAD": ("plane_pad", int),
    "SPT_FILM_BUDGET": ("film_budget_bytes", int),
    "SPT_PUBLIC_PERSISTENT": ("public_persistent", int),
    "SPT_PUBLIC_REFILL_IDLE": ("public_refill_idle", int),
    "SPT_PACK": ("pack_groups", int),
    "SPT_PIXEL_BLOCK": ("pixel_block", int),
    "SPT_WORK_ORDER": ("work_order", int),
    "SPT_QUEUE_CACHE": ("queue_cache", int),
    "SPT_DRAIN_Q8": ("drain_q8", int),
    "SPT_DRAIN_GRID_Q8": ("drain_grid_q8", int),
    "SPT_DRAIN_CASTS": ("drain_casts", int),
    "SPT_FIT_STREAMS": ("fit_streams", int),
    "SPT_FIT_PATHS": ("fit_paths", int),
    "SPT_SUB_QUEUES": ("sub_queues", int),
    "SPT_DRAIN_SORT": ("drain_sort", int),
    "SPT_LOCKSTEP_FIRST": ("lockstep_first", int),
    "SPT_FIT_CHUNKS": ("fit_chunks", int),
    "SPT_FIT_BYTES": ("fit_bytes", int),
    "SPT_DRAIN_IDLE": ("drain_refill_idle", int),
}


_ENV_BKEYS = tuple(os.environ.encodekey(k) for k in _ENV_CONFIG) if hasattr(os.environ, "encodekey") else None


def env_snapshot(environ=None) -> tuple:
    """The SPT_* variables' values, in _ENV_CONFIG order (None = unset).  For
    os.environ it reads the underlying dict: os.environ.get of an unset key
    costs ~1.3 us (a KeyError inside), which made every render pay ~30 us."""
    if environ is None:
        environ = os.environ
    data = getattr(environ, "_data", None)
    if environ is os.environ and _ENV_BKEYS is not None and isinstance(data, dict):
        return tuple(None if v is None else os.environ.decodevalue(v) for v in map(data.get, _ENV_BKEYS))
    return tuple(environ.get(k) for k in _ENV_CONFIG)


def config_from_env(base: Config = None, environ=None, snapshot: tuple = None) -> Config:
    """spt_config with the SPT_* environment variables applied over `base`
    (default: spt_default_config).  An unparsable value raises ValueError."""
    values = env_snapshot(environ) if snapshot is None else snapshot
    c = default_config() if base is None else Config.from_buffer_copy(base)
    for (var, (field, parse)), v in zip(_ENV_CONFIG.items(), values):
        if v is None or v == "":
            continue
        try:
            setattr(c, field, parse(v.strip()))
        except (KeyError, ValueError) as e:
            raise ValueError(f"{var}={v!r}: not a valid spt_config.{field}") from e
    return c


def tile_row_count(height: int, tile_index: int, tile_count: int, rows_per_group: int) -> int:
    """spt_tile_rows' count in closed form (no ctypes call on the render path):
    rows r < height with (r // rows_per_group) % tile_count == tile_index."""
    if tile_count == 0 or rows_per_group == 0 or tile_index >= tile_count:
        return 0
    groups, rem = divmod(height, rows_per_group)           # whole groups, rows of the last partial one
    mine = groups // tile_count + (1 if tile_index < groups % tile_count else 0)
    return mine * rows_per_group + (rem if groups % tile_count == tile_index else 0)


def tile_rows(height: int, tile_index: int, tile_count: int, rows_per_group: int):
    import numpy as np
    n = lib.spt_tile_rows(height, tile_index, tile_count, rows_per_group, None, 0)
    rows = np.zeros(max(n, 1), dtype=np.uint32)
    lib.spt_tile_rows(height, tile_index, tile_count, rows_per_group, rows.ctypes.data, n)
    return rows[:n].astype(np.int64)


__all__ = [
    "lib", "check", "SptError", "Rays", "Hits", "HitInfo", "Camera", "RenderParams", "RenderStats",
    "SceneStats", "Mesh", "Config", "default_params", "default_config", "config_from_env", "tile_rows", "EXPORTED",
    "LIB_PATH", "REPO_ROOT",
    "PCG32_DEFAULT_STATE", "SPT_RNG_Y_FIRST", "SPT_RNG_X_FIRST", "SPT_FLAG_TIMING", "c_uint8",
]
