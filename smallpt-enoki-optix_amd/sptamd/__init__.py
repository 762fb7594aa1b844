"""sptamd — host side of the MI355X-native wavefront path tracer.

Importing this package loads libspt.so (HIP kernels for gfx950 behind the C
ABI of include/spt.h) and fails loudly when it has not been built.
"""
from . import _lib
from ._lib import Config, SptError, check, config_from_env, default_config, default_params, lib, tile_rows
from .backend import (HipBackend, Ray3, Scene, TriangleHitInfo, make_params, queue_stream, reference_camera,
                      scene_cache_info, write_pfm)

__all__ = ["_lib", "Config", "SptError", "check", "config_from_env", "default_config", "default_params", "lib",
           "tile_rows", "HipBackend", "Ray3", "Scene",
           "TriangleHitInfo", "make_params", "queue_stream", "reference_camera", "scene_cache_info", "write_pfm"]
