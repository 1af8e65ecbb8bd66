"""distributed_raytracer_amd — MI355X-native trace worker for MWindels/distributed-raytracer.

The hot path (per-pixel ray generation, fp64 Möller–Trumbore nearest hit, shadow rays,
Phong) runs as hand-written gfx950 HIP kernels in libmirt.so behind the C ABI of
include/mirt.h.  This package is the Python host mirror of the reference's worker
interfaces (tracer.Trace, BulkTrace, draw) plus the multi-GPU framebuffer tiling.
Importing it loads libmirt.so and raises if it is missing: there is no CPU fallback.
"""
from . import _lib
from ._lib import MirtError

_lib.lib()  # fail loudly at import if the HIP library was not built

from .tracer import (RGB, Box, Camera, Context, EnvMutables, Environment, Framebuffer, Light,  # noqa: E402
                     SceneObject, TraceResults, Tracer, WorkOrder, draw, load_scene_arrays, trace,
                     trace_rays, trace_tile)

__all__ = ["MirtError", "RGB", "Box", "Camera", "Context", "EnvMutables", "Environment", "Framebuffer", "Light",
           "SceneObject", "TraceResults", "Tracer", "WorkOrder", "draw", "load_scene_arrays", "trace",
           "trace_rays", "trace_tile"]
