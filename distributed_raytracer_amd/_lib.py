"""ctypes binding of libmirt.so (include/mirt.h, include/mirt_scene.h).

This module never falls back to anything: if the HIP library is missing it raises,
and every failing C call raises MirtError with mirt_last_error()'s text.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIRT_LIB: load another build of the library (A/B experiments with kernel variants)
LIB_PATH = os.environ.get("MIRT_LIB") or os.path.join(_HERE, "libmirt.so")

MIRT_OK = 0
MIRT_E_INVALID = -1
MIRT_E_DEVICE = -2
MIRT_E_LIMIT = -3
MIRT_E_NOMEM = -4
MIRT_E_CAMERA = -5
MIRT_E_CANCELLED = -6
MIRT_E_IO = -7
MIRT_E_TIMEOUT = -8
MIRT_E_PEER = -9
MIRT_MAX_OBJECTS = 16
MIRT_NO_MESH = 0xFFFFFFFF
MIRT_MAX_LIGHTS = 16
MIRT_OPT_NO_PREFILTER = 1
MIRT_OPT_BRUTE_FORCE = 2
MIRT_OPT_STATIC_SCHEDULE = 4
MIRT_OPT_TIMELINE = 8
MIRT_OPT_NO_SEGMENT = 16
MIRT_OPT_SPLIT_KERNELS = 32
MIRT_OPT_NO_FRUSTUM = 64
MIRT_OPT_NO_OCTANT = 128
MIRT_OPT_VIEWS = 256
MIRT_OPT_REFLECT_CHAINS = 512
MIRT_OPT_NO_LIGHT_TABLE = 1024
MIRT_OPT_NO_BOX_GATE = 2048
MIRT_OPT_LDS_STREAM = 4096
MIRT_OPT_NO_LDS_STREAM = 8192

D3 = C.c_double * 3


class Material(C.Structure):
    _fields_ = [("ka", D3), ("kd", D3), ("ks", D3), ("ns", C.c_double)]


class Object(C.Structure):
    _fields_ = [("mesh_id", C.c_uint32), ("reserved", C.c_uint32), ("pos", D3)]


class Light(C.Structure):
    _fields_ = [("pos", D3), ("col", D3)]


class Camera(C.Structure):
    _fields_ = [("pos", D3), ("forward", D3), ("left", D3), ("up", D3), ("fov", C.c_double),
                ("proj_half_width", C.c_double)]


class Frame(C.Structure):
    _fields_ = [("objects", C.POINTER(Object)), ("n_objects", C.c_uint32),
                ("lights", C.POINTER(Light)), ("n_lights", C.c_uint32), ("camera", Camera),
                ("max_bounces", C.c_uint32), ("reserved", C.c_uint32)]


class Tile(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("w", C.c_uint32), ("h", C.c_uint32)]


class Outputs(C.Structure):
    _fields_ = [("rgb", C.c_void_p), ("rgb8", C.c_void_p), ("valid", C.c_void_p), ("face", C.c_void_p),
                ("object", C.c_void_p), ("rgbv", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("hits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("ms_primary", C.c_double), ("ms_shadow", C.c_double),
                ("ms_shade", C.c_double), ("ms_total", C.c_double), ("reflection_rays", C.c_uint64)]


class Profile(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("primary_ms_sum", C.c_double), ("shadow_ms_sum", C.c_double),
                ("shade_ms_sum", C.c_double), ("frame_ms_sum", C.c_double),
                ("primary_tri_tests", C.c_uint64), ("shadow_tri_tests", C.c_uint64),
                ("primary_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("hits", C.c_uint64),
                ("primary_node_visits", C.c_uint64), ("primary_leaf_visits", C.c_uint64),
                ("shadow_node_visits", C.c_uint64), ("shadow_leaf_visits", C.c_uint64),
                ("stack_overflows", C.c_uint64), ("reflection_rays", C.c_uint64), ("reflect_ms_sum", C.c_double),
                ("frames", C.c_uint64), ("primary_ms_median", C.c_double), ("frame_ms_median", C.c_double),
                ("redo_items", C.c_uint64)]


class MeshView(C.Structure):
    _fields_ = [("vertices", C.POINTER(C.c_double)), ("n_vertices", C.c_uint32),
                ("normals", C.POINTER(C.c_double)), ("n_normals", C.c_uint32),
                ("face_v", C.POINTER(C.c_uint32)), ("face_n", C.POINTER(C.c_uint32)),
                ("face_mat", C.POINTER(C.c_uint32)), ("n_faces", C.c_uint32),
                ("materials", C.POINTER(Material)), ("n_materials", C.c_uint32)]


class MirtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mirt error {code}: {msg}")
        self.code = code


# every symbol include/*.h declares: name -> (restype, argtypes)
_P = C.c_void_p
SIGNATURES = {
    "mirt_abi_version": (C.c_int, []),
    "mirt_build_id": (C.c_char_p, []),
    "mirt_last_error": (C.c_char_p, []),
    "mirt_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "mirt_destroy": (None, [_P]),
    "mirt_device": (C.c_int, [_P]),
    "mirt_camera_init": (C.c_int, [_P, _P, C.c_double, C.POINTER(Camera)]),
    "mirt_go_tan": (C.c_double, [C.c_double]),
    "mirt_go_pow": (C.c_double, [C.c_double, C.c_double]),
    "mirt_go_minmax": (C.c_double, [C.c_int, C.c_double, C.c_double]),
    "mirt_mesh_upload": (C.c_int, [_P, _P, C.c_uint32, _P, C.c_uint32, _P, _P, _P, C.c_uint32,
                                   C.POINTER(Material), C.c_uint32, C.POINTER(C.c_uint32)]),
    "mirt_mesh_release": (C.c_int, [_P, C.c_uint32]),
    "mirt_trace_tile": (C.c_int, [_P, C.POINTER(Frame), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_uint32, C.POINTER(Outputs), _P, C.POINTER(Stats)]),
    "mirt_trace_tiles_async": (C.c_int, [_P, C.POINTER(Frame), C.c_uint32, C.c_uint32, C.POINTER(Tile),
                                         C.c_uint32, C.POINTER(Outputs), _P, C.POINTER(Stats)]),
    "mirt_unpack_tiles_async": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(Tile), C.c_uint32,
                                          C.POINTER(Outputs), C.POINTER(Outputs), _P]),
    "mirt_trace_rays": (C.c_int, [_P, C.POINTER(Frame), C.c_uint32, _P, _P, _P, _P, _P, _P, _P]),
    "mirt_profile_enable": (C.c_int, [_P, C.c_int]),
    "mirt_profile_read": (C.c_int, [_P, C.POINTER(Profile)]),
    "mirt_set_options": (C.c_int, [_P, C.c_uint32]),
    "mirt_set_grid": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "mirt_stream_create": (C.c_int, [_P, C.POINTER(_P)]),
    "mirt_group_unique_id": (C.c_int, [_P]),
    "mirt_group_create": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32, _P, C.POINTER(_P)]),
    "mirt_trace_frame": (C.c_int, [_P, C.POINTER(Frame), C.POINTER(C.c_uint64)]),
    "mirt_group_set_batch": (C.c_int, [_P, C.c_uint32]),
    "mirt_group_wait": (C.c_int, [_P, _P]),
    "mirt_group_destroy": (None, [_P]),
    "mirt_plan_tiles": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P,
                                  C.c_uint32]),
    "mirt_group_plan_tiles": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P,
                                        C.c_uint32]),
    "mirt_stream_destroy": (C.c_int, [_P, _P]),
    "mirt_group_set_timeout": (C.c_int, [_P, C.c_uint32]),
    "mirt_group_failed_ranks": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "mirt_group_exclude": (C.c_int, [_P, C.c_uint64, _P]),
    "mirt_group_emulate": (C.c_int, [_P, C.c_uint32]),
    "mirt_group_emulate_drop": (C.c_int, [_P, C.c_uint64]),
    "mirt_group_set_host_output": (C.c_int, [_P, C.c_int]),
    "mirt_group_frame_host": (C.c_int, [_P, C.c_uint64, C.POINTER(Outputs)]),
    "mirt_debug_fp64": (C.c_int, [_P, C.c_int, C.c_uint32, _P, _P, _P]),
    "mirt_debug_timeline": (C.c_int, [_P, _P, C.c_uint32]),
    "mirt_debug_counters": (C.c_int, [_P, _P, C.c_uint32]),
    "mirt_debug_kernarg_layout": (C.c_int, [_P, C.c_uint32]),
    "mirt_debug_light_table": (C.c_int, [_P, C.c_uint32, C.c_double, _P, _P, C.c_uint32, _P]),
    "mirt_debug_light_table_gpu": (C.c_int, [_P, _P, C.c_uint32, C.c_double, _P, _P, C.c_uint32, _P]),
    "mirt_set_light_cache": (C.c_int, [_P, C.c_uint64]),
    "mirt_light_cache_stats": (C.c_int, [_P, _P]),
    "mirt_face_bounds": (None, [_P, _P, _P, _P]),
    "mirt_object_bounds": (None, [_P, C.c_uint32, _P, _P]),
    "mirt_unpack_tiles_at_async": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, C.c_uint32, _P, _P, _P]),
    "mirt_scene_load": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "mirt_scene_free": (None, [_P]),
    "mirt_scene_last_error": (C.c_char_p, []),
    "mirt_scene_mesh_count": (C.c_uint32, [_P]),
    "mirt_scene_mesh": (C.c_int, [_P, C.c_uint32, C.POINTER(MeshView)]),
    "mirt_scene_object_count": (C.c_uint32, [_P]),
    "mirt_scene_object": (C.c_int, [_P, C.c_uint32, C.POINTER(Object)]),
    "mirt_scene_light_count": (C.c_uint32, [_P]),
    "mirt_scene_light": (C.c_int, [_P, C.c_uint32, C.POINTER(Light)]),
    "mirt_scene_camera": (C.c_int, [_P, C.POINTER(Camera)]),
    "mirt_scene_from_gob": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "mirt_scene_link_gob": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "mirt_gob_json": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    # one process driving the GPUs of a box (ABI 7)
    "mirt_device_count": (C.c_int, []),
    "mirt_box_create": (C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    "mirt_box_destroy": (None, [_P]),
    "mirt_box_size": (C.c_int, [_P]),
    "mirt_box_ctx": (_P, [_P, C.c_uint32]),
    "mirt_box_set_transport": (C.c_int, [_P, C.c_int]),
    "mirt_box_transport": (C.c_int, [_P]),
    "mirt_box_set_strip": (C.c_int, [_P, C.c_uint32]),
    "mirt_box_set_options": (C.c_int, [_P, C.c_uint32]),
    "mirt_box_mesh_upload": (C.c_int, [_P, _P, C.c_uint32, _P, C.c_uint32, _P, _P, _P, C.c_uint32,
                                       C.POINTER(Material), C.c_uint32, C.POINTER(C.c_uint32)]),
    "mirt_box_mesh_release": (C.c_int, [_P, C.c_uint32]),
    "mirt_box_trace_tile": (C.c_int, [_P, C.POINTER(Frame), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_uint32, C.POINTER(Outputs), _P, C.POINTER(Stats)]),
}
MIRT_BOX_RCCL, MIRT_BOX_COPY, MIRT_BOX_HOST = 1, 2, 3

_lib = None


def lib() -> C.CDLL:
    """Load libmirt.so (built in-tree by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever
        # is loaded first serves the whole process, so load torch's first when torch is
        # installed: one HIP runtime per process, and torch stream handles passed to
        # mirt_trace_tiles_async are valid in libmirt.  A Go/C caller without torch gets
        # /opt/rocm's runtime through libmirt's RUNPATH.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: the HIP trace worker is not built. Run "
                f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
                f"There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("MIRT_LIB") and not hasattr(L, name):
                continue  # an older build under A/B (MIRT_LIB): entries it lacks stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != MIRT_OK:
        msg = lib().mirt_last_error()
        raise MirtError(rc, msg.decode() if msg else "")
