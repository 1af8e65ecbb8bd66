"""ctypes wrapper around oracle/librt_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  Parity status: unpinned by the reference (see rt_oracle.c header).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .scene_py import PyScene

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OrMesh(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("n_vertices", C.c_uint32),
                ("normals", C.c_void_p), ("n_normals", C.c_uint32),
                ("face_v", C.c_void_p), ("face_n", C.c_void_p), ("face_mat", C.c_void_p),
                ("n_faces", C.c_uint32),
                ("materials", C.c_void_p), ("n_materials", C.c_uint32)]


class OrObject(C.Structure):
    _fields_ = [("mesh", C.c_uint32), ("_pad", C.c_uint32), ("pos", C.c_double * 3)]


class OrLight(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("col", C.c_double * 3)]


class OrScene(C.Structure):
    _fields_ = [("meshes", C.POINTER(OrMesh)), ("n_meshes", C.c_uint32),
                ("objects", C.POINTER(OrObject)), ("n_objects", C.c_uint32),
                ("lights", C.POINTER(OrLight)), ("n_lights", C.c_uint32),
                ("cam_pos", C.c_double * 3), ("cam_dir", C.c_double * 3), ("fov", C.c_double)]


class OrTile(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("w", C.c_uint32), ("h", C.c_uint32)]


class OrStats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("hits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("box_tests", C.c_uint64), ("reflection_rays", C.c_uint64)]


def build() -> str:
    """Compile the oracle with its committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "librt_oracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "librt_oracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_build.restype = C.c_void_p
        L.or_build.argtypes = [C.POINTER(OrScene), C.c_int]
        L.or_free.argtypes = [C.c_void_p]
        L.or_set_bounces.argtypes = [C.c_void_p, C.c_int]
        L.or_camera_ok.argtypes = [C.c_void_p]
        L.or_trace_tiles.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(OrTile), C.c_uint32, C.c_int,
                                     C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.POINTER(OrStats)]
        L.or_trace_rays.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_rtree_audit.argtypes = [C.c_void_p, C.c_uint32] + [C.c_void_p] * 4
        L.or_face_box.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        L.or_object_box.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.or_box_intersect.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_triangle_intersection.argtypes = [C.c_void_p] * 7
        L.or_go_tan.restype = C.c_double
        L.or_go_tan.argtypes = [C.c_double]
        L.or_go_pow.restype = C.c_double
        L.or_go_pow.argtypes = [C.c_double, C.c_double]
        L.or_new_camera.argtypes = [C.c_void_p] * 5
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


CULL_MODES = {"brute": 0, "rtree": 1, "boxes": 2}


class Oracle:
    """Holds the C oracle context for one scene.

    culling (rt_oracle.c OR_CULL_*):
      "brute"  every face and object, no box test;
      "rtree"  the reference's rtreego search (object.go:76, tracer.go:32), DFS order;
      "boxes"  every face / object gated by Box.Intersect on its own padded box only —
               the reference's leaf-level test without rtreego's inner nodes; the set the
               GPU computes.
    use_rtree=True is the old spelling of culling="rtree"."""

    def __init__(self, scene: PyScene, use_rtree: bool = False, culling: str | None = None):
        if culling is None:
            culling = "rtree" if use_rtree else "brute"
        self.culling = culling
        self._keep = []
        L = lib()
        meshes = (OrMesh * max(1, len(scene.meshes)))()
        for i, m in enumerate(scene.meshes):
            arrs = [np.ascontiguousarray(m.vertices, np.float64), np.ascontiguousarray(m.normals, np.float64),
                    np.ascontiguousarray(m.face_v, np.uint32), np.ascontiguousarray(m.face_n, np.uint32),
                    np.ascontiguousarray(m.face_mat, np.uint32), np.ascontiguousarray(m.materials, np.float64)]
            self._keep.extend(arrs)
            meshes[i] = OrMesh(_ptr(arrs[0]), len(arrs[0]), _ptr(arrs[1]), len(arrs[1]), _ptr(arrs[2]),
                               _ptr(arrs[3]), _ptr(arrs[4]), len(arrs[2]), _ptr(arrs[5]), len(arrs[5]))
        objs = (OrObject * max(1, len(scene.objects)))()
        for i, (mi, pos) in enumerate(scene.objects):
            objs[i] = OrObject(mi, 0, (C.c_double * 3)(*pos))
        lights = (OrLight * max(1, len(scene.lights)))()
        for i, (pos, col) in enumerate(scene.lights):
            lights[i] = OrLight((C.c_double * 3)(*pos), (C.c_double * 3)(*col))
        self._sc = OrScene(meshes, len(scene.meshes), objs, len(scene.objects), lights, len(scene.lights),
                           (C.c_double * 3)(*scene.cam_pos), (C.c_double * 3)(*scene.cam_dir), scene.fov)
        self._keep.extend([meshes, objs, lights])
        self._ctx = L.or_build(C.byref(self._sc), CULL_MODES[culling])
        if not L.or_camera_ok(self._ctx):
            raise ValueError("camera dir is parallel to the global up vector (camera.go:37)")

    def close(self):
        if self._ctx:
            lib().or_free(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_bounces(self, bounces: int) -> None:
        """configs[4] reflection extension (rt_oracle.c shade_reflect); 0 = the reference."""
        lib().or_set_bounces(self._ctx, int(bounces))

    def trace_tiles(self, W: int, H: int, tiles, nthreads: int = 1, shade: bool = True):
        """Returns dict(valid, rgb, rgb8, face, obj, stats) with outputs packed per tile,
        column-major inside each tile (worker/distributed/main.go:82)."""
        tl = (OrTile * len(tiles))(*[OrTile(*t) for t in tiles])
        n = sum(t[2] * t[3] for t in tiles)
        valid = np.zeros(n, np.uint8)
        rgb = np.zeros((n, 3), np.float64)
        rgb8 = np.zeros((n, 3), np.uint8)
        face = np.zeros(n, np.int32)
        obj = np.zeros(n, np.int32)
        st = OrStats()
        rc = lib().or_trace_tiles(self._ctx, W, H, tl, len(tiles), nthreads, 1 if shade else 0, _ptr(valid),
                                  _ptr(rgb), _ptr(rgb8), _ptr(face), _ptr(obj), C.byref(st))
        if rc != 0:
            raise RuntimeError("oracle trace failed")
        stats = {k: getattr(st, k) for k, _ in OrStats._fields_}
        return dict(valid=valid, rgb=rgb, rgb8=rgb8, face=face, obj=obj, stats=stats)

    def frame(self, W: int, H: int, nthreads: int = 1, shade: bool = True):
        """worker/sequential framebuffer: one tile (0,0,W,H), pixel (i,j) at index i*H + j."""
        return self.trace_tiles(W, H, [(0, 0, W, H)], nthreads=nthreads, shade=shade)

    def trace_rays(self, origins: np.ndarray, dirs: np.ndarray):
        o = np.ascontiguousarray(origins, np.float64).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
        n = len(o)
        ok = np.zeros(n, np.uint8)
        hit = np.zeros((n, 3), np.float64)
        nrm = np.zeros((n, 3), np.float64)
        face = np.zeros(n, np.int32)
        obj = np.zeros(n, np.int32)
        lib().or_trace_rays(self._ctx, n, _ptr(o), _ptr(d), _ptr(ok), _ptr(hit), _ptr(nrm), _ptr(face), _ptr(obj))
        return dict(ok=ok, hit=hit, normal=nrm, face=face, obj=obj)


    def rtree_audit(self, origins: np.ndarray, dirs: np.ndarray):
        """Per ray (culling="rtree" only): (veto, ties) — candidates rtreego's inner nodes
        prune although their own box passes, and objects with two accepted faces at the same
        minimum distance (rt_oracle.c or_rtree_audit)."""
        o = np.ascontiguousarray(origins, np.float64).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
        veto = np.zeros(len(o), np.uint32)
        ties = np.zeros(len(o), np.uint32)
        if lib().or_rtree_audit(self._ctx, len(o), _ptr(o), _ptr(d), _ptr(veto), _ptr(ties)) != 0:
            raise ValueError("rtree_audit needs culling='rtree'")
        return veto, ties


    def face_box(self, mesh: int, face: int) -> np.ndarray:
        """{MinCorner, MaxCorner} of face.Bounds as NewBox makes them (mesh.go:30-50)."""
        out = np.zeros(6, np.float64)
        if lib().or_face_box(self._ctx, mesh, face, _ptr(out)) != 0:
            raise IndexError("no such face")
        return out

    def object_box(self, obj: int) -> np.ndarray:
        """{MinCorner, MaxCorner} of Object.Bounds as NewBox makes them (object.go:31-59)."""
        out = np.zeros(6, np.float64)
        if lib().or_object_box(self._ctx, obj, _ptr(out)) != 0:
            raise IndexError("no such object")
        return out


def box_intersect(box, origins, dirs) -> np.ndarray:
    """box.go:29-68 Box.Intersect of each ray with a box given as NewBox corners."""
    b = np.ascontiguousarray(box, np.float64)
    o = np.ascontiguousarray(origins, np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
    out = np.zeros(len(o), np.uint8)
    lib().or_box_intersect(_ptr(b), len(o), _ptr(o), _ptr(d), _ptr(out))
    return out.astype(bool)


def triangle_intersection(p1, p2, p3, o, d):
    a = [np.ascontiguousarray(x, np.float64) for x in (p1, p2, p3, o, d)]
    hit = np.zeros(3, np.float64)
    bc = np.zeros(3, np.float64)
    r = lib().or_triangle_intersection(*[_ptr(x) for x in a], _ptr(hit), _ptr(bc))
    return bool(r), hit, bc


def go_tan(x: float) -> float:
    return lib().or_go_tan(x)


def go_pow(x: float, y: float) -> float:
    return lib().or_go_pow(x, y)


def new_camera(pos, direction):
    f = np.zeros(3); l = np.zeros(3); u = np.zeros(3)
    p = np.ascontiguousarray(pos, np.float64); d = np.ascontiguousarray(direction, np.float64)
    rc = lib().or_new_camera(_ptr(p), _ptr(d), _ptr(f), _ptr(l), _ptr(u))
    if rc != 0:
        raise ValueError("camera dir parallel to global up")
    return f, l, u
