"""Host-side mirror of the reference's trace interfaces, over libmirt.so.

Reference interface                                  here
-------------------------------------------------    -----------------------------------
state.EnvironmentFromFile (environment.go:162)       Environment.from_file(path, ctx)
state.EnvMutables (environment.go:65-69)             EnvMutables (objects, lights, cam)
state.NewCamera (camera.go:35-44)                    Camera.new(pos, dir, fov)
tracer.Trace(i, j, w, h, env) (tracer.go:81-91)      trace(i, j, w, h, env) -> (RGB, bool)
tracer.trace(o, d, env) (tracer.go:27-50)            trace_rays(origins, dirs, env)
Tracer.BulkTrace(ctx, WorkOrder)                     Tracer.bulk_trace(WorkOrder)
  (worker/distributed/main.go:46-91)                   -> TraceResults (column-major u8)
Tracer.Heartbeat (worker/distributed/main.go:94)     Tracer.heartbeat()
draw (worker/sequential/main.go:15-32)               draw(env, W, H) -> Framebuffer
colour.RGB / .RGB() / .RGBA() (colour.go:16-61)      RGB, RGB.rgb(), RGB.rgba()

Every pixel is traced by the HIP kernels; there is no CPU path.  Errors surface as
MirtError (the reference returns Go errors; NewCamera's parallel-dir error maps to
MIRT_E_CAMERA, a cancelled BulkTrace to MIRT_E_CANCELLED).
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

Vec = Tuple[float, float, float]


def _d3(v) -> L.D3:
    return L.D3(float(v[0]), float(v[1]), float(v[2]))


# --------------------------------------------------------------------- colour
@dataclass(frozen=True)
class RGB:
    """colour.RGB (colour.go:16-18): channels in [0, 1] as fp64."""
    r: float = 0.0
    g: float = 0.0
    b: float = 0.0

    def rgb(self) -> Tuple[int, int, int]:
        """colour.go:59-61: uint8(255 * c), truncating."""
        return int(255 * self.r) & 0xFF, int(255 * self.g) & 0xFF, int(255 * self.b) & 0xFF

    def rgba(self) -> Tuple[int, int, int, int]:
        """colour.go:54-56: uint32(0xFFFF * c), alpha 0xFFFF."""
        return int(0xFFFF * self.r), int(0xFFFF * self.g), int(0xFFFF * self.b), 0xFFFF


def _upload_mesh(fn, handle, vertices, normals, face_v, face_n, face_mat, materials) -> int:
    """mirt_mesh_upload / mirt_box_mesh_upload: one mesh from numpy arrays; returns its id."""
    v = np.ascontiguousarray(vertices, np.float64).reshape(-1, 3)
    vn = np.ascontiguousarray(normals, np.float64).reshape(-1, 3)
    fv = np.ascontiguousarray(face_v, np.uint32).reshape(-1, 3)
    fn_ = np.ascontiguousarray(face_n, np.uint32).reshape(-1, 3)
    fm = np.ascontiguousarray(face_mat, np.uint32).reshape(-1)
    mats = np.ascontiguousarray(materials, np.float64).reshape(-1, 10)
    marr = (L.Material * max(1, len(mats)))()
    for i, m in enumerate(mats):
        marr[i] = L.Material(_d3(m[0:3]), _d3(m[3:6]), _d3(m[6:9]), float(m[9]))
    mid = C.c_uint32()
    L.check(fn(handle, v.ctypes.data if len(v) else None, len(v), vn.ctypes.data if len(vn) else None, len(vn),
               fv.ctypes.data if len(fv) else None, fn_.ctypes.data if len(fn_) else None,
               fm.ctypes.data if len(fm) else None, len(fm), marr, len(mats), C.byref(mid)))
    return mid.value


# --------------------------------------------------------------------- context
class Context:
    """One libmirt context bound to one HIP device (one process per GPU)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        L.check(L.lib().mirt_create(int(device), C.byref(self._h)))
        self.device = device
        self._lock = threading.Lock()
        self._streams = []  # mirt_stream_create handles, destroyed by close()

    @property
    def handle(self) -> C.c_void_p:
        if not self._h:
            raise L.MirtError(L.MIRT_E_INVALID, "context destroyed")
        return self._h

    def close(self) -> None:
        if self._h:
            for s in self._streams:
                L.lib().mirt_stream_destroy(self._h, C.c_void_p(s))
            self._streams = []
            L.lib().mirt_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _trace_tile_call(self):
        """(C entry, handle) that trace_tile calls: a Context traces on its GPU."""
        return L.lib().mirt_trace_tile, self.handle

    def upload_mesh(self, vertices, normals, face_v, face_n, face_mat, materials) -> int:
        return _upload_mesh(L.lib().mirt_mesh_upload, self.handle, vertices, normals, face_v, face_n, face_mat,
                            materials)

    def release_mesh(self, mesh_id: int) -> None:
        L.check(L.lib().mirt_mesh_release(self.handle, mesh_id))

    def set_options(self, flags: int) -> None:
        L.check(L.lib().mirt_set_options(self.handle, flags))

    def stream_create(self):
        """A torch stream on a hardware queue of its own (mirt.h mirt_stream_create),
        destroyed with the context."""
        import torch
        p = C.c_void_p()
        L.check(L.lib().mirt_stream_create(self.handle, C.byref(p)))
        self._streams.append(p.value)
        return torch.cuda.ExternalStream(p.value, device=torch.device("cuda", self.device))

    def set_grid(self, min_blocks_per_wg: int = 32, max_workgroups: int = 0) -> None:
        """Frame-kernel launch shape (mirt.h mirt_set_grid); results never change."""
        L.check(L.lib().mirt_set_grid(self.handle, min_blocks_per_wg, max_workgroups))

    def profile_enable(self, on: bool) -> None:
        L.check(L.lib().mirt_profile_enable(self.handle, 1 if on else 0))

    def profile_read(self) -> dict:
        p = L.Profile()
        L.check(L.lib().mirt_profile_read(self.handle, C.byref(p)))
        return {k: getattr(p, k) for k, _ in L.Profile._fields_}

    def debug_fp64(self, op: int, a, b) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        out = np.zeros_like(a)
        L.check(L.lib().mirt_debug_fp64(self.handle, op, len(a), a.ctypes.data, b.ctypes.data, out.ctypes.data))
        return out

    def light_cache_stats(self) -> dict:
        """mirt_light_cache_stats: the light-table cache's counters (mirt.h)."""
        if not hasattr(L.lib(), "mirt_light_cache_stats"):
            return {}  # an older build under A/B (MIRT_LIB)
        out = np.zeros(8, np.uint64)
        L.check(L.lib().mirt_light_cache_stats(self.handle, out.ctypes.data))
        return dict(zip(("builds", "hits", "evictions", "no_room", "reused_buffers", "tables", "bytes", "cap"),
                        (int(x) for x in out)))

    def set_light_cache(self, max_bytes: int) -> None:
        L.check(L.lib().mirt_set_light_cache(self.handle, int(max_bytes)))

    def debug_box_intersect(self, origins, dirs, boxes) -> np.ndarray:
        """box.go:29-68 Box.Intersect as the kernels evaluate it (mirt_debug_fp64 op 4):
        ray i (origins[i], dirs[i]) against box i ({MinCorner, MaxCorner}, 6 doubles)."""
        rays = np.ascontiguousarray(np.concatenate([np.reshape(origins, (-1, 3)), np.reshape(dirs, (-1, 3))], 1),
                                    np.float64)
        bx = np.ascontiguousarray(np.reshape(boxes, (-1, 6)), np.float64)
        assert len(rays) == len(bx)
        out = np.zeros(len(rays), np.float64)
        L.check(L.lib().mirt_debug_fp64(self.handle, 4, len(rays), rays.ctypes.data, bx.ctypes.data, out.ctypes.data))
        return out != 0.0

    def debug_timeline(self, max_records: int = 1 << 16) -> np.ndarray:
        """Per-wave stamps of the last frame traced with MIRT_OPT_TIMELINE (mirt.h)."""
        out = np.zeros((max_records, 8), np.uint64)
        n = L.lib().mirt_debug_timeline(self.handle, out.ctypes.data, max_records)
        L.check(min(n, 0))
        return out[:n]

    def debug_counters(self) -> np.ndarray:
        """Wave-level event counts of a -DMIRT_DIAG=1 build since the last call (mirt.h)."""
        out = np.zeros(32, np.uint64)
        L.check(L.lib().mirt_debug_counters(self.handle, out.ctypes.data, 32))
        return out


# --------------------------------------------------------------------- scene
class Box:
    """One process driving several GPUs behind BulkTrace (mirt.h mirt_box_*): an order is cut
    into `strip`-px column strips dealt round robin over the devices and assembled on the first
    (RCCL over xGMI, device copies when devices repeat, or per-device D2H).  It serves orders:
    Environment.from_file / from_gob, trace_tile, draw, Tracer.bulk_trace.  It is NOT a Context:
    every per-device call (trace_rays, frame groups, light cache, profiling) raises
    MIRT_E_INVALID on a Box (its handle is a mirt_box, never a mirt_ctx); use box.entry(i) for
    those.  Entries may repeat a device, so one GPU can stand in for a box."""

    def __init__(self, devices: Sequence[int]):
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        self._bh = C.c_void_p()
        L.check(L.lib().mirt_box_create(devs, len(devices), C.byref(self._bh)))
        self.devices = [int(d) for d in devices]
        self.device = self.devices[0]
        self._lock = threading.Lock()

    @property
    def box_handle(self) -> C.c_void_p:
        if not self._bh:
            raise L.MirtError(L.MIRT_E_INVALID, "box destroyed")
        return self._bh

    @property
    def handle(self) -> C.c_void_p:
        """A Box has no mirt_ctx handle: per-device entry points fail cleanly, never on a mirt_box."""
        raise L.MirtError(L.MIRT_E_INVALID, "a Box serves orders (trace_tile / draw / bulk_trace); "
                                            "use box.entry(i) for per-device calls")

    def close(self) -> None:
        if self._bh:
            L.lib().mirt_box_destroy(self._bh)
            self._bh = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _trace_tile_call(self):
        return L.lib().mirt_box_trace_tile, self.box_handle

    def upload_mesh(self, vertices, normals, face_v, face_n, face_mat, materials) -> int:
        return _upload_mesh(L.lib().mirt_box_mesh_upload, self.box_handle, vertices, normals, face_v, face_n,
                            face_mat, materials)

    def release_mesh(self, mesh_id: int) -> None:
        L.check(L.lib().mirt_box_mesh_release(self.box_handle, mesh_id))

    def set_options(self, flags: int) -> None:
        L.check(L.lib().mirt_box_set_options(self.box_handle, flags))

    @property
    def transport(self) -> int:
        return int(L.lib().mirt_box_transport(self.box_handle))

    def set_transport(self, transport: int) -> None:
        L.check(L.lib().mirt_box_set_transport(self.box_handle, int(transport)))

    def set_strip(self, strip: int) -> None:
        L.check(L.lib().mirt_box_set_strip(self.box_handle, int(strip)))

    def entry(self, i: int) -> "Context":
        """Entry i's context (profiling, light-cache statistics), owned by the box."""
        h = L.lib().mirt_box_ctx(self.box_handle, int(i))
        if not h:
            raise L.MirtError(L.MIRT_E_INVALID, f"no box entry {i}")
        c = Context.__new__(Context)
        c._h, c.device, c._lock, c._streams = C.c_void_p(h), self.devices[i], threading.Lock(), []
        c.close = lambda: None  # the box destroys its entries
        return c


@dataclass
class Camera:
    """state.Camera (camera.go:20-24) as NewCamera builds it, plus tan(fov/2)."""
    pos: Vec
    forward: Vec
    left: Vec
    up: Vec
    fov: float
    proj_half_width: float

    @staticmethod
    def new(pos: Sequence[float], direction: Sequence[float], fov: float) -> "Camera":
        c = L.Camera()
        p = (C.c_double * 3)(*map(float, pos))
        d = (C.c_double * 3)(*map(float, direction))
        L.check(L.lib().mirt_camera_init(p, d, float(fov), C.byref(c)))
        return Camera._from_c(c)

    @staticmethod
    def _from_c(c: L.Camera) -> "Camera":
        return Camera(tuple(c.pos), tuple(c.forward), tuple(c.left), tuple(c.up), c.fov, c.proj_half_width)

    def to_c(self) -> L.Camera:
        return L.Camera(_d3(self.pos), _d3(self.forward), _d3(self.left), _d3(self.up), float(self.fov),
                        float(self.proj_half_width))


@dataclass
class Light:
    pos: Vec
    col: Vec  # fp64 channels (NewRGB(u8)/255)


@dataclass
class SceneObject:
    mesh_id: int
    pos: Vec


@dataclass
class EnvMutables:
    """state.EnvMutables: the per-frame part (WorkOrder.diff)."""
    objects: List[SceneObject] = field(default_factory=list)
    lights: List[Light] = field(default_factory=list)
    cam: Optional[Camera] = None
    max_bounces: int = 0  # configs[4] reflection EXTENSION (mirt.h); 0 = the reference

    def to_frame(self) -> Tuple[L.Frame, list]:
        """C mirt_frame; the second value keeps the arrays alive for the call."""
        if self.cam is None:
            raise L.MirtError(L.MIRT_E_INVALID, "EnvMutables has no camera")
        objs = (L.Object * max(1, len(self.objects)))()
        for i, o in enumerate(self.objects):
            objs[i] = L.Object(o.mesh_id, 0, _d3(o.pos))
        lts = (L.Light * max(1, len(self.lights)))()
        for i, lt in enumerate(self.lights):
            lts[i] = L.Light(_d3(lt.pos), _d3(lt.col))
        fr = L.Frame(objs, len(self.objects), lts, len(self.lights), self.cam.to_c(), int(self.max_bounces), 0)
        return fr, [objs, lts]


@dataclass
class MeshArrays:
    vertices: np.ndarray
    normals: np.ndarray
    face_v: np.ndarray
    face_n: np.ndarray
    face_mat: np.ndarray
    materials: np.ndarray  # (nm, 10)


def _scene_meshes(h) -> List[MeshArrays]:
    lib = L.lib()
    meshes = []
    for i in range(lib.mirt_scene_mesh_count(h)):
        mv = L.MeshView()
        L.check(lib.mirt_scene_mesh(h, i, C.byref(mv)))

        def arr(ptr, n, dt):
            if n == 0 or not ptr:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)

        mats = np.zeros((mv.n_materials, 10))
        for k in range(mv.n_materials):
            m = mv.materials[k]
            mats[k] = list(m.ka) + list(m.kd) + list(m.ks) + [m.ns]
        meshes.append(MeshArrays(
            vertices=arr(mv.vertices, 3 * mv.n_vertices, np.float64).reshape(-1, 3),
            normals=arr(mv.normals, 3 * mv.n_normals, np.float64).reshape(-1, 3),
            face_v=arr(mv.face_v, 3 * mv.n_faces, np.uint32).reshape(-1, 3),
            face_n=arr(mv.face_n, 3 * mv.n_faces, np.uint32).reshape(-1, 3),
            face_mat=arr(mv.face_mat, mv.n_faces, np.uint32),
            materials=mats))
    return meshes


def _scene_mutables(h) -> Tuple[List[Tuple[int, Vec]], List[Light], Camera]:
    lib = L.lib()
    objects = []
    for i in range(lib.mirt_scene_object_count(h)):
        o = L.Object()
        L.check(lib.mirt_scene_object(h, i, C.byref(o)))
        objects.append((o.mesh_id, tuple(o.pos)))
    lights = []
    for i in range(lib.mirt_scene_light_count(h)):
        lt = L.Light()
        L.check(lib.mirt_scene_light(h, i, C.byref(lt)))
        lights.append(Light(tuple(lt.pos), tuple(lt.col)))
    cam = L.Camera()
    L.check(lib.mirt_scene_camera(h, C.byref(cam)))
    return objects, lights, Camera._from_c(cam)


def _scene_error(rc: int):
    return L.MirtError(rc, (L.lib().mirt_scene_last_error() or b"").decode())


def load_scene_arrays(path: str) -> Tuple[List[MeshArrays], List[Tuple[int, Vec]], List[Light], Camera]:
    """Parse scene.json + OBJ/MTL with the library's C++ loader (mirt_scene_load)."""
    lib = L.lib()
    h = C.c_void_p()
    rc = lib.mirt_scene_load(path.encode(), C.byref(h))
    if rc != L.MIRT_OK:
        raise _scene_error(rc)
    try:
        return (_scene_meshes(h),) + _scene_mutables(h)
    finally:
        lib.mirt_scene_free(h)


class Environment:
    """state.Environment: immutable meshes resident on the device + the mutable part."""

    def __init__(self, ctx: Context, mesh_ids: List[int], mutable: Optional[EnvMutables], meshes: List[MeshArrays],
                 gob_scene=None):
        self.ctx = ctx
        self.mesh_ids = mesh_ids
        self._mutable = mutable
        self.meshes = meshes
        self._gob = gob_scene  # mirt_scene handle of a gob environment (mirt_scene_link_gob)

    @classmethod
    def from_file(cls, path: str, ctx: Context) -> "Environment":
        meshes, objects, lights, cam = load_scene_arrays(path)
        ids = [ctx.upload_mesh(m.vertices, m.normals, m.face_v, m.face_n, m.face_mat, m.materials) for m in meshes]
        mut = EnvMutables([SceneObject(ids[mi], pos) for mi, pos in objects], lights, cam)
        return cls(ctx, ids, mut, meshes)

    @classmethod
    def from_gob(cls, state: bytes, ctx: Context) -> "Environment":
        """worker/distributed/main.go:118-126: the Register reply's MasterState.state (a gob
        state.Environment) decoded by the library (mirt_scene_from_gob); meshes uploaded.
        It has no mutable part until a WorkOrder diff is linked (link_gob)."""
        lib = L.lib()
        h = C.c_void_p()
        rc = lib.mirt_scene_from_gob(bytes(state), len(state), C.byref(h))
        if rc != L.MIRT_OK:
            raise _scene_error(rc)
        try:
            meshes = _scene_meshes(h)
            ids = [ctx.upload_mesh(m.vertices, m.normals, m.face_v, m.face_n, m.face_mat, m.materials) for m in meshes]
        except Exception:
            lib.mirt_scene_free(h)
            raise
        return cls(ctx, ids, None, meshes, gob_scene=h)

    def link_gob(self, diff: bytes) -> EnvMutables:
        """worker/distributed/main.go:56-64: decode a WorkOrder.diff (gob state.EnvMutables)
        and LinkTo this environment.  Objects whose id links to no mesh are dropped (a nil
        mesh is never hit, object.go:73-74)."""
        if self._gob is None:
            raise L.MirtError(L.MIRT_E_INVALID, "link_gob needs an environment made by from_gob")
        lib = L.lib()
        h = C.c_void_p()
        rc = lib.mirt_scene_link_gob(self._gob, bytes(diff), len(diff), C.byref(h))
        if rc != L.MIRT_OK:
            raise _scene_error(rc)
        try:
            objects, lights, cam = _scene_mutables(h)
        finally:
            lib.mirt_scene_free(h)
        return EnvMutables([SceneObject(self.mesh_ids[mi], pos) for mi, pos in objects if mi != L.MIRT_NO_MESH],
                           lights, cam)

    def mutable(self) -> EnvMutables:
        if self._mutable is None:
            raise L.MirtError(L.MIRT_E_INVALID, "a gob environment has no mutable part: link a diff (link_gob)")
        return self._mutable

    def __del__(self):
        if getattr(self, "_gob", None) is not None:
            try:
                L.lib().mirt_scene_free(self._gob)
            except Exception:  # noqa: BLE001 — interpreter shutdown
                pass
            self._gob = None


# --------------------------------------------------------------------- tracing
@dataclass
class TileResult:
    """Planes of one traced tile, column-major: pixel (x+i, y+j) at i*h + j."""
    rgb: np.ndarray    # (w*h, 3) f64
    rgb8: np.ndarray   # (w*h, 3) u8
    valid: np.ndarray  # (w*h,)  u8
    face: np.ndarray   # (w*h,)  i32
    obj: np.ndarray    # (w*h,)  i32
    stats: dict


def trace_tile(env: Environment, x: int, y: int, w: int, h: int, W: int, H: int,
               mut: Optional[EnvMutables] = None, cancel: Optional[C.c_int] = None) -> TileResult:
    mut = mut or env.mutable()
    fr, keep = mut.to_frame()
    n = w * h
    rgb = np.zeros((n, 3), np.float64)
    rgb8 = np.zeros((n, 3), np.uint8)
    valid = np.zeros(n, np.uint8)
    face = np.zeros(n, np.int32)
    obj = np.zeros(n, np.int32)
    out = L.Outputs(rgb.ctypes.data, rgb8.ctypes.data, valid.ctypes.data, face.ctypes.data, obj.ctypes.data)
    st = L.Stats()
    # a Context traces the tile on its GPU; a Box deals it over the box's GPUs (mirt_box_trace_tile)
    fn, handle = env.ctx._trace_tile_call()
    L.check(fn(handle, C.byref(fr), x, y, w, h, W, H, C.byref(out), C.byref(cancel) if cancel is not None else None,
               C.byref(st)))
    del keep
    return TileResult(rgb, rgb8, valid, face, obj, {k: getattr(st, k) for k, _ in L.Stats._fields_})


def trace(i: int, j: int, width: int, height: int, env: Environment) -> Tuple[RGB, bool]:
    """tracer.Trace (tracer.go:81-91) for one pixel (a 1x1 tile on the GPU)."""
    r = trace_tile(env, i, j, 1, 1, width, height)
    if r.valid[0]:
        return RGB(*map(float, r.rgb[0])), True
    return RGB(), False


def trace_rays(origins: np.ndarray, dirs: np.ndarray, env: Environment, mut: Optional[EnvMutables] = None) -> dict:
    """tracer.trace (tracer.go:27-50) on arbitrary rays: nearest hit by |hit - Cam.Pos|."""
    mut = mut or env.mutable()
    fr, keep = mut.to_frame()
    o = np.ascontiguousarray(origins, np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
    n = len(o)
    ok = np.zeros(n, np.uint8)
    hit = np.zeros((n, 3))
    nrm = np.zeros((n, 3))
    face = np.zeros(n, np.int32)
    obj = np.zeros(n, np.int32)
    L.check(L.lib().mirt_trace_rays(env.ctx.handle, C.byref(fr), n, o.ctypes.data, d.ctypes.data, ok.ctypes.data,
                                    hit.ctypes.data, nrm.ctypes.data, face.ctypes.data, obj.ctypes.data))
    del keep
    return dict(ok=ok, hit=hit, normal=nrm, face=face, obj=obj)


@dataclass
class Framebuffer:
    """worker/sequential surface: pixel (i, j) at index i*H + j; misses stay 0."""
    width: int
    height: int
    rgb: np.ndarray
    rgb8: np.ndarray
    valid: np.ndarray
    face: np.ndarray
    obj: np.ndarray
    stats: dict

    def image(self) -> np.ndarray:
        """(H, W, 3) uint8 image, row = y (for viewing; not a reference layout)."""
        return self.rgb8.reshape(self.width, self.height, 3).transpose(1, 0, 2)


def draw(env: Environment, width: int, height: int, mut: Optional[EnvMutables] = None) -> Framebuffer:
    """worker/sequential/main.go:15-32 draw: every pixel of the screen, one GPU call."""
    r = trace_tile(env, 0, 0, width, height, width, height, mut)
    return Framebuffer(width, height, r.rgb, r.rgb8, r.valid, r.face, r.obj, r.stats)


# --------------------------------------------------------------------- BulkTrace
@dataclass
class WorkOrder:
    """comms.WorkOrder (comms.proto:25-31).  diff: the wire bytes (a gob state.EnvMutables,
    decoded and linked as worker/distributed/main.go:56-64 does), an already decoded
    EnvMutables, or None for the registered scene's own state."""
    x: int
    y: int
    width: int
    height: int
    diff: Optional[object] = None


@dataclass
class TraceResults:
    """comms.TraceResults: results[i*height + j] = (r, g, b) as uint8 values."""
    results: np.ndarray  # (width*height, 3) uint8, column-major


class Tracer:
    """worker/distributed Tracer: serves BulkTrace / Heartbeat for one registered scene."""

    def __init__(self, scene: Environment, screen_width: int, screen_height: int):
        self.scene = scene
        self.screen_width = screen_width
        self.screen_height = screen_height

    def bulk_trace(self, req: WorkOrder, cancel: Optional[C.c_int] = None) -> TraceResults:
        diff = self.scene.link_gob(req.diff) if isinstance(req.diff, (bytes, bytearray)) else req.diff
        r = trace_tile(self.scene, req.x, req.y, req.width, req.height, self.screen_width, self.screen_height,
                       diff, cancel)
        return TraceResults(r.rgb8)

    def heartbeat(self) -> None:
        return None
