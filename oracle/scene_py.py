"""Pure-Python scene.json / OBJ / MTL loader — TEST INFRASTRUCTURE ONLY.

Independent restatement of the reference's loader, used to feed the oracle and to
cross-check the product's C++ loader (distributed_raytracer_amd/csrc/scene.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import it.

Follows (reference paths):
  shared/state/environment.go:162-234  EnvironmentFromFile (objects get id i+1, lights
                                       NewRGB(u8)/255, camera via NewCamera)
  shared/state/mesh.go:109-213         MeshFromFile (float32 coords widened to f64, vertex
                                       dedupe by exact value, normal dedupe by un-normalised
                                       value stored normalised, per-usemtl material)
  shared/state/util.go:11-13           relativePath
  shared/colour/colour.go:28-35        NewRGB / NewRGBFromFloats (clamp of float64(f32))
Third-party semantics assumed (github.com/mwindels/gwob, unpinned, not vendored):
  coordinates parsed as float32 by strconv.ParseFloat(s, 32) (one correct rounding); polygon faces fan-triangulated (v0, vi, vi+1);
  material per face = the last `usemtl` before it; MTL Ka/Kd/Ks/Ns parsed as float32.
Go's encoding/json matches object keys to struct fields case-insensitively.
"""
from __future__ import annotations

import json
import math
import os
from fractions import Fraction
from dataclasses import dataclass, field

import numpy as np

DEFAULT_MATERIAL = (16 / 255, 16 / 255, 16 / 255, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0)  # mesh.go:151


def _f32(s: str) -> float:
    """The decimal string rounded ONCE, correctly, to float32 (Go's strconv.ParseFloat(s, 32),
    which gwob uses), widened to float64.  float32(float64(s)) rounds twice and differs when
    the decimal lies within half a float64 ulp of a float32 halfway point; those rare cases
    are decided exactly."""
    f = float(s)
    r = np.float32(f)
    if float(r) == f or not math.isfinite(f):
        return float(r)
    nb = np.nextafter(r, np.float32(np.inf) if f > float(r) else np.float32(-np.inf))
    mid = (float(r) + float(nb)) / 2  # exact in float64
    if abs(f - mid) > math.ulp(f):
        return float(r)  # the exact value is on f's side of the halfway point
    q = Fraction(s.strip())
    best = None
    for c in (np.nextafter(r, np.float32(-np.inf)), r, np.nextafter(r, np.float32(np.inf))):
        d = abs(Fraction(float(c)) - q)
        if best is None or d < best[0] or (d == best[0] and int(np.float32(c).view(np.uint32)) & 1 == 0):
            best = (d, c)
    return float(best[1])


def _clamp01(v: float) -> float:
    # colour.go:33-35 NewRGBFromFloats: Max(0, Min(float64(f), 1))
    if math.isnan(v):
        return v
    return max(0.0, min(v, 1.0))


def relative_path(original: str, other: str) -> str:
    """util.go:11-13: dirname-with-separator of `original` + `other` without leading seps."""
    i = len(original)
    while i > 0 and original[i - 1] not in "/\\":
        i -= 1
    return original[:i] + other.lstrip("/\\")


@dataclass
class PyMesh:
    vertices: np.ndarray   # (nv, 3) f64
    normals: np.ndarray    # (nn, 3) f64 (normalised); nn may be 0
    face_v: np.ndarray     # (nf, 3) u32
    face_n: np.ndarray     # (nf, 3) u32
    face_mat: np.ndarray   # (nf,)  u32
    materials: np.ndarray  # (nm, 10) f64: ka[3] kd[3] ks[3] ns


@dataclass
class PyScene:
    meshes: list = field(default_factory=list)
    objects: list = field(default_factory=list)   # (mesh_index, (x, y, z))
    lights: list = field(default_factory=list)    # ((x, y, z), (r, g, b) f64)
    cam_pos: tuple = (0.0, 0.0, 0.0)
    cam_dir: tuple = (0.0, 0.0, -1.0)
    fov: float = 0.0


def _parse_mtl(path: str) -> dict:
    lib, cur = {}, None
    with open(path, "r") as fh:
        for raw in fh:
            p = raw.split()
            if not p or p[0].startswith("#"):
                continue
            if p[0] == "newmtl":
                cur = {"Ka": (0.0, 0.0, 0.0), "Kd": (0.0, 0.0, 0.0), "Ks": (0.0, 0.0, 0.0), "Ns": 0.0}
                lib[" ".join(p[1:])] = cur
            elif cur is not None and p[0] in ("Ka", "Kd", "Ks") and len(p) >= 4:
                cur[p[0]] = tuple(_f32(x) for x in p[1:4])
            elif cur is not None and p[0] == "Ns" and len(p) >= 2:
                cur["Ns"] = _f32(p[1])
    return lib


def _resolve(idx: str, count: int) -> int:
    i = int(idx)
    return i - 1 if i > 0 else count + i


def load_mesh(path: str) -> PyMesh:
    pos, nrm = [], []
    mtllib = ""
    cur_mtl = ""
    tris = []  # ((vi, ni) x3, mtl name)
    with open(path, "r") as fh:
        for raw in fh:
            p = raw.split()
            if not p or p[0].startswith("#"):
                continue
            tag = p[0]
            if tag == "v":
                pos.append(tuple(_f32(x) for x in p[1:4]))
            elif tag == "vn":
                nrm.append(tuple(_f32(x) for x in p[1:4]))
            elif tag == "mtllib":
                mtllib = " ".join(p[1:])
            elif tag == "usemtl":
                cur_mtl = " ".join(p[1:])
            elif tag == "f":
                corners = []
                for tok in p[1:]:
                    parts = tok.split("/")
                    vi = _resolve(parts[0], len(pos))
                    ni = _resolve(parts[2], len(nrm)) if len(parts) >= 3 and parts[2] else -1
                    corners.append((vi, ni))
                for k in range(1, len(corners) - 1):
                    tris.append(((corners[0], corners[k], corners[k + 1]), cur_mtl))
    lib = {}
    if mtllib:
        try:
            lib = _parse_mtl(relative_path(path, mtllib))
        except OSError:
            lib = _parse_mtl(mtllib)
    has_normals = len(nrm) > 0
    vmap, nmap, mmap = {}, {}, {}
    vertices, normals, materials = [], [], []
    face_v, face_n, face_mat = [], [], []
    for corners, mname in tris:
        if mname in lib:
            m = lib[mname]
            mat = tuple(_clamp01(x) for x in m["Ka"]) + tuple(_clamp01(x) for x in m["Kd"]) + \
                tuple(_clamp01(x) for x in m["Ks"]) + (m["Ns"],)
        else:
            mat = DEFAULT_MATERIAL
        if mat not in mmap:
            mmap[mat] = len(materials)
            materials.append(mat)
        fv, fn = [], []
        for vi, ni in corners:
            v = pos[vi]
            if v not in vmap:
                vmap[v] = len(vertices)
                vertices.append(v)
            fv.append(vmap[v])
            if has_normals:
                n = nrm[ni] if ni >= 0 else (0.0, 0.0, 0.0)
                if n not in nmap:
                    nmap[n] = len(normals)
                    mag = math.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2])
                    normals.append((n[0] / mag if mag else math.nan, n[1] / mag if mag else math.nan,
                                    n[2] / mag if mag else math.nan))
                fn.append(nmap[n])
            else:
                fn.append(0)
        face_v.append(fv)
        face_n.append(fn)
        face_mat.append(mmap[mat])
    return PyMesh(
        vertices=np.array(vertices, dtype=np.float64).reshape(-1, 3),
        normals=np.array(normals, dtype=np.float64).reshape(-1, 3),
        face_v=np.array(face_v, dtype=np.uint32).reshape(-1, 3),
        face_n=np.array(face_n, dtype=np.uint32).reshape(-1, 3),
        face_mat=np.array(face_mat, dtype=np.uint32),
        materials=np.array(materials, dtype=np.float64).reshape(-1, 10),
    )


def _ci(d: dict, key: str):
    for k, v in d.items():
        if k.lower() == key.lower():
            return v
    return None


def _vec(d) -> tuple:
    d = d or {}
    return tuple(float(_ci(d, c) or 0.0) for c in ("x", "y", "z"))


def load_scene(path: str) -> PyScene:
    with open(path, "r") as fh:
        doc = json.load(fh)
    sc = PyScene()
    by_model = {}
    for o in _ci(doc, "objs") or []:
        model = _ci(o, "model")
        if model not in by_model:
            try:
                mesh = load_mesh(relative_path(path, model))
            except OSError:
                mesh = load_mesh(model)
            by_model[model] = len(sc.meshes)
            sc.meshes.append(mesh)
        sc.objects.append((by_model[model], _vec(_ci(o, "pos"))))
    for lt in _ci(doc, "lights") or []:
        col = _ci(lt, "col") or {}
        sc.lights.append((_vec(_ci(lt, "pos")), tuple(int(_ci(col, c) or 0) / 255.0 for c in ("r", "g", "b"))))
    cam = _ci(doc, "cam") or {}
    sc.cam_pos = _vec(_ci(cam, "pos"))
    sc.cam_dir = _vec(_ci(cam, "dir"))
    sc.fov = float(_ci(cam, "fov") or 0.0)
    return sc
