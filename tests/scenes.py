"""Synthetic scenes for parity tests (seeded), shared by the oracle and the GPU side."""
from __future__ import annotations

import math

import numpy as np

from oracle.scene_py import DEFAULT_MATERIAL, PyMesh, PyScene


def f32(a):
    return np.asarray(a, np.float64).astype(np.float32).astype(np.float64)


def uv_sphere(stacks: int, slices: int, radius: float = 1.0, with_normals: bool = True,
              material=(0.1, 0.1, 0.1, 0.8, 0.8, 0.8, 0.5, 0.5, 0.5, 10.0)) -> PyMesh:
    """UV sphere, every cell emitted as 2 triangles (pole cells are degenerate, which
    the reference handles via incidence == 0)."""
    verts, norms = [], []
    for i in range(stacks + 1):
        th = math.pi * i / stacks
        for j in range(slices):
            ph = 2 * math.pi * j / slices
            n = (math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph))
            verts.append(tuple(radius * c for c in n))
            norms.append(n)
    V = f32(verts)
    N = f32(norms)
    # vertex dedupe like mesh.go (poles collapse to one vertex)
    key = {}
    vidx = np.zeros(len(V), np.int64)
    uv = []
    for k, v in enumerate(map(tuple, V)):
        if v not in key:
            key[v] = len(uv)
            uv.append(v)
        vidx[k] = key[v]
    nkey = {}
    nidx = np.zeros(len(N), np.int64)
    un = []
    for k, n in enumerate(map(tuple, N)):
        if n not in nkey:
            nkey[n] = len(un)
            mag = math.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2])
            un.append((n[0] / mag, n[1] / mag, n[2] / mag))
        nidx[k] = nkey[n]
    fv, fn = [], []
    for i in range(stacks):
        for j in range(slices):
            a = i * slices + j
            b = i * slices + (j + 1) % slices
            c = (i + 1) * slices + j
            d = (i + 1) * slices + (j + 1) % slices
            for tri in ((a, c, b), (b, c, d)):
                fv.append([vidx[t] for t in tri])
                fn.append([nidx[t] for t in tri])
    nf = len(fv)
    return PyMesh(
        vertices=np.array(uv, np.float64),
        normals=np.array(un, np.float64) if with_normals else np.zeros((0, 3)),
        face_v=np.array(fv, np.uint32),
        face_n=np.array(fn, np.uint32) if with_normals else np.zeros((nf, 3), np.uint32),
        face_mat=np.zeros(nf, np.uint32),
        materials=np.array([material], np.float64),
    )


def box_mesh(size=1.0) -> PyMesh:
    """Axis-aligned cube, no vertex normals (flat Normal() shading), default material."""
    s = size / 2
    V = f32([(x, y, z) for x in (-s, s) for y in (-s, s) for z in (-s, s)])
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    fv = []
    for q in quads:
        fv.append([q[0], q[1], q[2]])
        fv.append([q[0], q[2], q[3]])
    nf = len(fv)
    return PyMesh(vertices=V, normals=np.zeros((0, 3)), face_v=np.array(fv, np.uint32),
                  face_n=np.zeros((nf, 3), np.uint32), face_mat=np.zeros(nf, np.uint32),
                  materials=np.array([DEFAULT_MATERIAL], np.float64))


def multi_object_scene(suzanne: PyMesh) -> PyScene:
    """Two suzannes (one shadowing the other), a flat-shaded cube with the default
    material, and a sphere; four lights; an oblique camera."""
    sc = PyScene()
    sc.meshes = [suzanne, box_mesh(1.5), uv_sphere(12, 24, 0.7)]
    sc.objects = [(0, (1.0, 1.0, -1.0)), (0, (2.2, 1.6, -2.5)), (1, (-0.6, 0.2, -2.0)), (2, (0.4, -0.9, -0.4))]
    sc.lights = [((0.0, 0.0, 10.0), (0.0, 1.0, 0.0)), ((0.0, 10.0, 10.0), (1.0, 0.0, 0.0)),
                 ((5.0, 5.0, 3.0), (100 / 255, 200 / 255, 50 / 255)), ((-4.0, -2.0, 6.0), (0.0, 0.0, 1.0))]
    sc.cam_pos = (2.5, 2.0, 4.0)
    sc.cam_dir = (-0.3, -0.25, -1.0)
    sc.fov = 1.2
    return sc


def gpu_env(ctx, sc: PyScene):
    """Upload a PyScene's meshes and build the matching EnvMutables/Environment."""
    import distributed_raytracer_amd as rt
    ids = [ctx.upload_mesh(m.vertices, m.normals, m.face_v, m.face_n, m.face_mat, m.materials) for m in sc.meshes]
    cam = rt.Camera.new(sc.cam_pos, sc.cam_dir, sc.fov)
    mut = rt.EnvMutables([rt.SceneObject(ids[mi], pos) for mi, pos in sc.objects],
                         [rt.Light(tuple(p), tuple(c)) for p, c in sc.lights], cam)
    return rt.Environment(ctx, ids, mut, [])


def with_camera(scene: PyScene, pos, direction, fov=None) -> PyScene:
    """A shallow copy of `scene` seen from another camera (the oracle takes the camera from
    the scene; the GPU side from rt.Camera.new with the same values)."""
    import copy
    sc = copy.copy(scene)
    sc.cam_pos, sc.cam_dir = tuple(float(x) for x in pos), tuple(float(x) for x in direction)
    if fov is not None:
        sc.fov = float(fov)
    return sc
