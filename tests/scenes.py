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


def triangle_soup(rng, n: int, spread: float = 1.0, with_normals: bool = True, nmat: int = 3) -> PyMesh:
    """A seeded soup of n triangles in float32 vertices (as an OBJ parse gives them):
    mostly small clustered triangles, some sharing a vertex with the previous one, some
    long slivers, collinear and repeated-vertex (zero-area) faces, several materials."""
    verts, fv = [], []

    def vert(p):
        verts.append(p)
        return len(verts) - 1

    for i in range(n):
        c = rng.normal(scale=spread, size=3)
        kind = rng.random()
        if kind < 0.70:
            idx = [vert(c + rng.normal(scale=0.15 * spread, size=3)) for _ in range(3)]
            if fv and rng.random() < 0.3:
                idx[0] = fv[-1][int(rng.integers(3))]  # shared vertex (connected faces)
        elif kind < 0.85:  # sliver
            a = c + rng.normal(scale=0.1 * spread, size=3)
            b = a + rng.normal(scale=spread, size=3)
            idx = [vert(a), vert(b), vert(a + 0.5 * (b - a) + rng.normal(scale=1e-3 * spread, size=3))]
        elif kind < 0.93:  # collinear before the float32 rounding
            a = c
            d = rng.normal(scale=0.3 * spread, size=3)
            idx = [vert(a), vert(a + d), vert(a + 2.5 * d)]
        else:  # a repeated vertex: zero area
            k = vert(c)
            idx = [k, k, vert(c + rng.normal(scale=0.2 * spread, size=3))]
        fv.append(idx)
    V = f32(verts)
    fv = np.array(fv, np.uint32)
    mats = []
    for _ in range(nmat):
        ka = rng.uniform(0, 0.3, 3)
        kd = rng.uniform(0, 1, 3)
        ks = rng.uniform(0, 1, 3) * (rng.random() < 0.7)
        mats.append(tuple(f32(np.concatenate([ka, kd, ks]))) + (float(rng.choice([0.0, 1.0, 10.0, 57.5])),))
    if with_normals:
        N = f32(rng.normal(size=(max(4, n // 2), 3)))
        N = N / np.linalg.norm(N, axis=1, keepdims=True)
        fn = rng.integers(len(N), size=(n, 3)).astype(np.uint32)
    else:
        N, fn = np.zeros((0, 3)), np.zeros((n, 3), np.uint32)
    return PyMesh(vertices=V, normals=N, face_v=fv, face_n=fn,
                  face_mat=rng.integers(nmat, size=n).astype(np.uint32), materials=np.array(mats, np.float64))


def soup_scene(seed: int, ntri=(300, 700), vertex_light: bool = False) -> PyScene:
    """Two soups (one without vertex normals) placed as 1-3 overlapping objects, 1-5 lights
    (one inside the soups' extent; with vertex_light, one exactly on a vertex of the first
    object), a camera looking at the middle."""
    rng = np.random.default_rng(seed)
    sc = PyScene()
    sc.meshes = [triangle_soup(rng, ntri[0], 1.0, True), triangle_soup(rng, ntri[1], 1.5, False)]
    nobj = int(rng.integers(1, 4))
    sc.objects = [(k % 2, tuple(float(x) for x in rng.normal(scale=0.8, size=3))) for k in range(nobj)]
    on_vertex = tuple(float(x) for x in sc.meshes[0].vertices[int(rng.integers(len(sc.meshes[0].vertices)))]
                      + np.asarray(sc.objects[0][1]))
    lights = [on_vertex if vertex_light else tuple(float(x) for x in rng.normal(scale=3.0, size=3)),
              tuple(float(x) for x in rng.normal(scale=0.5, size=3))]
    for _ in range(int(rng.integers(0, 4))):
        lights.append(tuple(float(x) for x in rng.normal(scale=8.0, size=3)))
    sc.lights = [(p, tuple(float(x) for x in rng.uniform(0, 1, 3))) for p in lights[:5]]
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    sc.cam_pos = tuple(float(x) for x in 6.0 * d)
    sc.cam_dir = tuple(float(x) for x in -d + rng.normal(scale=0.05, size=3))
    sc.fov = float(rng.uniform(0.6, 1.4))
    return sc


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
