"""Parity of the HIP path (through the C ABI) with the oracle and the golden vectors.

Bar: hit mask, winning face and object bit-exact; RGB bit-exact (tolerance stated where
a test allows one: 1e-5 per channel is the north-star bound, but every path here is
expected to be bit-identical because both sides use unfused fp64 in the reference's
operation order).
"""
import ctypes as C
import os
import threading

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-5  # north-star bound per channel; asserted in addition to bit-exactness counts


def _golden(name):
    return np.load(os.path.join(GOLDEN, name))


def test_device_fp64_primitives_bit_exact(ctx):
    import distributed_raytracer_amd as rt
    rng = np.random.default_rng(7)
    a = np.concatenate([rng.random(20000) * 10, rng.random(2000) * 1e-300, np.array([0.0, 1.0, 4.0, 2.0, 1e-310,
                                                                                      5e-324, 1e300])])
    b = np.concatenate([rng.random(20000) + 0.1, rng.random(2000) * 1e10 + 1, np.ones(7)])
    assert np.array_equal(ctx.debug_fp64(0, a, b), np.sqrt(a)), "device sqrt is not correctly rounded"
    assert np.array_equal(ctx.debug_fp64(1, a, b), a / b), "device division is not IEEE"
    x = rng.random(5000)
    y = rng.integers(0, 40, 5000).astype(np.float64)
    host = np.array([rt._lib.lib().mirt_go_pow(float(p), float(q)) for p, q in zip(x, y)])
    assert np.array_equal(ctx.debug_fp64(2, x, y), host), "device go_pow differs from host"
    from oracle.oracle import go_pow
    assert np.array_equal(host, np.array([go_pow(float(p), float(q)) for p, q in zip(x, y)]))
    mx = ctx.debug_fp64(3, np.array([-0.0, 0.0, -1.0, np.nan]), np.array([0.0, -0.0, 0.0, 1.0]))
    assert np.signbit(mx[0]) == False and np.signbit(mx[1]) == False and mx[2] == 0.0 and np.isnan(mx[3])  # noqa: E712


def test_frame_64x48_matches_golden(env):
    import distributed_raytracer_amd as rt
    g = _golden("suzanne_64x48.npz")
    fb = rt.draw(env, 64, 48)
    assert np.array_equal(fb.valid, g["valid"])
    assert np.array_equal(fb.face, g["face"])
    assert np.array_equal(fb.obj, g["obj"])
    assert np.array_equal(fb.rgb, g["rgb"])
    assert np.array_equal(fb.rgb8, g["rgb8"])
    assert fb.stats["hits"] == int(g["valid"].sum())


def test_frame_320x240_matches_golden(env):
    import distributed_raytracer_amd as rt
    g = _golden("suzanne_320x240.npz")
    fb = rt.draw(env, 320, 240)
    hit = np.nonzero(fb.valid)[0]
    assert np.array_equal(hit, g["hit_index"].astype(np.int64))
    assert np.array_equal(fb.face[hit], g["face"])
    assert np.abs(fb.rgb[hit] - g["rgb"]).max() <= RGB_TOL
    assert np.array_equal(fb.rgb[hit], g["rgb"]), f"{(fb.rgb[hit] != g['rgb']).sum()} channels not bit-exact"
    assert np.array_equal(fb.rgb8[hit], g["rgb8"])
    miss = fb.valid == 0
    assert not fb.rgb[miss].any() and not fb.rgb8[miss].any() and (fb.face[miss] == -1).all()
    assert fb.stats["primary_rays"] == 76800 and fb.stats["shadow_rays"] == int(g["shadow_rays"])


def _variants(ctx, fn):
    """Run fn() under every kernel variant: BVH/brute force x prefilter on/off, and the
    static round-robin work split instead of the dynamic work queues."""
    import distributed_raytracer_amd as rt
    out = {}
    try:
        for opts in (0, rt._lib.MIRT_OPT_NO_PREFILTER, rt._lib.MIRT_OPT_BRUTE_FORCE,
                     rt._lib.MIRT_OPT_BRUTE_FORCE | rt._lib.MIRT_OPT_NO_PREFILTER,
                     rt._lib.MIRT_OPT_STATIC_SCHEDULE, rt._lib.MIRT_OPT_NO_SEGMENT,
                     rt._lib.MIRT_OPT_SPLIT_KERNELS, rt._lib.MIRT_OPT_SPLIT_KERNELS | rt._lib.MIRT_OPT_BRUTE_FORCE,
                     rt._lib.MIRT_OPT_NO_FRUSTUM, rt._lib.MIRT_OPT_VIEWS, rt._lib.MIRT_OPT_NO_LIGHT_TABLE):
            ctx.set_options(opts)
            out[opts] = fn()
    finally:
        ctx.set_options(0)
    return out


def _same_frames(res):
    keys = list(res)
    for k in keys[1:]:
        for plane in ("valid", "face", "obj", "rgb", "rgb8"):
            a, b = getattr(res[keys[0]], plane), getattr(res[k], plane)
            assert np.array_equal(a, b), f"variant {k}: {plane} differs in {(a != b).sum()} elements"


def test_kernel_variants_are_exact(ctx, env):
    """BVH culling and the divide-free pre-reject never change a result."""
    import distributed_raytracer_amd as rt
    _same_frames(_variants(ctx, lambda: rt.draw(env, 160, 120)))


def test_bvh_equals_brute_force_many_cameras_1080p(ctx, env):
    """Every pixel of full 1920x1080 frames, 6 cameras around suzanne (grazing views
    included): the culled kernels equal brute force bit-for-bit."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    rng = np.random.default_rng(11)
    for k in range(6):
        ang = rng.uniform(0, 2 * np.pi)
        pos = np.array([1.0 + 4.0 * np.sin(ang), 1.0 + rng.uniform(-2, 2), -1.0 + 4.0 * np.cos(ang)])
        target = np.array([1.0, 1.0, -1.0]) + rng.normal(scale=0.3, size=3)
        cam = rt.Camera.new(pos, target - pos, rng.uniform(0.6, 1.3))
        mut = rt.EnvMutables(base.objects, base.lights, cam)
        res = {}
        for opts in (0, rt._lib.MIRT_OPT_BRUTE_FORCE):
            ctx.set_options(opts)
            res[opts] = rt.draw(env, 1920, 1080, mut)
        ctx.set_options(0)
        assert res[0].valid.sum() > 10000
        _same_frames(res)


def test_block_frustum_exact_at_awkward_cameras(ctx, env):
    """The whole-block frustum pre-test (projected root-child rectangles) never changes a
    pixel: cameras inside the mesh's bounds, grazing the surface, with the object half
    behind the camera or cut by the screen edge, very narrow and very wide fields of view,
    odd frame sizes.  Default kernels vs the pre-test off vs brute force, bit-for-bit."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    c0 = np.array([1.0, 1.0, -1.0])  # suzanne's position in example/scene.json
    cases = [  # (pos, look direction, fov, W, H)
        (c0 + [0.0, 0.0, 0.1], [0.0, 0.0, -1.0], 1.2, 200, 150),       # inside the bounding box
        (c0 + [0.0, 0.2, 0.0], [0.3, -1.0, 0.2], 1.6, 161, 97),        # inside, looking down
        (c0 + [0.0, 0.0, 1.05], [0.0, 0.0, -1.0], 1.0, 240, 136),      # grazing the face
        (c0 + [0.0, 0.0, 0.9], [1.0, 0.0, 0.05], 1.3, 240, 136),       # object beside / behind
        (c0 + [3.0, 0.5, 3.0], [-0.2, -0.1, -1.0], 0.9, 320, 180),     # cut by the screen edge
        (c0 + [0.5, 0.3, 6.0], [-0.08, -0.05, -1.0], 0.06, 256, 256),  # very narrow field of view
        (c0 + [0.0, 0.0, 1.6], [0.0, 0.0, -1.0], 2.9, 300, 120),       # very wide field of view
        (c0 + [0.0, 6.0, 0.0], [0.0, -1.0, 0.001], 1.0, 2, 2),         # 2x2 frame
    ]
    for pos, look, fov, W, H in cases:
        cam = rt.Camera.new(tuple(pos), tuple(look), fov)
        mut = rt.EnvMutables(base.objects, base.lights, cam)
        res = {}
        for opts in (0, rt._lib.MIRT_OPT_NO_FRUSTUM, rt._lib.MIRT_OPT_VIEWS, rt._lib.MIRT_OPT_BRUTE_FORCE):
            ctx.set_options(opts)
            res[opts] = rt.draw(env, W, H, mut)
        ctx.set_options(0)
        _same_frames(res)


def test_shadow_segments_exact_with_lights_near_surfaces(ctx, env):
    """Shadow rays as segment / any-hit queries: lights placed on, just off and inside
    the mesh (occluders at the light's own distance: the ambiguous band of the segment
    rule) give the same frames as brute force."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    mesh = env.meshes[0]
    rng = np.random.default_rng(5)
    v = np.asarray(mesh.vertices, np.float64).reshape(-1, 3)
    obj_pos = np.asarray(base.objects[0].pos, np.float64)
    for trial in range(4):
        lights = []
        for _ in range(6):
            p = v[rng.integers(len(v))] + obj_pos
            kind = rng.integers(3)
            if kind == 1:
                p = p + rng.normal(scale=1e-4, size=3)
            elif kind == 2:
                p = p + rng.normal(scale=0.3, size=3)
            lights.append(rt.Light(tuple(float(x) for x in p), (1.0, 200 / 255, 100 / 255)))
        mut = rt.EnvMutables(base.objects, lights, base.cam)
        res = {}
        for opts in (0, rt._lib.MIRT_OPT_BRUTE_FORCE, rt._lib.MIRT_OPT_NO_SEGMENT, rt._lib.MIRT_OPT_SPLIT_KERNELS,
                     rt._lib.MIRT_OPT_VIEWS, rt._lib.MIRT_OPT_NO_LIGHT_TABLE):
            ctx.set_options(opts)
            res[opts] = rt.draw(env, 320, 240, mut)
        ctx.set_options(0)
        assert res[0].valid.sum() > 1000
        _same_frames(res)


def test_light_table_exact_for_light_placements(ctx, env):
    """The shadow segments' fp32 light-table pre-classification (kernels.hip SegPre) never
    changes a pixel: lights far away, on vertices, 1e-6 and 1e-3 off vertices and edge
    midpoints, on the mesh's face planes, inside the mesh, and an object moved off the
    origin; full 640x480 frames from two cameras, default vs MIRT_OPT_NO_LIGHT_TABLE vs
    brute force, bit-exact."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    mesh = env.meshes[0]
    rng = np.random.default_rng(23)
    v = np.asarray(mesh.vertices, np.float64).reshape(-1, 3)
    fv = np.asarray(mesh.face_v, np.int64).reshape(-1, 3)
    obj_pos = np.asarray(base.objects[0].pos, np.float64)
    col = (1.0, 200 / 255, 100 / 255)
    for trial in range(6):
        pts = []
        f = fv[rng.integers(len(fv), size=4)]
        a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        nrm = np.cross(b - a, c - a)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        pts.append(a[0])                                   # on a vertex
        pts.append(0.5 * (a[1] + b[1]) + 1e-6 * nrm[1])    # just off an edge midpoint
        pts.append((a[2] + b[2] + c[2]) / 3 + 1e-3 * nrm[2])
        pts.append(a[3] + 2.0 * (b[3] - a[3]))             # in a face's plane, outside the face
        pts.append(rng.normal(scale=0.2, size=3))          # inside / near the mesh
        pts.append(rng.normal(scale=30.0, size=3))         # far away
        objs = base.objects
        if trial >= 4:  # the object off its scene position (object space != world space)
            objs = [dataclasses_replace(o, pos=tuple(float(x) for x in obj_pos + rng.normal(scale=0.5, size=3)))
                    for o in base.objects]
        opos = np.asarray(objs[0].pos, np.float64)
        lights = [rt.Light(tuple(float(x) for x in p + opos), col) for p in pts]
        for cam in (base.cam, rt.Camera.new(tuple(opos + [2.5, 1.5, 2.0]), tuple(-np.array([2.5, 1.5, 2.0])), 0.9)):
            mut = rt.EnvMutables(objs, lights, cam)
            res = {}
            for opts in (0, rt._lib.MIRT_OPT_NO_LIGHT_TABLE, rt._lib.MIRT_OPT_BRUTE_FORCE):
                ctx.set_options(opts)
                res[opts] = rt.draw(env, 640, 480, mut)
            ctx.set_options(0)
            assert res[0].valid.sum() > 1000
            _same_frames(res)


def dataclasses_replace(o, **kw):
    import dataclasses
    return dataclasses.replace(o, **kw)


def test_view_tables_exact_for_light_and_camera_placements(ctx, env):
    """The per-view leaf tables (primary rays from the camera, shadow segments from each
    light) never change a pixel: lights far away, at the mesh's centre, inside its bounding
    box, just above the surface, behind the camera and level with the object; cameras from
    several sides.  The BVH walk (default) vs view tables (MIRT_OPT_VIEWS) vs brute force, bit-exact."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    c0 = np.array([1.0, 1.0, -1.0])
    v = np.asarray(env.meshes[0].vertices, np.float64).reshape(-1, 3) + c0
    col = (1.0, 200 / 255, 100 / 255)
    lights = [c0 + [0.0, 0.0, 40.0], c0 + [0.0, 0.0, 0.0], c0 + [0.1, 0.2, -0.1], v[17] * 1.0 + [0.0, 0.0, 1e-3],
              np.asarray(base.cam.pos) + [0.0, 0.0, 1.0], c0 + [3.0, 0.0, 0.0], c0 + [0.0, -5.0, 0.0],
              v[200] + [0.0, 1e-4, 0.0]]
    cams = [(base.cam.pos, base.cam.forward, base.cam.fov), (c0 + [4.0, 1.0, 0.5], (-1.0, -0.2, -0.1), 0.9),
            (c0 + [0.0, -3.0, 0.2], (0.0, 1.0, -0.05), 1.1)]
    for pos, fwd, fov in cams:
        for k in range(0, len(lights), 4):
            mut = rt.EnvMutables(base.objects, [rt.Light(tuple(float(x) for x in p), col) for p in lights[k:k + 4]],
                                 rt.Camera.new(tuple(pos), tuple(fwd), fov))
            res = {}
            for opts in (0, rt._lib.MIRT_OPT_VIEWS, rt._lib.MIRT_OPT_BRUTE_FORCE):
                ctx.set_options(opts)
                res[opts] = rt.draw(env, 256, 192, mut)
            ctx.set_options(0)
            assert res[0].valid.sum() > 500
            _same_frames(res)


def test_bvh_far_camera_and_streamed_mesh(ctx, py_scene):
    """A camera far outside the cull limit (culling disabled per lane) and a mesh too big
    for LDS (BVH walked from HBM) against the oracle."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from oracle.scene_py import PyScene
    from scenes import gpu_env, uv_sphere
    sc = PyScene()
    sc.meshes = [uv_sphere(48, 64, 1.0), py_scene.meshes[0]]
    sc.objects = [(0, (1.0, 1.0, -1.0)), (1, (2.2, 1.5, -0.5))]
    sc.lights = [((0.0, 0.0, 10.0), (0.0, 1.0, 0.0)), ((3.0, 10.0, 4.0), (1.0, 0.5, 0.0))]
    sc.cam_pos, sc.cam_dir, sc.fov = (1.5, 1.2, 900.0), (0.0, 0.0, -1.0), 0.004
    env = gpu_env(ctx, sc)
    res = _variants(ctx, lambda: rt.draw(env, 80, 60))
    _same_frames(res)
    ref = Oracle(sc).frame(80, 60, nthreads=8)
    fb = res[0]
    assert ref["valid"].sum() > 500
    for k in ("valid", "face", "obj", "rgb"):
        assert np.array_equal(getattr(fb, k), ref[k]), k


@pytest.mark.parametrize("tile", [(0, 0, 1, 1), (37, 11, 50, 33), (319, 239, 1, 1), (100, 80, 120, 90),
                                  (0, 0, 320, 240), (13, 200, 307, 40), (150, 0, 1, 240)])
def test_tile_contract_column_major(env, tile):
    """BulkTrace: pixel (x+i, y+j) at i*h + j, global pixel coords, full-screen W,H."""
    import distributed_raytracer_amd as rt
    g = _golden("suzanne_320x240.npz")
    W, H = 320, 240
    full_valid = np.zeros(W * H, np.uint8)
    full_valid[g["hit_index"]] = 1
    full_rgb8 = np.zeros((W * H, 3), np.uint8)
    full_rgb8[g["hit_index"]] = g["rgb8"]
    x, y, w, h = tile
    r = rt.trace_tile(env, x, y, w, h, W, H)
    exp_valid = full_valid.reshape(W, H)[x:x + w, y:y + h].reshape(-1)
    exp_rgb8 = full_rgb8.reshape(W, H, 3)[x:x + w, y:y + h].reshape(-1, 3)
    assert np.array_equal(r.valid, exp_valid)
    assert np.array_equal(r.rgb8, exp_rgb8)


def test_bulk_trace_master_partition(env):
    """Every rectangle of the master's bisection (master/main.go:54-91) for 24 workers,
    traced as BulkTrace orders and reassembled, equals the full frame."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import master_partition, unpack_host
    g = _golden("suzanne_320x240.npz")
    W, H = 320, 240
    parts, _ = master_partition((0, 0, W, H), 24)
    tr = rt.Tracer(env, W, H)
    packed = np.concatenate([tr.bulk_trace(rt.WorkOrder(*p)).results for p in parts])
    fb = np.zeros((W * H, 3), np.uint8)
    unpack_host(W, H, parts, packed, fb)
    exp = np.zeros((W * H, 3), np.uint8)
    exp[g["hit_index"]] = g["rgb8"]
    assert np.array_equal(fb, exp)


def test_trace_single_pixel_api(env):
    import distributed_raytracer_amd as rt
    g = _golden("suzanne_64x48.npz")
    for (i, j) in [(32, 24), (0, 0), (40, 20), (20, 30)]:
        col, ok = rt.trace(i, j, 64, 48, env)
        idx = i * 48 + j
        assert ok == bool(g["valid"][idx])
        assert (col.r, col.g, col.b) == tuple(g["rgb"][idx])
        assert col.rgb() == tuple(int(v) for v in g["rgb8"][idx])


def test_device_tiles_packed_and_unpacked(ctx, env):
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import framebuffer as fbm
    g = _golden("suzanne_320x240.npz")
    W, H = 320, 240
    tiles = fbm.plan_tiles(W, H, 48)
    dev = torch.device("cuda", 0)
    mut = env.mutable()
    frame = mut.to_frame()
    for world, rgbv in ((1, False), (3, False), (3, True)):
        full = fbm.alloc_planes(W * H, dev, with_rgb=True)
        full.valid.zero_()
        for r in range(world):
            mine = fbm.assign(tiles, world, r)
            # rgbv: the multi-GPU packed form (one r|g|b|valid word per pixel), expanded by k_unpack
            packed = fbm.alloc_planes(fbm.pixels_of(mine), dev, with_rgb=True, packed=rgbv)
            fbm.trace_tiles_device(ctx, frame, W, H, mine, packed, torch.cuda.current_stream().cuda_stream)
            fbm.unpack_device(ctx, W, H, mine, packed, full, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        valid = full.valid.cpu().numpy()
        hit = np.nonzero(valid)[0]
        assert np.array_equal(hit, g["hit_index"].astype(np.int64))
        assert np.array_equal(full.rgb.cpu().numpy()[hit], g["rgb"])
        assert np.array_equal(full.rgb8.cpu().numpy()[hit], g["rgb8"])


def test_trace_rays_matches_oracle(env, py_scene):
    """Rays aimed exactly at vertices (box corners of their faces), edge midpoints and surface
    points: every output equals the oracle with the reference's face and object boxes
    (culling="boxes"; on these rays it differs from brute force on 6, and from the R-tree
    oracle only on rays with two faces at the minimum distance, whose order rtreego's DFS
    decides: tests/test_box_gate.py)."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    oracle = Oracle(py_scene, culling="boxes")
    rng = np.random.default_rng(3)
    n = 4000
    m = py_scene.meshes[0]
    pos = np.array(py_scene.objects[0][1])
    # rays aimed exactly at vertices, edge midpoints and random surface points
    V = m.vertices[m.face_v]
    targets = np.concatenate([V[:, 0], (V[:, 0] + V[:, 1]) / 2, V.mean(axis=1)])[:n] + pos
    origins = targets + rng.normal(size=targets.shape) * 3.0
    dirs = targets - origins
    dirs /= np.linalg.norm(dirs, axis=1)[:, None]
    g = rt.trace_rays(origins, dirs, env)
    o = oracle.trace_rays(origins, dirs)
    assert np.array_equal(g["ok"], o["ok"])
    assert np.array_equal(g["face"], o["face"])
    assert np.array_equal(g["hit"], o["hit"])
    assert np.array_equal(g["normal"], o["normal"])


def test_multi_object_flat_and_default_material(ctx, py_scene):
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from scenes import gpu_env, multi_object_scene
    sc = multi_object_scene(py_scene.meshes[0])
    env = gpu_env(ctx, sc)
    W, H = 96, 72
    fb = rt.draw(env, W, H)
    ref = Oracle(sc).frame(W, H, nthreads=8)
    assert ref["valid"].sum() > 1000 and len(np.unique(ref["obj"][ref["valid"] == 1])) == 4
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.obj, ref["obj"])
    assert np.array_equal(fb.face, ref["face"])
    assert np.array_equal(fb.rgb, ref["rgb"])


def test_streamed_mesh_larger_than_lds(ctx):
    """> kLdsTris triangles: the batch-streaming path (not LDS-resident)."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from oracle.scene_py import PyScene
    from scenes import gpu_env, uv_sphere
    sc = PyScene()
    sc.meshes = [uv_sphere(40, 60, 1.2)]  # 4800 triangles
    sc.objects = [(0, (1.0, 1.0, -1.0))]
    sc.lights = [((0.0, 0.0, 10.0), (0.0, 1.0, 0.0)), ((0.0, 10.0, 10.0), (1.0, 0.0, 0.0))]
    sc.cam_pos, sc.cam_dir, sc.fov = (1.0, 1.0, 5.0), (0.0, 0.0, -1.0), 1.04719755
    env = gpu_env(ctx, sc)
    fb = rt.draw(env, 64, 48)
    ref = Oracle(sc).frame(64, 48, nthreads=8)
    assert ref["valid"].sum() > 200
    for k in ("valid", "face", "rgb"):
        assert np.array_equal(getattr(fb, k), ref[k]), k


def test_1080p_full_frame_matches_oracle(ctx, env, py_scene):
    """configs[1] size through mirt_trace_tile (the BulkTrace path): every pixel of the
    1920x1080 frame — valid, winning face, fp64 colour and rgb8 — against the oracle
    (its rtreego-style R-tree variant, which equals its brute force on the fixtures)."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    W, H = 1920, 1080
    fb = rt.draw(env, W, H)
    ref = Oracle(py_scene, use_rtree=True).frame(W, H, nthreads=16)
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.face, ref["face"])
    assert np.array_equal(fb.rgb, ref["rgb"])
    assert np.array_equal(fb.rgb8, ref["rgb8"])
    # SURVEY.md §8c sanity figure for the whole frame
    assert int(fb.valid.sum()) == 209584
    assert fb.stats["shadow_rays"] == 3 * 209584


def test_concurrent_calls_with_different_cameras(ctx, env):
    """Re-entrancy: BulkTrace calls from many threads, each with its own camera."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    cams = [rt.Camera.new((1.0 + 0.1 * k, 1.0, 5.0 - 0.2 * k), (0.05 * k, 0.0, -1.0), 1.04719755)
            for k in range(6)]
    muts = [rt.EnvMutables(base.objects, base.lights, c) for c in cams]
    expect = [rt.trace_tile(env, 0, 0, 80, 60, 80, 60, m) for m in muts]
    got = [None] * (len(muts) * 3)
    errs = []

    def work(k):
        try:
            got[k] = rt.trace_tile(env, 0, 0, 80, 60, 80, 60, muts[k % len(muts)])
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ths = [threading.Thread(target=work, args=(k,)) for k in range(len(got))]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert not errs
    for k, r in enumerate(got):
        e = expect[k % len(muts)]
        assert np.array_equal(r.rgb, e.rgb) and np.array_equal(r.valid, e.valid)


def test_cancel_and_errors(ctx, env):
    import distributed_raytracer_amd as rt
    cancel = C.c_int(1)
    with pytest.raises(rt.MirtError) as ei:
        rt.trace_tile(env, 0, 0, 32, 32, 64, 48, cancel=cancel)
    assert ei.value.code == rt._lib.MIRT_E_CANCELLED
    with pytest.raises(rt.MirtError) as ei:
        rt.trace_tile(env, 60, 0, 10, 10, 64, 48)  # exceeds the screen
    assert ei.value.code == rt._lib.MIRT_E_INVALID
    base = env.mutable()
    bad = rt.EnvMutables([rt.SceneObject(999, (0, 0, 0))], base.lights, base.cam)
    with pytest.raises(rt.MirtError):
        rt.trace_tile(env, 0, 0, 8, 8, 64, 48, bad)
    many = rt.EnvMutables(base.objects, base.lights * 6, base.cam)
    with pytest.raises(rt.MirtError) as ei:
        rt.trace_tile(env, 0, 0, 8, 8, 64, 48, many)
    assert ei.value.code == rt._lib.MIRT_E_LIMIT
    # the context still works after errors
    assert rt.trace_tile(env, 0, 0, 8, 8, 64, 48).valid.shape == (64,)


def test_profile_counters(ctx, env):
    import distributed_raytracer_amd as rt
    ctx.profile_enable(True)
    rt.draw(env, 320, 240)
    rt.draw(env, 320, 240)
    p = ctx.profile_read()
    ctx.set_options(rt._lib.MIRT_OPT_BRUTE_FORCE)
    rt.draw(env, 320, 240)
    b = ctx.profile_read()
    ctx.set_options(0)
    ctx.profile_enable(False)
    assert p["launches"] == 2 and b["launches"] == 1
    assert p["primary_rays"] == 2 * 76800 and p["hits"] == 2 * 5820
    # brute force tests every triangle for every ray; the BVH far fewer
    assert b["primary_tri_tests"] == 76800 * 968 and b["shadow_tri_tests"] == 3 * 5820 * 968
    assert 0 < p["primary_tri_tests"] < 2 * 76800 * 968 / 5
    assert p["primary_ms_sum"] > 0 and p["frame_ms_sum"] >= p["primary_ms_sum"]
    # two launches: the median is their mean; one launch: the launch itself
    assert p["frame_ms_median"] == pytest.approx(p["frame_ms_sum"] / 2, rel=1e-5)
    assert b["frame_ms_median"] == pytest.approx(b["frame_ms_sum"], rel=1e-5)
    assert 0 < p["primary_ms_median"] <= p["frame_ms_median"] * (1 + 1e-6)
    assert p["stack_overflows"] == 0 and b["stack_overflows"] == 0


@pytest.mark.parametrize("inflight,grid", [(3, (32, 0)), (4, (1, 0)), (2, (8, 7))])
def test_frames_in_flight_alternating_cameras(ctx, env, inflight, grid):
    """FrameSharder with several frames in flight (one stream and framebuffer each):
    consecutive frames with DIFFERENT cameras overlap on the GPU; every framebuffer must
    equal its own camera's frame drawn alone (a buffer reused too early would mix
    frames).  Also exercises the launch-shape knob (mirt_set_grid: 1 block per
    workgroup and the default), which never changes results."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder
    W, H = 160, 120
    base = env.mutable()
    c = base.cam
    cams = [c, rt.Camera.new(tuple(np.asarray(c.pos) + np.array([0.7, 0.3, 0.0])), c.forward, c.fov),
            rt.Camera.new(tuple(np.asarray(c.pos) + np.array([-0.5, -0.2, 0.4])), c.forward, c.fov * 0.8)]
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in cams]
    frames = [m.to_frame() for m in muts]
    refs = [rt.draw(env, W, H, m) for m in muts]
    assert len({int(r.valid.sum()) for r in refs}) == 3  # three different images
    ctx.set_grid(*grid)
    try:
        sh = FrameSharder(ctx, W, H, 0, 1, inflight=inflight)
        order = [0, 1, 2, 1, 0, 2, 2, 1, 0, 1, 2, 0]
        for q in order:
            sh.render(frames[q])
        sh.flush()
        torch.cuda.synchronize()
        for k in range(len(order) - inflight, len(order)):  # the last `inflight` frames' buffers
            q = order[k]
            got = sh.frames[k % inflight]
            assert np.array_equal(got.valid.cpu().numpy(), refs[q].valid), f"frame {k} (camera {q}) valid differs"
            assert np.array_equal(got.rgb8.cpu().numpy(), refs[q].rgb8), f"frame {k} (camera {q}) rgb8 differs"
        assert sh.frame is sh.frames[(len(order) - 1) % inflight]
    finally:
        ctx.set_grid()


def test_octant_child_test_changes_nothing(ctx, env):
    """The sign-octant walk (the node copy of the packet's octant: near/far planes loaded
    pre-ordered, children sorted near to far) and the generic walk (copy 0 with the sorted
    min/max test, MIRT_OPT_NO_OCTANT) must give identical frames for views whose packets
    are uniform and views that mix signs.  Their traversal counters differ: the nearest
    query skips boxes beyond a lane's best candidate, which depends on the visiting order."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    c = base.cam
    cams = [c,
            rt.Camera.new(tuple(np.asarray(c.pos) + np.array([0.9, 0.6, 0.2])), tuple(-np.asarray(c.pos)), c.fov),
            rt.Camera.new((0.3, 0.2, 0.1), (0.2, -0.1, -1.0), 2.0)]  # inside the mesh's box: mixed signs
    try:
        for cam in cams:
            mut = rt.EnvMutables(base.objects, base.lights, cam)
            res = []
            for opt in (0, rt._lib.MIRT_OPT_NO_OCTANT):
                ctx.set_options(opt)
                ctx.profile_enable(True)
                fb = rt.draw(env, 320, 240, mut)
                ctx.profile_enable(False)
                res.append((fb, ctx.profile_read()))
            (a, pa), (b, pb) = res
            assert np.array_equal(a.valid, b.valid) and np.array_equal(a.rgb, b.rgb) and np.array_equal(a.face, b.face)
            assert pa["hits"] == pb["hits"] and pa["primary_node_visits"] > 0 and pb["primary_node_visits"] > 0
    finally:
        ctx.set_options(0)


@pytest.mark.parametrize("tile,tile_h,inflight,batch", [
    (None, 0, 4, 1), (32, 32, 3, 1), (8, 0, 2, 1), (48, 0, 1, 1),
    (None, 0, 4, 4), (8, 0, 4, 2), (32, 32, 6, 3), (None, 0, 3, 2), (8, 0, 8, 8)])
def test_native_frame_group_matches_draw(ctx, env, tile, tile_h, inflight, batch):
    """mirt_trace_frame (the native multi-GPU frame driver) on one GPU: the whole screen
    (tile=None) or the tiled path rehearsed with world = 1 (packed rgbv tiles or
    full-height strips, the unpack table with per-rank offsets), frames in flight with
    alternating cameras, and several frames per k_trace launch (batch; a frame with
    fewer lights cannot share a launch and closes the batch early); every framebuffer
    equals its frame drawn alone."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W, H = 160, 120
    base = env.mutable()
    c = base.cam
    cams = [c, rt.Camera.new(tuple(np.asarray(c.pos) + np.array([0.7, 0.3, 0.0])), c.forward, c.fov)]
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in cams]
    muts.append(rt.EnvMutables(base.objects, base.lights[:2], cams[1]))  # fewer lights
    c0 = np.array([1.0, 1.0, -1.0])  # suzanne's position
    muts.append(rt.EnvMutables(base.objects, base.lights,  # turned away: an empty hit rectangle
                               rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov)))
    muts.append(rt.EnvMutables(base.objects, base.lights,  # object cut by the screen edge
                               rt.Camera.new(tuple(c0 + [3.0, 0.5, 3.0]), (-0.2, -0.1, -1.0), 0.9)))
    muts.append(rt.EnvMutables(base.objects, base.lights,  # camera inside the bounding box
                               rt.Camera.new(tuple(c0 + [0.0, 0.0, 0.1]), (0.0, 0.0, -1.0), 1.2)))
    frames = [m.to_frame() for m in muts]
    refs = [rt.draw(env, W, H, m) for m in muts]
    assert refs[3].valid.sum() == 0 and 0 < refs[4].valid.sum() and 0 < refs[5].valid.sum()
    try:
        g = NativeFrameGroup(ctx, W, H, 0, 1, tile, inflight=inflight, tile_h=tile_h, batch=batch)
        order = [0, 1, 4, 0, 3, 5, 0, 1, 2, 0, 1, 4, 5, 2, 3, 0, 4, 5, 1, 4, 0, 3]
        for q in order:
            g.render(frames[q])
        g.flush()
        torch.cuda.synchronize()
        for k in range(len(order) - inflight, len(order)):
            got = g.frames[k % inflight]
            q = order[k]
            assert np.array_equal(got.valid.cpu().numpy(), refs[q].valid), f"frame {k} valid differs"
            assert np.array_equal(got.rgb8.cpu().numpy(), refs[q].rgb8), f"frame {k} rgb8 differs"
        g.close()
    finally:
        ctx.set_grid()


@pytest.mark.parametrize("inflight", [1, 2, 3])
def test_frame_slots_refill_only_stale_columns(ctx, env, inflight):
    """Whole-screen framebuffers are refilled only in the columns an earlier frame of the
    same slot may have hit: every frame, checked as soon as it is done, equals its frame
    drawn alone, whatever the slot held before (a wide hit rectangle, then narrow ones, an
    empty one, the whole screen)."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W, H = 200, 150
    base = env.mutable()
    c = base.cam
    c0 = np.array([1.0, 1.0, -1.0])
    cams = [rt.Camera.new(tuple(c0 + [0.0, 0.0, 0.1]), (0.0, 0.0, -1.0), 1.2),   # inside the box: wide
            c,                                                                  # default
            rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov),         # turned away: empty
            rt.Camera.new(tuple(c0 + [3.0, 0.5, 3.0]), (-0.2, -0.1, -1.0), 0.9),  # cut by the left edge
            rt.Camera.new(tuple(np.asarray(c.pos) + [-1.5, 0.0, 0.0]), c.forward, c.fov)]  # shifted
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in cams]
    frames = [m.to_frame() for m in muts]
    refs = [rt.draw(env, W, H, m) for m in muts]
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=inflight)
    try:
        for k, q in enumerate([0, 1, 2, 3, 0, 4, 1, 3, 2, 0, 1, 4, 4, 3]):
            g.render(frames[q])
            g.flush()
            torch.cuda.synchronize()
            got = g.frame
            assert np.array_equal(got.valid.cpu().numpy(), refs[q].valid), f"frame {k} valid differs"
            assert np.array_equal(got.rgb8.cpu().numpy(), refs[q].rgb8), f"frame {k} rgb8 differs"
    finally:
        g.close()
        ctx.set_grid()


def test_group_batch_arguments(ctx):
    """mirt_group_set_batch: 1..min(8, inflight) frames per launch, before the first frame."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    env = rt.Environment.from_file(os.path.join(GOLDEN, "example", "scene.json"), ctx)
    try:
        g = NativeFrameGroup(ctx, 64, 48, 0, 1, None, inflight=4)
        lib = L.lib()
        assert lib.mirt_group_set_batch(g._h, 0) == L.MIRT_E_INVALID
        assert lib.mirt_group_set_batch(g._h, 5) == L.MIRT_E_INVALID  # more than in flight
        assert lib.mirt_group_set_batch(g._h, 4) == L.MIRT_OK
        g.render(env.mutable().to_frame())
        assert lib.mirt_group_set_batch(g._h, 2) == L.MIRT_E_INVALID  # after the first frame
        g.flush()
        g.close()
    finally:
        ctx.set_grid()


@pytest.mark.gpu
def test_near_coplanar_and_subnormal_direction_rays(ctx, env, py_scene):
    """DESIGN.md §4.2's documented exception of BVH culling, pinned on constructed rays:
    (a) rays grazing a face at 1e-8 and 1e-12 of its plane (the Möller–Trumbore determinant
    small but well above its rounding error): the culled walk equals brute force and the
    oracle exactly; at 1e-16 and 0 (the ray lies in the face's plane to within rounding, the
    determinant is rounding noise and so is t) the culled walk may differ only on rays whose
    oracle or culled winner is such a face (|det| <= 2^-40 |e1||e2||d|); (b) rays whose
    direction is subnormal, so the determinant underflows and t overflows: brute force
    equals the oracle (the reference reports such hits at infinity), and the culled walk
    may differ from them only on rays whose oracle hit is not finite."""
    import distributed_raytracer_amd as rt
    import distributed_raytracer_amd._lib as L
    from oracle.oracle import Oracle
    rng = np.random.default_rng(29)
    m = py_scene.meshes[0]
    pos = np.array(py_scene.objects[0][1])
    V = np.asarray(m.vertices, np.float64).reshape(-1, 3)[np.asarray(m.face_v).reshape(-1, 3)] + pos
    faces = rng.choice(len(V), 300, replace=False)
    P1, P2, P3 = V[faces, 0], V[faces, 1], V[faces, 2]
    X = (P1 + P2 + P3) / 3
    n = np.cross(P2 - P1, P3 - P1)
    n /= np.linalg.norm(n, axis=1)[:, None]
    u = (P2 - P1) / np.linalg.norm(P2 - P1, axis=1)[:, None]
    graze_o, graze_d = [], []
    for delta in (1e-8, 1e-12, 1e-16, 0.0):
        d = -(u + n * delta)
        graze_o.append(X - d * 0.5)
        graze_d.append(d / np.linalg.norm(d, axis=1)[:, None])
    go, gd = np.concatenate(graze_o), np.concatenate(graze_d)
    so = X + rng.normal(size=X.shape) * 2.0
    sd = (X - so) / np.linalg.norm(X - so, axis=1)[:, None]
    sub_o = np.concatenate([so, so])
    sub_d = np.concatenate([sd * 1e-310, sd * 4e-320])
    orc = Oracle(py_scene, culling="boxes")  # the kernels' semantics: every candidate box-gated
    try:
        for origins, dirs, exact in ((go, gd, True), (sub_o, sub_d, False)):
            ref = orc.trace_rays(origins, dirs)
            ctx.set_options(L.MIRT_OPT_BRUTE_FORCE)
            brute = rt.trace_rays(origins, dirs, env)
            ctx.set_options(0)
            bvh = rt.trace_rays(origins, dirs, env)
            for k in ("ok", "face"):
                assert np.array_equal(brute[k], ref[k]), f"brute force vs oracle ({k})"
            assert np.array_equal(brute["hit"], ref["hit"], equal_nan=True)
            diff = (bvh["ok"] != ref["ok"]) | (bvh["face"] != ref["face"])
            if exact:
                well = np.arange(len(diff)) < 2 * len(faces)  # deltas 1e-8, 1e-12
                assert not (diff & well).any(), f"{int((diff & well).sum())} grazing rays differ from the oracle"
                assert np.array_equal(bvh["hit"][well], ref["hit"][well]) and ref["ok"][well].sum() > 0

                def coplanar(fi, k):  # the ray lies in face fi's plane to within rounding
                    P = V[fi]
                    e1, e2 = P[1] - P[0], P[2] - P[0]
                    det = abs(np.dot(e1, np.cross(e2, -dirs[k])))
                    return det <= 2.0 ** -40 * np.linalg.norm(e1) * np.linalg.norm(e2) * np.linalg.norm(dirs[k])
                for k in np.flatnonzero(diff):
                    cands = [int(r["face"][k]) for r in (ref, bvh) if r["ok"][k]]
                    assert any(coplanar(fi, k) for fi in cands), \
                        f"ray {k}: oracle face {ref['face'][k]} ok={ref['ok'][k]}, culled {bvh['face'][k]} ok={bvh['ok'][k]}"
                same = ~diff
                assert np.array_equal(bvh["hit"][same], ref["hit"][same], equal_nan=True)
            else:
                finite = np.isfinite(ref["hit"]).all(axis=1)
                assert not (diff & (~ref["ok"].astype(bool) | finite)).any(), \
                    "the culled walk differs on a ray whose reference hit is finite (or absent)"
    finally:
        ctx.set_options(0)


@pytest.mark.gpu
def test_rays_at_triangle_edges_and_vertices(ctx, env, py_scene):
    """The divide-free classification of the barycentric conditions on the
    rays it must leave undecided: rays aimed exactly at vertices, edge midpoints and points
    1e-15 .. 1e-9 (relative) inside and outside edges, from random origins (primary-like)
    and from just above the surface (shadow-like).  Default kernel, MIRT_OPT_NO_PREFILTER
    (the reference's divides for every lane) and brute force all equal the oracle with the
    reference's face and object boxes (culling="boxes"; vertices are box corners)."""
    import distributed_raytracer_amd as rt
    import distributed_raytracer_amd._lib as L
    from oracle.oracle import Oracle
    rng = np.random.default_rng(31)
    m = py_scene.meshes[0]
    pos = np.array(py_scene.objects[0][1])
    V = np.asarray(m.vertices, np.float64).reshape(-1, 3)[np.asarray(m.face_v).reshape(-1, 3)] + pos
    faces = rng.choice(len(V), 200, replace=False)
    P1, P2, P3 = V[faces, 0], V[faces, 1], V[faces, 2]
    C = (P1 + P2 + P3) / 3
    targets = [P1, P2, P3, (P1 + P2) / 2, (P2 + P3) / 2, (P3 + P1) / 2]
    for eps in (1e-15, 1e-12, 1e-9):
        M = (P1 + P2) / 2
        targets += [M + (C - M) * eps, M - (C - M) * eps]
    T = np.concatenate(targets)
    n = np.cross(P2 - P1, P3 - P1)
    n /= np.linalg.norm(n, axis=1)[:, None]
    N = np.tile(n, (len(targets), 1))
    far = T + rng.normal(size=T.shape) * 3.0
    near = T + N * 1e-3 + rng.normal(size=T.shape) * 1e-3
    origins = np.concatenate([far, near])
    dirs = np.concatenate([T, T]) - origins
    dirs /= np.linalg.norm(dirs, axis=1)[:, None]
    ref = Oracle(py_scene, culling="boxes").trace_rays(origins, dirs)
    assert ref["ok"].sum() > len(origins) // 2
    try:
        for opts in (0, L.MIRT_OPT_NO_PREFILTER, L.MIRT_OPT_BRUTE_FORCE):
            ctx.set_options(opts)
            got = rt.trace_rays(origins, dirs, env)
            for k in ("ok", "face"):
                assert np.array_equal(got[k], ref[k]), (opts, k, int((got[k] != ref[k]).sum()))
            assert np.array_equal(got["hit"], ref["hit"], equal_nan=True), opts
    finally:
        ctx.set_options(0)


@pytest.mark.gpu
@pytest.mark.parametrize("inflight,batch", [(4, 1), (8, 2)])
def test_1080p_frame_group_bench_path_matches_oracle(ctx, env, py_scene, inflight, batch):
    """The bench's own path at configs[1] size: the native frame group (frames in flight,
    `batch` frames per k_trace launch, host output on), every pixel of the D2H'd rgb8 and
    valid planes and of the device fp64 rgb plane against the oracle, for the last frame
    of a run long enough to reuse every frame slot."""
    import torch
    from oracle.oracle import Oracle
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W, H = 1920, 1080
    ref = Oracle(py_scene, use_rtree=True).frame(W, H, nthreads=16)
    fr = env.mutable().to_frame()
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=inflight, batch=batch, with_rgb=True, host_output=True)
    try:
        last = None
        for _ in range(2 * inflight + 1):
            last = g.render(fr)
        g.wait()
        g.flush()
        torch.cuda.synchronize()
        rgb8, valid = g.host_frame(last)
        assert np.array_equal(valid, ref["valid"])
        assert np.array_equal(rgb8, ref["rgb8"])
        dev = g.frames[last % inflight]
        assert np.array_equal(dev.rgb.cpu().numpy(), ref["rgb"])
        assert int(valid.sum()) == 209584
    finally:
        g.close()



@pytest.mark.parametrize("max_wg", [1, 3])
def test_hit_chunk_ring_many_batches_per_workgroup(ctx, env, oracle, max_wg):
    """k_trace's hit-chunk ring (kernels.hip ring_take) under the heaviest
    reuse: 1 or 3 workgroups for a 640x480 frame (4,800 blocks: up to 19 batches of 256 blocks
    per workgroup, hundreds of hit chunks through 8 ring positions, and positions past the ring
    whenever more than 8 chunks are live).  The default camera's frame must equal the oracle's;
    a close camera (more hit blocks) must equal the default grid's frame."""
    import distributed_raytracer_amd as rt
    W, H = 640, 480
    base = env.mutable()
    c = base.cam
    close = rt.EnvMutables(base.objects, base.lights, rt.Camera.new(tuple(np.asarray(c.pos) * 0.55), c.forward, c.fov))
    ctx.set_grid(1, max_wg)
    try:
        fb = rt.draw(env, W, H)
        fc = rt.draw(env, W, H, close)
    finally:
        ctx.set_grid()
    ref = oracle.frame(W, H, nthreads=8)
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.rgb, ref["rgb"])
    assert np.array_equal(fb.rgb8, ref["rgb8"])
    full = rt.draw(env, W, H, close)
    assert int(full.valid.sum()) > int(fb.valid.sum())  # the close view hits more pixels
    assert np.array_equal(fc.valid, full.valid) and np.array_equal(fc.rgb, full.rgb)
    assert np.array_equal(fc.rgb8, full.rgb8)
