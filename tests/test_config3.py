"""BASELINE.json configs[3]: the synthetic 1,000,000-triangle UV sphere (SURVEY.md §8(d),
tools/gen_sphere_obj.py) at 3840x2160.  The mesh is far beyond the LDS (BVH and
triangles are read from HBM).  Parity: every 8th column of the full frame against the
oracle (R-tree variant) — valid, rgb8 and the fp64 rgb bit-exact (and within 1e-5) — through
mirt_trace_tile and through the bench's frame group; the generator and both OBJ loaders are
checked on CPU at a small size."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_generator_counts_and_loaders_agree(tmp_path):
    import gen_sphere_obj as g
    from oracle.scene_py import load_scene
    import distributed_raytracer_amd.tracer as tr
    v, n, f = g.sphere_arrays(500, 1000)
    assert f.shape == (1_000_000, 3) and v.shape == (501 * 1001, 3)
    scene = g.write(str(tmp_path), stacks=20, slices=40)
    py = load_scene(scene)
    meshes, objs, lights, cam = tr.load_scene_arrays(scene)
    assert len(py.meshes[0].face_v) == 2 * 20 * 40 == len(meshes[0].face_v)
    assert np.array_equal(np.asarray(py.meshes[0].vertices, np.float64).reshape(-1, 3),
                          np.asarray(meshes[0].vertices, np.float64).reshape(-1, 3))
    assert np.array_equal(np.asarray(py.meshes[0].face_v).reshape(-1, 3), np.asarray(meshes[0].face_v).reshape(-1, 3))


@pytest.fixture(scope="module")
def config3(tmp_path_factory):
    import gen_sphere_obj as g
    return g.write(str(tmp_path_factory.mktemp("config3")))


W4K, H4K = 3840, 2160
RGB_TOL = 1e-5  # north_star's bound per channel (asserted beside bit-exactness)


@pytest.fixture(scope="module")
def config3_ref(config3):
    """The oracle (R-tree restatement) on every 8th column of the 4K frame, and those pixels'
    indices in the column-major framebuffer."""
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    cols = list(range(7, W4K, 8))
    ref = Oracle(load_scene(config3), use_rtree=True).trace_tiles(W4K, H4K, [(x, 0, 1, H4K) for x in cols],
                                                                  nthreads=16)
    sub = np.concatenate([np.arange(x * H4K, (x + 1) * H4K) for x in cols])
    assert ref["valid"].sum() > 10000
    return ref, sub


def _check_rgb(rgb, ref):
    """fp64 colour: bit-exact, and within north_star's 1e-5 per channel."""
    assert float(np.abs(rgb - ref["rgb"]).max()) <= RGB_TOL
    assert np.array_equal(rgb, ref["rgb"])


@pytest.mark.gpu
def test_config3_1m_triangles_4k_subsample_vs_oracle(ctx, config3, config3_ref):
    import distributed_raytracer_amd as rt
    W, H = W4K, H4K
    ref, sub = config3_ref
    env = rt.Environment.from_file(config3, ctx)
    assert sum(len(m.face_v) for m in env.meshes) == 1_000_000
    ctx.profile_enable(True)
    fb = rt.draw(env, W, H)
    p = ctx.profile_read()
    ctx.profile_enable(False)
    assert p["stack_overflows"] == 0
    assert np.array_equal(fb.valid[sub], ref["valid"])
    assert np.array_equal(fb.rgb8[sub], ref["rgb8"])
    _check_rgb(fb.rgb[sub], ref)
    # culling: far fewer tests than brute force (8.3e12 primary alone)
    assert 0 < p["primary_tri_tests"] < W * H * 100


@pytest.mark.gpu
def test_config3_frame_group_8x2_vs_oracle(ctx, config3, config3_ref):
    """The bench's path at configs[3]: the native frame group with 8 frames in flight, 2 per
    k_trace launch, host output on; the last frame of a run that reuses every slot, through
    the D2H (rgb8, valid) and the device fp64 rgb plane, on every 8th column."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W, H = W4K, H4K
    ref, sub = config3_ref
    env = rt.Environment.from_file(config3, ctx)
    fr = env.mutable().to_frame()
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=8, batch=2, with_rgb=True, host_output=True)
    try:
        last = None
        for _ in range(2 * 8 + 2):
            last = g.render(fr)
        g.wait()
        g.flush()
        torch.cuda.synchronize()
        rgb8, valid = g.host_frame(last)
        assert np.array_equal(valid[sub], ref["valid"])
        assert np.array_equal(rgb8[sub], ref["rgb8"])
        dev = g.frames[last % 8]
        _check_rgb(dev.rgb.cpu().numpy()[sub], ref)
    finally:
        g.close()
        ctx.set_grid()


@pytest.fixture(scope="module")
def sphere6k(tmp_path_factory):
    """A 6,400-face UV sphere (the configs[3] generator, 40 x 80 cells): beyond the LDS, so its
    triangles and nodes are read from HBM, small enough for a full-frame oracle."""
    import gen_sphere_obj as g
    return g.write(str(tmp_path_factory.mktemp("sphere6k")), stacks=40, slices=80)


@pytest.mark.gpu
def test_hbm_mesh_kernels_and_lds_streaming_equal_oracle(ctx, sphere6k):
    """Every kernel an HBM-resident mesh can take gives the oracle's frame, every pixel: the
    one-object HBM k_trace with the primary rays' triangles streamed through each wave's LDS
    window (the default: north_star's LDS batch streaming; MIRT_OPT_LDS_STREAM is accepted and
    changes nothing), the same reading the triangles with scalar loads (MIRT_OPT_NO_LDS_STREAM),
    the generic k_trace (MIRT_OPT_NO_SEGMENT) and the split kernels; and the streamed frame
    group, 4 frames per launch."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    W, H = 160, 120
    env = rt.Environment.from_file(sphere6k, ctx)
    assert sum(len(m.face_v) for m in env.meshes) == 6400
    ref = Oracle(load_scene(sphere6k), use_rtree=True).frame(W, H, nthreads=16)
    assert ref["valid"].sum() > 1000
    L = rt._lib
    for opts in (0, L.MIRT_OPT_NO_LDS_STREAM, L.MIRT_OPT_LDS_STREAM, L.MIRT_OPT_NO_SEGMENT, L.MIRT_OPT_SPLIT_KERNELS,
                 L.MIRT_OPT_NO_OCTANT, L.MIRT_OPT_NO_LDS_STREAM | L.MIRT_OPT_NO_OCTANT):
        ctx.set_options(opts)
        try:
            fb = rt.draw(env, W, H)
        finally:
            ctx.set_options(0)
        for k in ("valid", "face", "rgb", "rgb8"):
            assert np.array_equal(getattr(fb, k), ref[k]), (opts, k)
    ctx.set_options(0)
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=8, batch=4, with_rgb=True)
    try:
        fr = env.mutable().to_frame()
        last = None
        for _ in range(9):
            last = g.render(fr)
        g.wait()
        g.flush()
        torch.cuda.synchronize()
        dev = g.frames[last % 8]
        assert np.array_equal(dev.rgb.cpu().numpy(), ref["rgb"])
        assert np.array_equal(dev.valid.cpu().numpy(), ref["valid"])
    finally:
        g.close()
        ctx.set_options(0)
        ctx.set_grid()


@pytest.mark.gpu
def test_config3_scalar_load_path_4k_subsample_vs_oracle(ctx, config3, config3_ref):
    """configs[3] with the triangles read by scalar loads instead of streamed through LDS
    (MIRT_OPT_NO_LDS_STREAM, the round-4 default): every 8th column, bit-exact."""
    import distributed_raytracer_amd as rt
    ref, sub = config3_ref
    env = rt.Environment.from_file(config3, ctx)
    ctx.set_options(rt._lib.MIRT_OPT_NO_LDS_STREAM)
    try:
        fb = rt.draw(env, W4K, H4K)
    finally:
        ctx.set_options(0)
    assert np.array_equal(fb.valid[sub], ref["valid"])
    assert np.array_equal(fb.rgb8[sub], ref["rgb8"])
    _check_rgb(fb.rgb[sub], ref)
