"""BASELINE.json configs[3]: the synthetic 1,000,000-triangle UV sphere (SURVEY.md §8(d),
tools/gen_sphere_obj.py) at 3840x2160.  The mesh is far beyond the LDS (BVH and
triangles are read from HBM).  Parity: every 8th column of the full frame against the
oracle (R-tree variant), bit-exact; the generator and both OBJ loaders are checked on CPU
at a small size."""
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


@pytest.mark.gpu
def test_config3_1m_triangles_4k_subsample_vs_oracle(ctx, config3):
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    W, H = 3840, 2160
    env = rt.Environment.from_file(config3, ctx)
    assert sum(len(m.face_v) for m in env.meshes) == 1_000_000
    ctx.profile_enable(True)
    fb = rt.draw(env, W, H)
    p = ctx.profile_read()
    ctx.profile_enable(False)
    assert p["stack_overflows"] == 0
    cols = list(range(7, W, 8))  # every 8th column
    ref = Oracle(load_scene(config3), use_rtree=True).trace_tiles(W, H, [(x, 0, 1, H) for x in cols], nthreads=16)
    sub = np.concatenate([np.arange(x * H, (x + 1) * H) for x in cols])
    assert ref["valid"].sum() > 10000
    assert np.array_equal(fb.valid[sub], ref["valid"])
    assert np.array_equal(fb.rgb8[sub], ref["rgb8"])
    # culling: far fewer tests than brute force (8.3e12 primary alone)
    assert 0 < p["primary_tri_tests"] < W * H * 100
