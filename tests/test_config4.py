"""BASELINE.json configs[4]: the 4-bounce reflection EXTENSION (not in the reference;
SURVEY.md §8(d) "defined by the build").  The oracle is the build's own
CPU restatement (oracle/rt_oracle.c shade_reflect), checked against the kernels
bit-for-bit: full frames at small sizes (one and several objects, 1..4 bounces) and a
subsample of the 3840x2160 configs[4] frame."""
import dataclasses

import numpy as np
import pytest


def _oracle(sc, bounces):
    from oracle.oracle import Oracle
    o = Oracle(sc)
    o.set_bounces(bounces)
    return o


def test_oracle_bounces_zero_is_the_reference(py_scene):
    from oracle.oracle import Oracle
    a = Oracle(py_scene).frame(80, 60, nthreads=8)
    b = _oracle(py_scene, 0).frame(80, 60, nthreads=8)
    assert np.array_equal(a["rgb"], b["rgb"]) and b["stats"]["reflection_rays"] == 0
    c = _oracle(py_scene, 2).frame(80, 60, nthreads=8)
    assert c["stats"]["reflection_rays"] >= c["stats"]["hits"]  # one per primary hit at least
    assert np.array_equal(a["valid"], c["valid"])               # reflections only change colours
    assert (c["rgb"] >= a["rgb"] - 1e-12).all()                  # and only add light (Ks >= 0)


@pytest.mark.gpu
@pytest.mark.parametrize("bounces", [1, 4])
def test_reflections_full_frame_bit_exact(ctx, env, py_scene, bounces):
    import distributed_raytracer_amd as rt
    mut = dataclasses.replace(env.mutable(), max_bounces=bounces)
    ctx.profile_enable(True)
    fb = rt.draw(env, 320, 240, mut)
    p = ctx.profile_read()
    ctx.profile_enable(False)
    ref = _oracle(py_scene, bounces).frame(320, 240, nthreads=8)
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.rgb, ref["rgb"]), f"{(fb.rgb != ref['rgb']).any(axis=1).sum()} pixels differ"
    assert np.array_equal(fb.rgb8, ref["rgb8"])
    assert p["reflection_rays"] == ref["stats"]["reflection_rays"]
    assert p["shadow_rays"] == ref["stats"]["shadow_rays"] and p["stack_overflows"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("bounces", [1, 4])
def test_reflection_chains_full_frame_bit_exact(ctx, env, py_scene, bounces):
    """MIRT_OPT_REFLECT_CHAINS (one k_reflect launch following each pixel's chain) gives the
    level waves' frames (the default: k_pack, k_bounce, k_shadow per level, k_refl_fold) and
    ray counts bit for bit."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    mut = dataclasses.replace(env.mutable(), max_bounces=bounces)
    ctx.set_options(L.MIRT_OPT_REFLECT_CHAINS)
    try:
        ctx.profile_enable(True)
        fb = rt.draw(env, 320, 240, mut)
        p = ctx.profile_read()
        ctx.profile_enable(False)
    finally:
        ctx.set_options(0)
    ref = _oracle(py_scene, bounces).frame(320, 240, nthreads=8)
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.rgb, ref["rgb"]), f"{(fb.rgb != ref['rgb']).any(axis=1).sum()} pixels differ"
    assert np.array_equal(fb.rgb8, ref["rgb8"])
    assert p["reflection_rays"] == ref["stats"]["reflection_rays"]
    assert p["shadow_rays"] == ref["stats"]["shadow_rays"] and p["stack_overflows"] == 0


@pytest.mark.gpu
def test_reflections_multi_object(ctx, py_scene):
    import distributed_raytracer_amd as rt
    from scenes import gpu_env, multi_object_scene
    sc = multi_object_scene(py_scene.meshes[0])
    env = gpu_env(ctx, sc)
    mut = dataclasses.replace(env.mutable(), max_bounces=3)
    fb = rt.draw(env, 120, 90, mut)
    ref = _oracle(sc, 3).frame(120, 90, nthreads=8)
    assert ref["stats"]["reflection_rays"] > ref["stats"]["hits"]  # inter-object bounces happen
    assert np.array_equal(fb.valid, ref["valid"])
    assert np.array_equal(fb.rgb, ref["rgb"])


@pytest.mark.gpu
def test_config4_4k_subsample(ctx, env, py_scene):
    import distributed_raytracer_amd as rt
    W, H = 3840, 2160
    mut = dataclasses.replace(env.mutable(), max_bounces=4)
    fb = rt.draw(env, W, H, mut)
    cols = list(range(11, W, 8))  # every 8th column
    ref = _oracle(py_scene, 4).trace_tiles(W, H, [(x, 0, 1, H) for x in cols], nthreads=16)
    sub = np.concatenate([np.arange(x * H, (x + 1) * H) for x in cols])
    assert ref["valid"].sum() > 10000
    assert np.array_equal(fb.valid[sub], ref["valid"])
    assert np.array_equal(fb.rgb[sub], ref["rgb"])
    assert np.array_equal(fb.rgb8[sub], ref["rgb8"])


@pytest.mark.gpu
def test_max_bounces_limit(ctx, env):
    import distributed_raytracer_amd as rt
    mut = dataclasses.replace(env.mutable(), max_bounces=99)
    with pytest.raises(rt.MirtError):
        rt.draw(env, 8, 8, mut)
