"""The box-level drop-in (mirt.h mirt_box_*): one worker process serving every
BulkTrace order (worker/distributed/main.go:46-91) on several GPUs.  An order is cut into
column strips dealt over the box's entries and assembled on the first; the bytes must equal
a one-GPU mirt_trace_tile of the same order and the oracle, for every transport, strip width
and order shape.  The box on the GPU box has one MI355X, so several entries share device 0
(the deal, the per-entry contexts and the assembly are the same; device copies stand in for
RCCL, which refuses two ranks on one GPU)."""
import ctypes as C
import threading

import numpy as np
import pytest

from conftest import SCENE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def box8():
    import distributed_raytracer_amd as rt
    b = rt.Box([0] * 8)
    yield b
    b.close()


@pytest.fixture(scope="module")
def box_env(box8):
    import distributed_raytracer_amd as rt
    return rt.Environment.from_file(SCENE, box8)


def _frame_from_orders(tr, parts, W, H):
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import unpack_host
    packed = np.concatenate([tr.bulk_trace(rt.WorkOrder(*p)).results for p in parts])
    fb = np.zeros((W * H, 3), np.uint8)
    unpack_host(W, H, parts, packed, fb)
    return fb


def test_box_of_one_gpu_equals_oracle(py_scene):
    """n = 1 through the C ABI: the whole 320x240 screen and an odd order, every plane."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    b = rt.Box([0])
    try:
        assert b.transport in (rt._lib.MIRT_BOX_COPY, rt._lib.MIRT_BOX_RCCL)
        env = rt.Environment.from_file(SCENE, b)
        W, H = 320, 240
        fb = rt.draw(env, W, H)
        ref = Oracle(py_scene, use_rtree=True).frame(W, H, nthreads=8)
        for k in ("valid", "rgb", "rgb8", "face"):
            assert np.array_equal(getattr(fb, k), ref[k]), k
        r = rt.trace_tile(env, 37, 11, 50, 33, W, H)
        exp = ref["rgb8"].reshape(W, H, 3)[37:87, 11:44].reshape(-1, 3)
        assert np.array_equal(r.rgb8, exp)
        assert r.stats["primary_rays"] == 50 * 33
    finally:
        b.close()


def test_box_emulated_8_master_partition_1080p_matches_oracle(box8, box_env, py_scene):
    """The master's bisection for 8 workers (master/main.go:54-91) at 1920x1080, every
    rectangle served by ONE box worker of 8 entries: the assembled frame equals the oracle
    (the R-tree restatement) on every pixel, rgb8 and the hit count."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import master_partition
    from oracle.oracle import Oracle
    W, H = 1920, 1080
    ref = Oracle(py_scene, use_rtree=True).frame(W, H, nthreads=16)
    parts, _ = master_partition((0, 0, W, H), 8)
    assert len(parts) == 8
    fb = _frame_from_orders(rt.Tracer(box_env, W, H), parts, W, H)
    assert np.array_equal(fb, ref["rgb8"])
    assert int((fb != 0).any(axis=1).sum()) <= 209584


@pytest.mark.parametrize("transport,strip", [("copy", 8), ("host", 8), ("copy", 5), ("host", 13), ("copy", 4096)])
def test_box_every_plane_equals_one_gpu(ctx, env, box8, box_env, transport, strip):
    """Every plane (fp64 rgb, rgb8, valid, face, object) of orders whose width is not a
    multiple of the strip (a partial last strip), narrower than 8 strips (fewer active
    entries than the box has) and one column wide, on both non-RCCL transports, equals
    mirt_trace_tile on one context bit for bit."""
    import distributed_raytracer_amd as rt
    box8.set_transport(rt._lib.MIRT_BOX_COPY if transport == "copy" else rt._lib.MIRT_BOX_HOST)
    box8.set_strip(strip)
    try:
        W, H = 640, 480
        for (x, y, w, h) in [(0, 0, W, H), (101, 57, 333, 211), (300, 200, 19, 50), (320, 0, 1, H), (0, 0, 63, 1)]:
            a = rt.trace_tile(env, x, y, w, h, W, H)
            b = rt.trace_tile(box_env, x, y, w, h, W, H)
            for k in ("rgb", "rgb8", "valid", "face", "obj"):
                assert np.array_equal(getattr(a, k), getattr(b, k)), (transport, strip, (x, y, w, h), k)
            # (tri_tests depend on how the 8x8 packets fall: strips other than 8 px regroup the rays)
            for k in ("primary_rays", "hits", "shadow_rays"):
                assert a.stats[k] == b.stats[k], k
    finally:
        box8.set_transport(rt._lib.MIRT_BOX_COPY)
        box8.set_strip(8)


def test_box_concurrent_orders_with_different_cameras(box8, box_env, py_scene):
    """gRPC serves each BulkTrace in its own goroutine: 8 threads issue orders of two frames
    with different cameras at once on one box; every order equals the oracle's slice."""
    import dataclasses
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    W, H = 320, 240
    base = box_env.mutable()
    pos2 = tuple(float(v) for v in np.asarray(py_scene.cam_pos) * 0.6)
    close = dataclasses.replace(base, cam=rt.Camera.new(pos2, py_scene.cam_dir, py_scene.fov))
    refs = [Oracle(py_scene, use_rtree=True).frame(W, H, nthreads=8)]
    sc2 = dataclasses.replace(py_scene, cam_pos=pos2)
    refs.append(Oracle(sc2, use_rtree=True).frame(W, H, nthreads=8))
    orders = [(x, 0, 40, H) for x in range(0, W, 40)]
    errors = []

    def work(t):
        try:
            for i in range(6):
                k = (t + i) % 2
                x, y, w, h = orders[(3 * t + i) % len(orders)]
                r = rt.trace_tile(box_env, x, y, w, h, W, H, [base, close][k])
                exp = refs[k]["rgb8"].reshape(W, H, 3)[x:x + w, y:y + h].reshape(-1, 3)
                if not np.array_equal(r.rgb8, exp):
                    errors.append((t, i))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors


def test_box_cancel_and_bad_orders(box8, box_env):
    import distributed_raytracer_amd as rt
    W, H = 320, 240
    flag = C.c_int(1)
    with pytest.raises(rt.MirtError) as e:
        rt.trace_tile(box_env, 0, 0, W, H, W, H, cancel=flag)
    assert e.value.code == rt._lib.MIRT_E_CANCELLED
    for bad in [(0, 0, 0, 10), (300, 0, 40, 10), (0, 230, 10, 20)]:
        with pytest.raises(rt.MirtError) as e:
            rt.trace_tile(box_env, *bad, W, H)
        assert e.value.code == rt._lib.MIRT_E_INVALID
    # the box still serves orders afterwards
    r = rt.trace_tile(box_env, 0, 0, W, H, W, H)
    assert int(r.valid.sum()) == 5820
    with pytest.raises(rt.MirtError):
        box8.set_transport(rt._lib.MIRT_BOX_RCCL)  # repeated devices: no communicator
    with pytest.raises(rt.MirtError):
        box8.set_strip(0)


def test_box_entry_profiles_and_options(box8, box_env):
    """Options reach every entry (brute force gives the same frame), and entry contexts expose
    their own counters: the entries' tests add up to the box's."""
    import distributed_raytracer_amd as rt
    W, H = 160, 120
    a = rt.trace_tile(box_env, 0, 0, W, H, W, H)
    box8.set_options(rt._lib.MIRT_OPT_BRUTE_FORCE)
    try:
        b = rt.trace_tile(box_env, 0, 0, W, H, W, H)
    finally:
        box8.set_options(0)
    assert np.array_equal(a.rgb, b.rgb) and np.array_equal(a.valid, b.valid)
    assert b.stats["tri_tests"] > a.stats["tri_tests"]
    e3 = box8.entry(3)
    assert e3.device == 0 and e3.light_cache_stats()["cap"] > 0


def test_box_is_not_a_context(box8, box_env):
    """A Box's handle is a mirt_box: every per-device entry point (trace_rays, the light cache,
    profiling, frame groups, async tiles) raises MIRT_E_INVALID instead of reading a mirt_box
    as a mirt_ctx; its entries still serve those calls."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib
    from distributed_raytracer_amd.framebuffer import trace_tiles_device

    class Planes:
        def outputs(self):
            return _lib.Outputs()
    assert not isinstance(box8, rt.Context)
    o = np.zeros((4, 3))
    d = np.tile([0.0, 0.0, -1.0], (4, 1))
    calls = [lambda: rt.trace_rays(o, d, box_env), lambda: box8.handle,
             lambda: trace_tiles_device(box8, box_env.mutable().to_frame(), 8, 8, [(0, 0, 8, 8)], Planes())]
    for call in calls:
        with pytest.raises(rt.MirtError) as e:
            call()
        assert e.value.code == rt._lib.MIRT_E_INVALID
    for name in ("light_cache_stats", "profile_enable", "stream_create", "debug_timeline", "set_grid"):
        assert not hasattr(box8, name), name
    assert box8.entry(0).light_cache_stats()["cap"] > 0
