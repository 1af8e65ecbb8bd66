"""configs[2] frame assembly, bit for bit, on one GPU (the reference's
master gathers BulkTrace rectangles and draws them, master/main.go:130-176).

mirt_group_emulate makes a world == 1 frame group trace EVERY rank's share of an N-way
deal (mirt_group_plan_tiles, the root weighted down), pack each share into that rank's
transfer buffer with the same k_pack_rect offsets a peer uses, copy exactly the bytes an
RCCL send would carry into the root's gathered region, check every region's trailer and
unpack all N regions.  Every pixel of every 1920x1080 frame is compared with the oracle
(rtreego-style R-tree restatement, oracle/rt_oracle.c).  Also: the bench's own whole-screen
path (2 frames per launch) on full frames, the host output (D2H) of assembled frames, and
the fault path (a rank stops answering -> MIRT_E_PEER naming it -> re-deal over the
survivors -> exact frames again)."""
import numpy as np
import pytest

from conftest import SCENE

W, H = 1920, 1080
C0 = np.array([1.0, 1.0, -1.0])  # suzanne's position in example/scene.json


def _cameras(base):
    c = base.cam
    return {
        "default": (tuple(c.pos), tuple(c.forward), c.fov),
        "away": (tuple(c.pos), tuple(-np.asarray(c.forward)), c.fov),  # empty hit rectangle
        "edge": (tuple(C0 + [3.0, 0.5, 3.0]), (-0.2, -0.1, -1.0), 0.9),  # object cut by the screen edge
        "inside": (tuple(C0 + [0.0, 0.0, 0.1]), (0.0, 0.0, -1.0), 1.2),  # camera inside the bounding box
    }


@pytest.fixture(scope="module")
def views(env, py_scene):
    """name -> (frame for the GPU, oracle frame) for the four cameras."""
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from scenes import with_camera
    base = env.mutable()
    out = {}
    for name, (pos, d, fov) in _cameras(base).items():
        mut = rt.EnvMutables(base.objects, base.lights, rt.Camera.new(pos, d, fov))
        ref = Oracle(with_camera(py_scene, pos, d, fov), use_rtree=True).frame(W, H, nthreads=16)
        out[name] = (mut.to_frame(), ref)
    assert out["away"][1]["valid"].sum() == 0 and out["edge"][1]["valid"].sum() > 0
    assert out["default"][1]["valid"].sum() == 209584
    return out


def _check(got_valid, got_rgb8, ref, what):
    assert np.array_equal(got_valid, ref["valid"]), f"{what}: valid differs in {(got_valid != ref['valid']).sum()} px"
    assert np.array_equal(got_rgb8, ref["rgb8"]), f"{what}: rgb8 differs in {(got_rgb8 != ref['rgb8']).any(1).sum()} px"


ORDER = ["default", "edge", "away", "inside", "default", "inside", "edge", "default"]


@pytest.mark.gpu
@pytest.mark.parametrize("world,tile,tile_h,batch", [
    (2, 8, 0, 1), (4, 8, 0, 1), (8, 8, 0, 1), (2, 8, 0, 4), (4, 8, 0, 4), (8, 8, 0, 4), (4, 32, 32, 2)])
def test_emulated_world_full_frames(ctx, views, world, tile, tile_h, batch):
    """N = 2, 4, 8 ranks (8-px strips, the bench's deal; and 32x32 tiles), one or several
    frames per launch, cameras alternating between the default view, an edge cut, a turned
    away camera (empty transfers) and one inside the box: every framebuffer equals the
    oracle on every pixel."""
    import torch
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    F = 4
    g = NativeFrameGroup(ctx, W, H, 0, 1, tile, inflight=F, tile_h=tile_h, batch=batch, emulate=world)
    try:
        for name in ORDER:
            g.render(views[name][0])
        g.wait()
        torch.cuda.synchronize()
        for k in range(len(ORDER) - F, len(ORDER)):
            got = g.frames[k % F]
            _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[ORDER[k]][1],
                   f"world {world} frame {k} ({ORDER[k]})")
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("world,tile,chains", [(4, 8, False), (2, 32, True), (1, None, False)])
def test_emulated_world_reflections(ctx, env, world, tile, chains):
    """configs[4] (3 bounces) through the frame group: each rank's share traced with the
    reflection level waves (k_pack walks the share's own block table) or the chains, packed,
    gathered and unpacked; frames equal the single-call draw() (itself checked against the
    oracle in test_config4.py) on every pixel."""
    import dataclasses
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W2, H2 = 640, 360
    mut = dataclasses.replace(env.mutable(), max_bounces=3)
    ctx.set_options(L.MIRT_OPT_REFLECT_CHAINS if chains else 0)
    try:
        ref = rt.draw(env, W2, H2, mut)
        assert ref.valid.sum() > 1000
        g = NativeFrameGroup(ctx, W2, H2, 0, 1, tile, inflight=2, emulate=world if world > 1 else 0)
        try:
            for _ in range(3):
                g.render(mut.to_frame())
            g.wait()
            torch.cuda.synchronize()
            for k in range(2):
                got = g.frames[k]
                assert np.array_equal(got.valid.cpu().numpy(), ref.valid), f"frame {k}: valid differs"
                assert np.array_equal(got.rgb8.cpu().numpy(), ref.rgb8), f"frame {k}: rgb8 differs"
        finally:
            g.close()
            ctx.set_grid()
    finally:
        ctx.set_options(0)


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", [1, 2])
def test_reflection_frames_narrowed_to_the_hit_rectangle(ctx, env, inflight):
    """Reflection frames through a whole-screen frame group are narrowed to their hit rectangle
    (k_primary skips the blocks outside FrameRec::live; the group refills the columns an earlier
    frame of the slot hit).  Cameras whose rectangles differ — the default view, a turned-away
    camera (empty), an edge cut, one inside the box — follow each other on the same slots: every
    frame equals the single-call draw() of its camera (itself checked against the oracle in
    test_config4.py) on every pixel."""
    import dataclasses
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W2, H2 = 640, 360
    base = env.mutable()
    cams = _cameras(base)
    order = ["default", "away", "edge", "inside", "default", "edge", "away", "default"]
    refs = {}
    for name in set(order):
        pos, d, fov = cams[name]
        mut = dataclasses.replace(rt.EnvMutables(base.objects, base.lights, rt.Camera.new(pos, d, fov)), max_bounces=3)
        refs[name] = (mut, rt.draw(env, W2, H2, mut))
    assert refs["away"][1].valid.sum() == 0 and refs["default"][1].valid.sum() > 1000
    g = NativeFrameGroup(ctx, W2, H2, 0, 1, None, inflight=inflight)
    try:
        for k, name in enumerate(order):
            g.render(refs[name][0].to_frame())
            g.wait()
            torch.cuda.synchronize()
            got, ref = g.frames[k % inflight], refs[name][1]
            assert np.array_equal(got.valid.cpu().numpy(), ref.valid), f"frame {k} ({name}): valid differs"
            assert np.array_equal(got.rgb8.cpu().numpy(), ref.rgb8), f"frame {k} ({name}): rgb8 differs"
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
def test_adaptive_grid_lone_and_burst_frames(ctx, views, monkeypatch):
    """MIRT_ADAPTIVE_GRID=2: a frame issued while none runs gets the whole chip's grid, a
    frame of a burst the fixed one; one slot sees both launch shapes in turn (its hit
    buffers are sized for any grid) and every frame equals the oracle."""
    import torch
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_ADAPTIVE_GRID", "2")
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=2)
    try:
        for k, name in enumerate(ORDER):
            g.render(views[name][0])
            if k % 3 == 0:  # a lone frame next: nothing left running
                g.wait()
                torch.cuda.synchronize()
                got = g.frames[k % 2]
                _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[name][1], f"frame {k} ({name})")
        g.wait()
        torch.cuda.synchronize()
        for k in range(len(ORDER) - 2, len(ORDER)):
            got = g.frames[k % 2]
            _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[ORDER[k]][1], f"frame {k} ({ORDER[k]})")
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("hold,host_output", [("1", False), ("1", True), ("0", True)])
def test_lone_hold_lone_and_burst_frames(ctx, views, hold, host_output, monkeypatch):
    """Lone-frame hold (MIRT_LONE_HOLD, mirt.cpp mirt_trace_frame): a frame submitted while the
    group runs nothing is held; a wait launches it alone on the whole chip, a further submit
    launches it with the fixed grid.  Lone frames (render + wait), bursts and host frames read
    between renders (mirt_group_frame_host on a held frame) all equal the oracle, with the fused
    host copies (8 in flight) carrying copies across both launch shapes."""
    import torch
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_LONE_HOLD", hold)
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=8, host_output=host_output)
    try:
        for rep in range(2):
            for k, name in enumerate(ORDER):
                idx = g.render(views[name][0])
                if k % 3 == 0:  # a lone frame: its wait launches it
                    if host_output:
                        rgb8, valid = g.host_frame(idx)  # the held frame, launched by this call
                        _check(valid, rgb8, views[name][1], f"host frame {idx} ({name})")
                    g.wait()
                    torch.cuda.synchronize()
                    got = g.frames[idx % 8]
                    _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[name][1], f"frame {idx} ({name})")
            g.wait()
            torch.cuda.synchronize()
            for k in range(len(ORDER) - 3, len(ORDER)):
                idx = rep * len(ORDER) + k
                got = g.frames[idx % 8]
                _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[ORDER[k]][1], f"frame {idx} ({ORDER[k]})")
                if host_output:
                    rgb8, valid = g.host_frame(idx)
                    _check(valid, rgb8, views[ORDER[k]][1], f"host frame {idx} ({ORDER[k]})")
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", [2, 8])
def test_host_output_odd_height(ctx, env, py_scene, inflight, monkeypatch):
    """The host copy's span search reads the valid plane in aligned 8-byte words: with an odd
    screen height (333 x 201) the columns start at every byte alignment and the last column's
    words run past the plane's end (masked).  Host frames over moving and emptying hit
    rectangles, lone frames (waited one by one) and bursts (fused copies at 8 in flight) equal
    the oracle on every pixel."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    from oracle.oracle import Oracle
    from scenes import with_camera
    W2, H2 = 333, 201
    base = env.mutable()
    frames = []
    for name, (pos, d, fov) in _cameras(base).items():
        mut = rt.EnvMutables(base.objects, base.lights, rt.Camera.new(pos, d, fov))
        ref = Oracle(with_camera(py_scene, pos, d, fov), use_rtree=True).frame(W2, H2, nthreads=8)
        frames.append((name, mut.to_frame(), ref))
    g = NativeFrameGroup(ctx, W2, H2, 0, 1, None, inflight=inflight, host_output=True)
    try:
        seq = frames + frames[::-1] + frames
        for k, (name, fr, ref) in enumerate(seq):  # lone frames
            idx = g.render(fr)
            rgb8, valid = g.host_frame(idx)
            _check(valid, rgb8, ref, f"lone host frame {k} ({name})")
        run = [(g.render(fr), name, ref) for name, fr, ref in seq]  # a burst
        g.wait()
        for idx, name, ref in run[-inflight:]:
            rgb8, valid = g.host_frame(idx)
            _check(valid, rgb8, ref, f"host frame {idx} ({name})")
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
def test_bench_path_full_frame(ctx, views):
    """The bench's own configuration (whole screen, 8 frames in flight, 2 frames per
    k_trace launch, frame records staged per launch): every pixel of each frame, valid,
    rgb8, and the fp64 colour of tracer.Trace (with_rgb)."""
    import torch
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    for with_rgb in (False, True):
        g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=8, batch=2, with_rgb=with_rgb)
        try:
            for name in ORDER:
                g.render(views[name][0])
            g.wait()
            torch.cuda.synchronize()
            for k, name in enumerate(ORDER):
                got, ref = g.frames[k % 8], views[name][1]
                _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), ref, f"frame {k} ({name})")
                if with_rgb:
                    assert np.array_equal(got.rgb.cpu().numpy(), ref["rgb"]), f"frame {k} ({name}): rgb differs"
        finally:
            g.close()
            ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("tile,emulate,wait", [(None, 0, "sync"), (8, 8, "sync"), (None, 0, "spin"), (8, 8, "spin")])
def test_host_output_frames(ctx, views, tile, emulate, wait, monkeypatch):
    """mirt_group_set_host_output: the assembled frame lands in pinned host memory (the copy
    kernel covers only each column's hit span and the slot's previous one); the host planes
    equal the oracle on every pixel while the rectangle moves and empties between frames,
    and after host output was switched off and on again.  wait: the group's completion waits
    (MIRT_WAIT, read at creation): blocking, or polled events."""
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_WAIT", wait)
    g = NativeFrameGroup(ctx, W, H, 0, 1, tile, inflight=2, batch=1, emulate=emulate, host_output=True)
    try:
        prev = None
        for k, name in enumerate(ORDER):
            if k == 4:  # frames traced with the host output off never reach the host slots
                g.set_host_output(False)
                g.render(views["inside"][0])
                g.render(views["edge"][0])
                g.wait()
                g.set_host_output(True)
                prev = None
            idx = g.render(views[name][0])
            if prev is not None:
                rgb8, valid = g.host_frame(prev[0])
                _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
            prev = (idx, name)
        rgb8, valid = g.host_frame(prev[0])
        _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
        g.wait()
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("inflight,batch", [(4, 1), (8, 1), (8, 2)])
def test_host_output_fused_copies(ctx, views, inflight, batch, monkeypatch):
    """Fused host copies (MIRT_FUSED_COPY=1, mirt.cpp update_fused_copy): a batch's copy runs in
    the next k_trace launch on its stream, or as its own kernel when the caller asks for the frame
    first (host_frame, wait).  Host frames read right after each render (every copy flushed on
    demand) and a run of frames read only after a wait (copies fused into later launches): every
    host frame equals the oracle over moving, emptying and refilling hit rectangles."""
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_FUSED_COPY", "1")
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=inflight, batch=batch, host_output=True)
    try:
        prev = None
        for name in ORDER * 2:
            idx = g.render(views[name][0])
            if prev is not None:
                rgb8, valid = g.host_frame(prev[0])
                _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
            prev = (idx, name)
        g.wait()
        run = []
        for name in ORDER * 3:
            run.append((g.render(views[name][0]), name))
        g.wait()
        for idx, name in run[-inflight:]:  # the frames whose host slots still hold them
            rgb8, valid = g.host_frame(idx)
            _check(valid, rgb8, views[name][1], f"host frame {idx} ({name})")
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", [2, 4])
def test_host_output_runahead_reserved_copy_cus(ctx, views, inflight, monkeypatch):
    """Host run-ahead 4 (MIRT_RUNAHEAD) with the host copies on a stream of reserved CUs
    (MIRT_D2H_CUS): an untiled group of one-frame batches, where batch nb - FB's copy on that
    stream is the only guard on a framebuffer's reuse (mirt.cpp group_flush).  Three passes over
    the moving, emptying and refilling hit rectangles: every host frame equals the oracle."""
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_RUNAHEAD", "4")
    monkeypatch.setenv("MIRT_D2H_CUS", "8")
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=inflight, batch=1, host_output=True)
    try:
        prev = None
        for k, name in enumerate(ORDER * 3):
            idx = g.render(views[name][0])
            if prev is not None:
                rgb8, valid = g.host_frame(prev[0])
                _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
            prev = (idx, name)
        rgb8, valid = g.host_frame(prev[0])
        _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
        g.wait()
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("emulate_after_host_output", [False, True])
def test_library_owned_planes_host_output(ctx, views, emulate_after_host_output):
    """fbs == NULL on a tiled root (the group allocates its own rgb8 + valid planes, as the
    C / Go workers use it at N > 1) with host output on, and mirt_group_emulate called
    before or after mirt_group_set_host_output: group_plan's buffer growth must not free the
    group's own planes or the host-copy spans (a regression: it once did, and the unpack and
    host copy then wrote freed memory).  Every host frame equals the oracle."""
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    if emulate_after_host_output:
        g = NativeFrameGroup(ctx, W, H, 0, 1, 8, inflight=2, batch=1, host_output=True, library_planes=True)
        L.check(L.lib().mirt_group_emulate(g._h, 4))
    else:
        g = NativeFrameGroup(ctx, W, H, 0, 1, 8, inflight=2, batch=1, emulate=4, host_output=True,
                             library_planes=True)
    try:
        assert g.frames is None
        prev = None
        for name in ORDER:
            idx = g.render(views[name][0])
            if prev is not None:
                rgb8, valid = g.host_frame(prev[0])
                _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
            prev = (idx, name)
        rgb8, valid = g.host_frame(prev[0])
        _check(valid, rgb8, views[prev[1]][1], f"host frame {prev[0]} ({prev[1]})")
        g.wait()
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
def test_peer_failure_is_named_and_redealt(ctx, views):
    """A rank that stops answering (emulated: its transfers are dropped) fails the frame
    with MIRT_E_PEER naming that rank — the master skips such frames, master/main.go:153-161
    — and after mirt_group_exclude the survivors' re-deal gives exact frames again (the pool
    drops the worker, master/pool/pool.go:224-260)."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    g = NativeFrameGroup(ctx, W, H, 0, 1, 8, inflight=2, batch=1, emulate=4, timeout_ms=20000)
    try:
        g.render(views["default"][0])
        g.wait()
        _check(g.frames[0].valid.cpu().numpy(), g.frames[0].rgb8.cpu().numpy(), views["default"][1], "before")
        g.drop([2])
        g.render(views["edge"][0])
        with pytest.raises(rt.MirtError) as e:
            g.wait()
        assert e.value.code == L.MIRT_E_PEER and "rank(s) 2" in str(e.value)
        assert g.failed_ranks() == [2]
        g.exclude([0, 1, 3])
        for k, name in enumerate(["edge", "default", "inside"]):
            g.render(views[name][0])
            g.wait()
            torch.cuda.synchronize()
            got = g.frames[(2 + k) % 2]
            _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), views[name][1], f"after re-deal ({name})")
        assert g.failed_ranks() == []
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
def test_group_argument_errors(ctx):
    """Tiled groups cannot produce the fp64 colour plane; emulation needs world == 1 and a
    tile; the root cannot be dropped or excluded."""
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    with pytest.raises(rt.MirtError):
        NativeFrameGroup(ctx, 64, 48, 0, 1, 8, inflight=2, with_rgb=True)
    with pytest.raises(rt.MirtError):
        NativeFrameGroup(ctx, 64, 48, 0, 1, None, inflight=2, emulate=4)
    g = NativeFrameGroup(ctx, 64, 48, 0, 1, 8, inflight=2, emulate=2)
    try:
        assert L.lib().mirt_group_emulate_drop(g._h, 1) == L.MIRT_E_INVALID
        assert L.lib().mirt_group_exclude(g._h, 2, None) == L.MIRT_E_INVALID
    finally:
        g.close()
        ctx.set_grid()


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["mesh_release", "destroy", "host_frame_of_previous"])
def test_held_frame_is_launched_not_dropped(ctx, views, how, monkeypatch):
    """A frame the lone-frame hold keeps (submitted to an idle group) is traced by every call
    that can follow it: mirt_mesh_release launches it before freeing the mesh its record points
    at, mirt_group_destroy before the group goes, and mirt_group_frame_host of the PREVIOUS frame
    (a pipelined caller) before it waits.  The framebuffer then equals the oracle without any
    mirt_group_wait."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    monkeypatch.setenv("MIRT_LONE_HOLD", "1")
    env2 = rt.Environment.from_file(SCENE, ctx)  # a mesh of its own (the scene's default camera), released below
    mut = env2.mutable()
    ref = views["default"][1]
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=2, host_output=(how == "host_frame_of_previous"))
    planes = g.frames
    try:
        if how == "host_frame_of_previous":
            i0 = g.render(mut.to_frame())
            g.wait()
            i1 = g.render(mut.to_frame())  # held: the group is idle
            rgb8, valid = g.host_frame(i0)
            _check(valid, rgb8, ref, "host frame 0")
        else:
            i1 = g.render(mut.to_frame())  # held
            if how == "mesh_release":
                for mid in env2.mesh_ids:
                    ctx.release_mesh(mid)
            else:
                g.close()
        torch.cuda.synchronize()
        got = planes[i1 % 2]
        _check(got.valid.cpu().numpy(), got.rgb8.cpu().numpy(), ref, f"{how}: held frame {i1}")
    finally:
        g.close()
        ctx.set_grid()
