"""k_trace's cost deal (kernels.hip k_trace): blocks whose trace on a slot's
previous launch took long are dealt over the workgroups from that launch's cost lists, every
other block by the lattice, and the previous launch's stamps keep the two sets disjoint.  A
block missed by both would leave stale pixels; a block queued twice would count its hits twice
(and its shadow rays: the bench's rays).  These tests change everything the lists depend on
between launches of one slot — camera, tile list, grid, frames per launch — and check every
pixel and the hit count of every frame (reference: worker/shared/tracer/tracer.go:81-91; the
deal changes the order of work only)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cameras(rt, base):
    c = base.cam
    c0 = np.array([1.0, 1.0, -1.0])  # suzanne's position
    return [c,
            rt.Camera.new(tuple(np.asarray(c.pos) * 0.55), c.forward, c.fov),  # close: more hit blocks
            rt.Camera.new(tuple(np.asarray(c.pos) + np.array([0.7, 0.3, 0.0])), c.forward, c.fov),
            rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov),  # turned away: nothing listed
            rt.Camera.new(tuple(c0 + [3.0, 0.5, 3.0]), (-0.2, -0.1, -1.0), 0.9)]


@pytest.mark.parametrize("inflight,batch", [(1, 1), (3, 1), (4, 2), (6, 3)])
def test_deal_traces_each_block_once_in_frame_groups(ctx, env, inflight, batch):
    """A frame group with alternating cameras (each slot's lists come from another view) and
    several frames per launch: every framebuffer equals its frame drawn alone, and the hits
    summed over the run equal the hit pixels of the frames rendered."""
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    W, H = 320, 240
    base = env.mutable()
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in _cameras(rt, base)]
    frames = [m.to_frame() for m in muts]
    refs = [rt.draw(env, W, H, m) for m in muts]
    assert refs[3].valid.sum() == 0 and refs[1].valid.sum() > refs[0].valid.sum()
    order = [0, 0, 1, 1, 0, 2, 3, 0, 4, 1, 1, 4, 0, 3, 2, 2, 1, 0, 0, 4, 1, 0, 2, 3]
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=inflight, batch=batch)
    try:
        ctx.profile_enable(True)
        for q in order:
            g.render(frames[q])
        g.flush()
        torch.cuda.synchronize()
        prof = ctx.profile_read()
        ctx.profile_enable(False)
        for k in range(len(order) - inflight, len(order)):
            q = order[k]
            got = g.frames[k % inflight]
            assert np.array_equal(got.valid.cpu().numpy(), refs[q].valid), f"frame {k} (camera {q}) valid differs"
            assert np.array_equal(got.rgb8.cpu().numpy(), refs[q].rgb8), f"frame {k} (camera {q}) rgb8 differs"
        assert prof["hits"] == sum(int(refs[q].valid.sum()) for q in order)
        assert prof["stack_overflows"] == 0
    finally:
        ctx.profile_enable(False)
        g.close()


@pytest.mark.parametrize("grid", [(1, 0), (8, 7), (1, 3), (32, 0), (2, 64)])
def test_deal_across_grids_tile_lists_and_cameras(ctx, env, grid):
    """One context's slots serve draws and BulkTrace orders of other sizes, cameras and grids
    in turn (a slot's lists index another block table, or a larger launch's blocks): every
    result equals the reference drawn at the default launch shape, hits included.  Few
    workgroups (7 or 3) take hundreds of listed blocks each, over several LDS batches."""
    import distributed_raytracer_amd as rt
    base = env.mutable()
    cams = _cameras(rt, base)
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in cams]
    sizes = [(320, 240), (640, 480), (160, 120)]
    refs = {(s, q): rt.draw(env, s[0], s[1], muts[q]) for s in sizes for q in range(len(muts))}
    tr = rt.Tracer(env, 640, 480)
    seq = [((640, 480), 1), ((640, 480), 1), ((320, 240), 0), ((640, 480), 1), ((160, 120), 4),
           ((640, 480), 0), ((640, 480), 3), ((320, 240), 2), ((640, 480), 1)]
    ctx.set_grid(*grid)
    try:
        for i, (s, q) in enumerate(seq):
            fb = rt.draw(env, s[0], s[1], muts[q])
            ref = refs[(s, q)]
            assert np.array_equal(fb.valid, ref.valid), f"draw {i} {s} camera {q}"
            assert np.array_equal(fb.rgb, ref.rgb), f"draw {i} {s} camera {q}"
            assert fb.stats["hits"] == int(ref.valid.sum()), f"draw {i}: a block traced twice or never"
            # a BulkTrace order (master/main.go:54-91 rectangles) on the same slots
            x, y, w, h = (64 * i) % 320, (40 * i) % 240, 320, 240
            res = tr.bulk_trace(rt.WorkOrder(x, y, w, h, muts[1]))
            full = refs[((640, 480), 1)]
            want = full.rgb8.reshape(640, 480, 3)[x:x + w, y:y + h].reshape(-1, 3)
            assert np.array_equal(res.results, want), f"order {i} ({x}, {y}, {w}, {h})"
    finally:
        ctx.set_grid()
