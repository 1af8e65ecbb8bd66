"""The shadow segments' fp32 light-table pre-classification (kernels.hip SegPre,
mirt.cpp light_records), checked on the host: the records the library builds
(mirt_debug_light_table) and the kernel's reject rule restated in numpy float32 never
reject a (shadow ray, triangle) pair that the reference's fp64 Möller–Trumbore
(triangle.go:37-77, as np_oracle restates it) reports as a hit, over shadow rays built as
tracer.go:60-64 builds them from hit points on suzanne, with lights on vertices, just off
edges, in face planes, inside the mesh and far away — and they do reject most misses.
CPU only (no device call)."""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENE = os.path.join(ROOT, "tests", "golden", "example", "scene.json")


def _lib():
    import distributed_raytracer_amd._lib as L
    return L.lib()


def _mesh():
    from oracle.scene_py import load_scene
    sc = load_scene(SCENE)
    mi, pos = sc.objects[0]
    m = sc.meshes[mi]
    V = np.asarray(m.vertices, np.float64)
    F = np.asarray(m.face_v, np.int64)
    P1, P2, P3 = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    tri = np.concatenate([P1, P2 - P1, P3 - P1], axis=1)  # the kernels' record: P1, E1, E2
    return tri, float(np.abs(V).max()), np.asarray(pos, np.float64), V, F


def _records(tri, scale, pos, lights):
    n, nl = len(tri), len(lights)
    out = np.zeros((nl, n, 16), np.float32)
    t = np.ascontiguousarray(tri, np.float64)
    p = np.ascontiguousarray(pos, np.float64)
    lp = np.ascontiguousarray(lights, np.float64)
    assert _lib().mirt_debug_light_table(t.ctypes.data, n, scale, p.ctypes.data, lp.ctypes.data, nl,
                                         out.ctypes.data) == 0
    return out


def _fma(a, b, c):
    # float32 fma: the product of two float32 is exact in float64; the sum rounds twice
    # (float64 then float32), within 1 ulp of the fused result — far inside the bounds' margin
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def _reject(rec, d, lh):
    """kernels.hip seg_reject for rays (rows) x triangles (columns), float32."""
    f = np.float32
    dx, dy, dz = (d[:, k].astype(f)[:, None] for k in range(3))
    ninf = np.maximum(np.maximum(np.abs(dx), np.abs(dy)), np.abs(dz))
    lam = (lh - 1e-4).astype(f)[:, None]
    lamn = f(2.0) * np.abs(lam) * ninf
    w = [rec[None, :, q] for q in range(16)]
    m = [_fma(w[3 * k + 2], dz, _fma(w[3 * k + 1], dy, w[3 * k] * dx)) for k in range(4)]
    a = m[3]
    E, Ea = ninf * w[13], ninf * w[14]
    nt = _fma(-lam, a, w[12])
    Et = _fma(lamn, w[14], w[15])
    lo = np.minimum(np.minimum(m[0], m[1]), m[2])
    hi = np.maximum(np.maximum(m[0], m[1]), m[2])
    return ((a > Ea) & ((lo < -E) | (nt > Et))) | ((a < -Ea) & ((hi > E) | (nt < -Et)))


def _mt_hits(tri, ro, d):
    """triangle.go:37-77 in fp64 for rays (rows) x triangles (columns): the hit decision."""
    with np.errstate(all="ignore"):
        p1 = [tri[None, :, k] for k in range(3)]
        e1 = [tri[None, :, 3 + k] for k in range(3)]
        e2 = [tri[None, :, 6 + k] for k in range(3)]
        o = [ro[:, k][:, None] for k in range(3)]
        neg = [-1.0 * d[:, k][:, None] for k in range(3)]

        def cross(a, b):
            return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]

        def dot(a, b):
            return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]
        c = cross(e2, neg)
        inc = dot(e1, c)
        p1or = [o[k] - p1[k] for k in range(3)]
        r2 = dot(p1or, c) / inc
        r3 = dot(e1, cross(p1or, neg)) / inc
        s = r2 + r3
        r1 = 1.0 - r2 - r3
        t = dot(e1, cross(e2, p1or)) / inc
        return (inc != 0.0) & (0.0 <= r2) & (r2 <= 1.0) & (0.0 <= s) & (s <= 1.0) & (r1 >= 0.0) & (r2 >= 0.0) & \
            (r3 >= 0.0) & (t >= 0.0)


def _shadow_rays(V, F, pos, L, rng, n):
    """Hit points on the mesh (world space) and the shadow rays of tracer.go:60-64 to L."""
    f = F[rng.integers(len(F), size=n)]
    b = rng.dirichlet((1.0, 1.0, 1.0), size=n)
    b[: n // 8] = np.round(b[: n // 8], 1)          # some on edges and vertices
    b /= b.sum(axis=1, keepdims=True)
    hit = (b[:, :1] * V[f[:, 0]] + b[:, 1:2] * V[f[:, 1]] + b[:, 2:] * V[f[:, 2]]) + pos
    v = L[None, :] - hit
    lh = np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2])
    d = v / lh[:, None]                                  # tracer.go:61 Norm
    o = hit + d * 0.0001                                 # tracer.go:64
    return o - pos, d, lh                                # object.go:71 rOrigin.Sub(o.Pos)


def _light_positions(V, F, rng):
    f = F[rng.integers(len(F), size=3)]
    a, b, c = V[f[:, 0]], V[f[:, 1]], V[f[:, 2]]
    nrm = np.cross(b - a, c - a)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    return [a[0], 0.5 * (a[1] + b[1]) + 1e-6 * nrm[1], (a[2] + b[2] + c[2]) / 3 + 1e-3 * nrm[2],
            a[0] + 2.0 * (b[0] - a[0]), rng.normal(scale=0.2, size=3), rng.normal(scale=30.0, size=3),
            np.array([4.0, 5.0, -3.0])]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_light_table_never_rejects_a_hit(seed):
    tri, scale, pos0, V, F = _mesh()
    rng = np.random.default_rng(seed)
    pos = pos0 + (rng.normal(scale=0.5, size=3) if seed == 3 else 0.0)
    lights = [p + pos for p in _light_positions(V, F, rng)]
    rec = _records(tri, scale, pos, np.array(lights))
    hits = rejected_miss = misses = 0
    for li, L in enumerate(lights):
        ro, d, lh = _shadow_rays(V, F, pos, L, rng, 640)
        hit = _mt_hits(tri, ro, d)
        rej = _reject(rec[li], d, lh)
        bad = hit & rej
        assert not bad.any(), f"light {li}: {int(bad.sum())} hits rejected"
        hits += int(hit.sum())
        misses += int((~hit).sum())
        rejected_miss += int((rej & ~hit).sum())
    assert hits > 100
    # the pre-classification decides nearly every miss (undecided: near edges, t ~ 0)
    assert rejected_miss > 0.97 * misses, (rejected_miss, misses)


def test_light_table_sound_on_nan_and_overflow():
    """A light so far away that the W vectors overflow fp32 (the bound is then infinite:
    only the t test can decide), and NaN directions (never rejected)."""
    tri, scale, pos, V, F = _mesh()
    rng = np.random.default_rng(4)
    L = np.array([1e30, 2e30, -1e30])
    rec = _records(tri, scale, pos, L[None, :])[0]
    assert np.isinf(rec[:, 13]).all()
    ro, d, lh = _shadow_rays(V, F, pos, L, rng, 64)
    hit = _mt_hits(tri, ro, d)
    assert not (hit & _reject(rec, d, lh)).any()
    d[:8] = np.nan
    assert not _reject(rec, d, lh)[:8].any()


def test_light_table_record_layout():
    """W1 + W2 + W3 = A = E1 x E2 and ntL = A.(L - P1) (to fp32 rounding); bounds positive."""
    tri, scale, pos, V, F = _mesh()
    L = np.array([4.0, 5.0, -3.0])
    rec = _records(tri, scale, pos, L[None, :])[0].astype(np.float64)
    A = np.cross(tri[:, 3:6], tri[:, 6:9])
    Wsum = rec[:, 0:3] + rec[:, 3:6] + rec[:, 6:9]
    mag = np.abs(rec[:, 0:9]).max(axis=1)
    assert np.all(np.abs(Wsum - A).max(axis=1) <= 1e-5 * mag + 1e-12)
    assert np.allclose(rec[:, 9:12], A, rtol=1e-6, atol=0)
    ntL = np.einsum("ij,ij->i", A, (L - pos)[None, :] - tri[:, 0:3])
    assert np.allclose(rec[:, 12], ntL, rtol=1e-5, atol=1e-9)
    assert (rec[:, 13:16] > 0).all()


@pytest.mark.gpu
def test_device_light_table_equals_host(ctx):
    """k_light_table (the builder the cache uses) and the host builder share lighttab.hpp's
    arithmetic: bit-identical records for suzanne with lights on a vertex, in a face plane,
    inside the mesh, far away and at 1e30, and for a soup at an offset position."""
    from scenes import soup_scene
    tri, scale, pos, V, F = _mesh()
    rng = np.random.default_rng(4)
    lights = np.concatenate([_light_positions(V, F, rng), [[0.1, 0.2, 0.3], [1e30, -2.0, 3.0], [40.0, 50.0, -60.0]]])
    cases = [(tri, scale, pos, lights[:16])]
    sc = soup_scene(12, vertex_light=True)
    m = sc.meshes[0]
    Vs, Fs = np.asarray(m.vertices, np.float64), np.asarray(m.face_v, np.int64)
    ts = np.concatenate([Vs[Fs[:, 0]], Vs[Fs[:, 1]] - Vs[Fs[:, 0]], Vs[Fs[:, 2]] - Vs[Fs[:, 0]]], axis=1)
    cases.append((ts, float(np.abs(Vs).max()), np.array([0.5, -3.0, 2.25]), np.array([l[0] for l in sc.lights])))
    for t, s, p, L in cases:
        host = _records(t, s, p, L)
        dev = np.zeros_like(host)
        tt = np.ascontiguousarray(t, np.float64)
        pp = np.ascontiguousarray(p, np.float64)
        lp = np.ascontiguousarray(L, np.float64)
        assert _lib().mirt_debug_light_table_gpu(ctx.handle, tt.ctypes.data, len(t), s, pp.ctypes.data, lp.ctypes.data,
                                                 len(L), dev.ctypes.data) == 0
        assert host.tobytes() == dev.tobytes()


def _cache_stats(ctx):
    out = np.zeros(8, np.uint64)
    assert _lib().mirt_light_cache_stats(ctx.handle, out.ctypes.data) == 0
    return dict(zip(("builds", "hits", "evictions", "fallbacks", "reused", "live", "bytes", "cap"), map(int, out)))


@pytest.mark.gpu
def test_light_cache_cycles_more_keys_than_fit(ctx):
    """Lights moving every frame with a cache that holds three tables: 40 light sets, each
    traced twice in a row, then the first ones again.  Every frame equals the oracle; tables
    are built on the device, reused on a repeat, evicted (least recently used, once their
    readers are done) and their buffers reused; frames that find no room are counted."""
    import dataclasses
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.tracer import Light
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    sc = load_scene(SCENE)
    env = rt.Environment.from_file(SCENE, ctx)
    base = env.mutable()
    n_tri = len(sc.meshes[0].face_v)
    one = len(sc.lights) * n_tri * 64
    W, H = 48, 36
    s0 = _cache_stats(ctx)
    _lib().mirt_set_light_cache(ctx.handle, 3 * one + 1024)
    rng = np.random.default_rng(9)
    keys = [[(tuple(np.array(p) + rng.normal(size=3) * 0.5), c) for p, c in sc.lights] for _ in range(40)]
    try:
        for k in list(range(40)) + list(range(4)):
            lights = keys[k]
            mut = dataclasses.replace(base, lights=[Light(pos=p, col=c) for p, c in lights])
            sck = dataclasses.replace(sc, lights=lights)
            ref = Oracle(sck, culling="rtree").frame(W, H, nthreads=8)
            for _ in range(2):
                fb = rt.draw(env, W, H, mut)
                assert np.array_equal(fb.rgb, ref["rgb"]) and np.array_equal(fb.valid, ref["valid"]), k
        st = _cache_stats(ctx)
        d = {k: st[k] - s0[k] for k in ("builds", "hits", "evictions", "fallbacks", "reused")}
        # (tables of the last 16 calls are never evicted, so some frames find no room here)
        assert d["builds"] > 3 and d["hits"] > 3 and d["evictions"] > 0 and d["reused"] > 0, d
        assert st["bytes"] <= 3 * one + 1024 and st["live"] <= 3
    finally:
        _lib().mirt_set_light_cache(ctx.handle, 4 << 30)


@pytest.mark.gpu
def test_light_table_pinned_by_open_batch(ctx):
    """A frame staged in a group's open batch holds its light table (LightTab::pins) until the
    batch launches: 24 synchronous frames with other light sets on the same context, under a
    cache that holds two tables, must neither evict it nor hand its buffer to another key.  The
    staged frame, flushed afterwards, equals the oracle; so does every frame in between."""
    import dataclasses
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    from distributed_raytracer_amd.tracer import Light
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    sc = load_scene(SCENE)
    env = rt.Environment.from_file(SCENE, ctx)
    base = env.mutable()
    n_tri = len(sc.meshes[0].face_v)
    one = len(sc.lights) * n_tri * 64
    W, H = 48, 36
    rng = np.random.default_rng(21)
    keys = [[(tuple(np.array(p) + rng.normal(size=3) * 0.5), c) for p, c in sc.lights] for _ in range(25)]

    def mut_of(k):
        return dataclasses.replace(base, lights=[Light(pos=p, col=c) for p, c in keys[k]])

    def ref_of(k):
        return Oracle(dataclasses.replace(sc, lights=keys[k]), culling="rtree").frame(W, H, nthreads=8)

    s0 = _cache_stats(ctx)
    _lib().mirt_set_light_cache(ctx.handle, 2 * one + 1024)
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=4, batch=4, with_rgb=True)
    try:
        idx = g.render(mut_of(0).to_frame())  # staged: the batch holds 1 of 4 frames
        for k in range(1, 25):
            fb = rt.draw(env, W, H, mut_of(k))
            ref = ref_of(k)
            assert np.array_equal(fb.rgb, ref["rgb"]) and np.array_equal(fb.valid, ref["valid"]), k
        st = _cache_stats(ctx)
        assert st["evictions"] > s0["evictions"]  # the other keys did cycle through the cache
        g.wait()
        g.flush()
        torch.cuda.synchronize()
        dev = g.frames[idx % 4]
        ref = ref_of(0)
        assert np.array_equal(dev.rgb.cpu().numpy(), ref["rgb"])
        assert np.array_equal(dev.valid.cpu().numpy().astype(bool), ref["valid"].astype(bool))
        # the staged key was never rebuilt: its table survived the 24 other frames
        d = _cache_stats(ctx)
        assert d["fallbacks"] - s0["fallbacks"] < 24, d
    finally:
        g.close()
        _lib().mirt_set_light_cache(ctx.handle, 4 << 30)
