"""Host-side checks that need no GPU: the C-ABI library loads and exports every declared
symbol, the C++ loader matches the independent Python loader, the Go-math / camera
restatements agree, and the tile planning / assembly logic is consistent."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared_functions():
    names = set()
    for h in ("mirt.h", "mirt_scene.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(mirt_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    import distributed_raytracer_amd._lib as L
    lib = L.lib()
    names = _declared_functions()
    assert len(names) >= 25
    for n in sorted(names):
        assert hasattr(lib, n), f"libmirt.so does not export {n}"
    assert names == set(L.SIGNATURES), "ctypes signatures out of sync with include/*.h"
    assert lib.mirt_abi_version() == 7


def test_no_gpu_is_a_loud_error():
    """Without a HIP device the product raises; it never falls back to a CPU path."""
    import torch
    import distributed_raytracer_amd as rt
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rt.MirtError) as e:
        rt.Context(0)
    assert e.value.code == -2


def test_cpp_loader_matches_python_loader(scene_path, py_scene):
    import distributed_raytracer_amd as rt
    meshes, objects, lights, cam = rt.load_scene_arrays(scene_path)
    a, b = meshes[0], py_scene.meshes[0]
    for k in ("vertices", "normals", "face_v", "face_n", "face_mat", "materials"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert [(m, tuple(p)) for m, p in objects] == py_scene.objects
    assert [(l.pos, l.col) for l in lights] == py_scene.lights


OBJ_VARIANTS = """mtllib mats.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 0.5 1
v 0 0 0
vn 0 0 1
vn 0 0 2
vn 1 1 1
usemtl red
f 1//1 2//1 3//2 4//2
f 1//3 2//3 5//3
usemtl nosuch
f -6//-1 -5//-2 -2//-3
usemtl blue
f 2 3 5 4 1
"""
MTL = """newmtl red
Ka 0.2 0 0
Kd 1.5 0.3 -0.2
Ks 0.1 0.1 0.1
Ns 32.5
newmtl blue
Kd 0 0 1
"""


def test_loaders_agree_on_obj_variants(tmp_path):
    """quads, a pentagon, negative indices, faces without normals, unknown usemtl
    (default material), MTL values outside [0,1] (clamped), duplicate positions."""
    import distributed_raytracer_amd as rt
    from oracle.scene_py import load_scene
    (tmp_path / "m.obj").write_text(OBJ_VARIANTS)
    (tmp_path / "mats.mtl").write_text(MTL)
    (tmp_path / "s.json").write_text('{"objs":[{"model":"m.obj","pos":{"x":0,"y":0,"z":-3}},'
                                     '{"MODEL":"m.obj","Pos":{"X":1,"Y":0,"Z":-4}}],'
                                     '"lights":[{"pos":{"x":1,"y":2,"z":3},"col":{"r":255,"g":128,"b":0}}],'
                                     '"cam":{"pos":{"x":0,"y":0,"z":2},"dir":{"x":0,"y":0,"z":-1},"fov":1.0}}')
    meshes, objects, lights, cam = rt.load_scene_arrays(str(tmp_path / "s.json"))
    ps = load_scene(str(tmp_path / "s.json"))
    assert len(meshes) == 1 and len(objects) == 2 and objects[1][0] == 0
    a, b = meshes[0], ps.meshes[0]
    for k in ("vertices", "normals", "face_v", "face_n", "face_mat", "materials"):
        x, y = getattr(a, k), getattr(b, k)
        assert x.shape == y.shape and np.array_equal(x, y, equal_nan=x.dtype.kind == "f"), k
    assert np.isnan(a.normals).any()  # the face without normal indices: Norm(0,0,0) = NaN
    assert len(a.face_v) == 2 + 1 + 1 + 3
    assert a.vertices.shape == (5, 3)  # v 6 duplicates v 1
    mats = {tuple(m) for m in a.materials}
    assert (16 / 255, 16 / 255, 16 / 255, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0) in mats
    red = [m for m in a.materials if m[9] == 32.5][0]
    assert red[3] == 1.0 and red[5] == 0.0  # Kd clamped to [0, 1]
    assert lights[0].col == (1.0, 128 / 255, 0.0)


# decimal strings within half a float64 ulp of a float32 halfway point: rounding them to
# float64 first and then to float32 gives the neighbouring float32 (found by exact search)
NEAR_HALFWAY = {"-1.462542951107025136484375": -1.4625428915023804, "1.389735043048858652578125": 1.3897351026535034}


def test_float32_parse_rounds_once(tmp_path):
    """gwob parses with strconv.ParseFloat(s, 32): one correct rounding to float32.  Both
    loaders must agree with the exact rounding where float32(float64(s)) does not."""
    import distributed_raytracer_amd as rt
    from fractions import Fraction
    from oracle.scene_py import _f32, load_scene
    for s, want in NEAR_HALFWAY.items():
        assert float(np.float32(float(s))) != want  # the double-rounded value is the other float32
        assert _f32(s) == want
        lo = np.nextafter(np.float32(want), np.float32(-np.inf))
        hi = np.nextafter(np.float32(want), np.float32(np.inf))
        d = abs(Fraction(want) - Fraction(s))
        assert d <= abs(Fraction(float(lo)) - Fraction(s)) and d <= abs(Fraction(float(hi)) - Fraction(s))
    a, b = list(NEAR_HALFWAY)
    (tmp_path / "h.obj").write_text(f"v {a} {b} 0.5\nv 1 0 {b}\nv {b} 1 {a}\nf 1 2 3\n")
    (tmp_path / "s.json").write_text('{"objs":[{"model":"h.obj","pos":{"x":0,"y":0,"z":0}}],"lights":[],'
                                     '"cam":{"pos":{"x":0,"y":0,"z":2},"dir":{"x":0,"y":0,"z":-1},"fov":1.0}}')
    meshes, _, _, _ = rt.load_scene_arrays(str(tmp_path / "s.json"))
    py = load_scene(str(tmp_path / "s.json")).meshes[0]
    want = np.array([[NEAR_HALFWAY[a], NEAR_HALFWAY[b], 0.5], [1, 0, NEAR_HALFWAY[b]],
                     [NEAR_HALFWAY[b], 1, NEAR_HALFWAY[a]]])
    assert np.array_equal(meshes[0].vertices, want) and np.array_equal(py.vertices, want)


def test_camera_and_go_math_match_oracle():
    import distributed_raytracer_amd as rt
    import distributed_raytracer_amd._lib as L
    from oracle.oracle import go_pow, go_tan, new_camera
    rng = np.random.default_rng(5)
    for _ in range(200):
        pos, d, fov = rng.normal(size=3), rng.normal(size=3), float(rng.uniform(0.1, 3.0))
        cam = rt.Camera.new(pos, d, fov)
        f, l, u = new_camera(pos, d)
        assert cam.forward == tuple(f) and cam.left == tuple(l) and cam.up == tuple(u)
        assert cam.proj_half_width == go_tan(fov / 2)
    for x in rng.uniform(-1.5, 1.5, 5000):
        assert L.lib().mirt_go_tan(float(x)) == go_tan(float(x))
    for x, y in zip(rng.random(5000), rng.integers(0, 50, 5000)):
        assert L.lib().mirt_go_pow(float(x), float(y)) == go_pow(float(x), float(y))
    # the small-integer-exponent path and its edges (x in [2^-60, 16], 2 <= y <= 16)
    xs = np.concatenate([rng.uniform(0, 16.5, 3000), 2.0 ** rng.uniform(-70, -50, 500),
                         [2.0 ** -60, np.nextafter(2.0 ** -60, 0), 16.0, np.nextafter(16.0, 99), 1.0, 0.5, 0.0, -0.0]])
    for x in xs:
        for y in (2.0, 3.0, 7.0, 10.0, 16.0, 17.0, 2.5):
            assert L.lib().mirt_go_pow(float(x), y) == go_pow(float(x), y), (x, y)
    with pytest.raises(rt.MirtError) as e:
        rt.Camera.new((0, 0, 0), (0, 3, 0), 1.0)
    assert e.value.code == L.MIRT_E_CAMERA


def test_constant_operand_min_max_are_go_min_max():
    """colour.go's clamps with a constant operand (go_min1 = Min(a, 1), go_max0 = Max(a, 0)
    = Max(0, a)) return Go's Min / Max result bit for bit, signed zeros and NaN included."""
    import distributed_raytracer_amd._lib as L
    from oracle.np_oracle import go_max as py_max, go_min as py_min
    f = L.lib().mirt_go_minmax
    rng = np.random.default_rng(11)
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 1.0 + 2 ** -52, 1.0 - 2 ** -53, np.inf, -np.inf, np.nan, 5e-324, -5e-324,
            1e308, -1e308] + list(rng.normal(size=200)) + list(rng.uniform(0.9, 1.1, 200))
    same = lambda a, b: (np.isnan(a) and np.isnan(b)) or (a == b and np.signbit(a) == np.signbit(b))  # noqa: E731
    for a in vals:
        a = float(a)
        assert same(f(2, a, 0.0), f(0, a, 1.0)) and same(f(0, a, 1.0), py_min(a, 1.0)), a
        assert same(f(3, a, 0.0), f(1, a, 0.0)) and same(f(3, a, 0.0), f(1, 0.0, a)), a
        assert same(f(1, a, 0.0), py_max(a, 0.0)) and same(f(1, 0.0, a), py_max(0.0, a)), a


def test_tile_deal_spreads_rows_and_columns():
    """assign(): column c of tile row r goes to rank (c + skew * r) % world; every rank
    holds tiles in every row band and in many columns."""
    from distributed_raytracer_amd.framebuffer import assign, plan_tiles, skew
    assert [skew(n) for n in (1, 2, 3, 4, 6, 8)] == [1, 3, 2, 3, 5, 3]
    tiles = plan_tiles(1920, 1080, 32)
    for world in (2, 3, 8):
        for r in range(world):
            mine = assign(tiles, world, r)
            assert len({y for _, y, _, _ in mine}) == 34  # every tile row
            assert len({x for x, _, _, _ in mine}) == 60  # every tile column (skew spreads columns)
            assert all(((x // 32) + skew(world) * (y // 32)) % world == r for x, y, _, _ in mine)


def test_tile_plan_covers_screen_once():
    from distributed_raytracer_amd.framebuffer import assign, packed_capacity, pixels_of, plan_tiles
    for W, H, t in ((1920, 1080, 64), (320, 240, 48), (7, 5, 3), (64, 64, 64)):
        tiles = plan_tiles(W, H, t)
        cover = np.zeros((W, H), np.int32)
        for x, y, w, h in tiles:
            cover[x:x + w, y:y + h] += 1
        assert (cover == 1).all()
        for world in (1, 2, 3, 8):
            parts = [assign(tiles, world, r) for r in range(world)]
            assert sum(len(p) for p in parts) == len(tiles)
            assert packed_capacity(tiles, world) == max(pixels_of(p) for p in parts)


def test_unpack_host_inverts_packing():
    from distributed_raytracer_amd.framebuffer import plan_tiles, unpack_host
    W, H = 50, 30
    fb = np.arange(W * H * 3, dtype=np.int64).reshape(W * H, 3)
    tiles = plan_tiles(W, H, 16)[::-1]
    packed = np.concatenate([fb.reshape(W, H, 3)[x:x + w, y:y + h].reshape(-1, 3) for x, y, w, h in tiles])
    out = np.zeros_like(fb)
    unpack_host(W, H, tiles, packed, out)
    assert np.array_equal(out, fb)


def test_master_partition_restatement():
    """master/main.go:54-91: rectangles tile the screen exactly; 8 workers on 1920x1080
    gives eight 480x540 rectangles."""
    from distributed_raytracer_amd.framebuffer import master_partition
    for n in (1, 2, 3, 5, 8, 24, 100):
        parts, _ = master_partition((0, 0, 320, 240), n)
        cover = np.zeros((320, 240), np.int32)
        for x, y, w, h in parts:
            cover[x:x + w, y:y + h] += 1
        assert (cover == 1).all()
    parts, _ = master_partition((0, 0, 1920, 1080), 8)
    assert sorted(set((w, h) for _, _, w, h in parts)) == [(480, 540)] and len(parts) == 8


def test_interleaved_tiles_balance_better_than_bisection():
    """Shadow + primary work per rank on the 320x240 golden hit mask: interleaved tiles
    stay near the mean, the master's bisection does not."""
    from distributed_raytracer_amd.framebuffer import assign, master_partition, plan_tiles
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "suzanne_320x240.npz"))
    W, H = 320, 240
    hits = np.zeros((W, H), np.int64)
    hits.reshape(-1)[g["hit_index"]] = 1
    work = 1 + 3 * hits

    def imbalance(rects_per_rank):
        loads = [sum(work[x:x + w, y:y + h].sum() for x, y, w, h in rs) for rs in rects_per_rank]
        return max(loads) / (sum(loads) / len(loads))

    tiles = plan_tiles(W, H, 8)  # 1/16 of the 1080p frame's pixels: the bench's 32-px tiles scaled down
    inter = imbalance([assign(tiles, 8, r) for r in range(8)])
    bis = imbalance([[p] for p in master_partition((0, 0, W, H), 8)[0]])
    assert inter < 1.05 < bis


def test_native_tile_deal_equals_python():
    """mirt_plan_tiles (the C++ deal of mirt_group) == assign(plan_tiles(...))."""
    from distributed_raytracer_amd.framebuffer import assign, plan_rank_tiles_native, plan_tiles
    for W, H, t, th in ((1920, 1080, 32, None), (1920, 1080, 64, None), (320, 240, 48, None), (7, 5, 3, None),
                        (1920, 1080, 8, 0), (320, 240, 16, 0), (1920, 1080, 32, 16)):
        tiles = plan_tiles(W, H, t, th)
        for world in (1, 2, 3, 4, 6, 8):
            for r in range(world):
                assert plan_rank_tiles_native(W, H, t, world, r, th) == assign(tiles, world, r), (W, H, t, th, world, r)


def test_group_deal_weights_the_root_down():
    """mirt_group_plan_tiles: every tile exactly once over the ranks; rank 0 (which also
    unpacks every frame) holds (b - 1) / (b N - 1) of the deal slots, the others b / (b N - 1),
    b = round(32 / N); world 1 is the whole tile list."""
    from distributed_raytracer_amd.framebuffer import plan_group_tiles, plan_tiles
    for W, H, t, th in ((1920, 1080, 8, 0), (1920, 1080, 32, 32), (320, 240, 16, 0), (7, 5, 3, 3)):
        tiles = plan_tiles(W, H, t, th)
        assert plan_group_tiles(W, H, t, 1, 0, th) == tiles
        for world in (2, 3, 4, 8):
            parts = [plan_group_tiles(W, H, t, world, r, th) for r in range(world)]
            assert sorted(x for p in parts for x in p) == sorted(tiles), (W, H, t, th, world)
    b = 4  # N = 8
    strips = [plan_group_tiles(1920, 1080, 8, 8, r, 0) for r in range(8)]
    n = [len(p) for p in strips]  # 240 strips, 31-slot pattern
    assert abs(n[0] / 240 - (b - 1) / 31) < 0.02 and all(abs(k / 240 - b / 31) < 0.02 for k in n[1:])
