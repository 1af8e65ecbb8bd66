"""Cost model of the Box.Intersect gate's plane order, on the CPU.

Traces the driver's frame (a 480x270 sample of suzanne's 1080p camera) and its three shadow
rays per hit with the oracle, takes each ray's winning face box and the object box, and counts
per 64-ray wave how many exact plane evaluations (box.go:29-68) each plane order needs until
every lane is proven (1 unit = one far-plane body; the old run-time-axis loop costs 2 units
per plane):
  old   : the lean axis's far plane, then the six planes in a fixed order (run-time axis)
  far   : the lean axis's far plane, the other far planes, then the near planes (the kernel's)
  python tests/gate_order_model.py     (tests/test_gate_order.py asserts the comparison)
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # the repo (this file is in tests/)
sys.path.insert(0, ROOT)
from oracle.oracle import Oracle  # noqa: E402  (test infrastructure: the checker's traces)
from oracle.scene_py import load_scene  # noqa: E402


def plane(box, o, d, a, hi):
    b, c = [x for x in range(3) if x != a]
    with np.errstate(divide="ignore", invalid="ignore"):
        ds = ((box[:, 3 + a] if hi else box[:, a]) - o[:, a]) / d[:, a]
        ib = o[:, b] + ds * d[:, b]
        ic = o[:, c] + ds * d[:, c]
    return ((d[:, a] != 0) & (ds >= 0) & (box[:, b] <= ib) & (ib <= box[:, 3 + b]) & (box[:, c] <= ic)
            & (ic <= box[:, 3 + c]))


def side(box, o, d, a, far):
    pos = d[:, a] > 0
    return np.where(pos == far, plane(box, o, d, a, True), plane(box, o, d, a, False))


def cost(box, o, d):
    P = [plane(box, o, d, q >> 1, (q & 1) == 0) for q in range(6)]
    F = [side(box, o, d, a, True) for a in range(3)]
    N = [side(box, o, d, a, False) for a in range(3)]
    old = new = 0.0
    waves = 0
    for w0 in range(0, len(o), 64):
        sl = slice(w0, min(len(o), w0 + 64))
        waves += 1
        a = int(np.argmax(np.abs(d[w0])))
        r = F[a][sl].copy()
        old += 1
        ro = r.copy()
        for q in range(6):
            if ro.all():
                break
            old += 2
            ro |= P[q][sl]
        new += 1
        for A in [x for x in range(3) if x != a] + [None, 0, 1, 2]:
            if r.all():
                break
            if A is None:
                continue
            new += 1
            r |= (F if A != a or new < 3 else N)[A][sl]
    return round(old / waves, 2), round(new / waves, 2)


def model(W: int = 480, H: int = 270):
    """{query: (face (old, far-first), object (old, far-first))} per-wave plane evaluations."""
    sc = load_scene(os.path.join(ROOT, "tests", "golden", "example", "scene.json"))
    orc = Oracle(sc, culling="rtree")
    cam = np.array(sc.cam_pos)
    fwd = np.array(sc.cam_dir) / np.linalg.norm(sc.cam_dir)
    left = np.cross([0, 1.0, 0], fwd)
    left /= np.linalg.norm(left)
    up = np.cross(fwd, left)
    th = math.tan(sc.fov / 2)
    ii, jj = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    s = th * ((W / 2 - ii) - 0.5) / (W / 2)
    t = th * (H / W) * ((H / 2 - jj) - 0.5) / (H / 2)
    d = fwd[None] + left[None] * s.reshape(-1, 1) + up[None] * t.reshape(-1, 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(cam[None], len(d), 0)
    pos = np.array(sc.objects[0][1], np.float64)

    out = {}

    def run(name, o, d):
        r = orc.trace_rays(o, d)
        hit = r["ok"].astype(bool)
        fb = np.array([orc.face_box(0, f) for f in r["face"][hit]])
        ob = np.repeat(orc.object_box(0)[None], hit.sum(), 0)
        out[name] = (cost(fb, o[hit] - pos, d[hit]), cost(ob, o[hit], d[hit]))
        return r

    r = run("primary", o, d)
    hit = r["ok"].astype(bool)
    for li, (lp, _) in enumerate(sc.lights):
        hp = r["hit"][hit]
        L = np.array(lp) - hp
        L /= np.linalg.norm(L, axis=1, keepdims=True)
        run(f"shadow{li}", hp + L * 1e-4, L)
    return out


if __name__ == "__main__":
    for k, (f, ob) in model().items():
        print(f"{k:8s} plane evaluations per wave (old, far-first): face box {f}  object box {ob}")
