"""Independent numpy restatement of the trace path — TEST INFRASTRUCTURE ONLY.

Written separately from rt_oracle.c so that the two restatements pin each other: they
must agree bit-for-bit (tests/test_oracle.py).  Brute force over faces, vectorised over
rays; the nearest hit is the FIRST face index reaching the minimum distance, which is
the strict-`<` scan of shared/state/object.go:97-103 in ascending face order.
Shading (tracer.go:53-77) is scalar Python floats (IEEE f64, never fused), with Go's
math.Pow / math.Tan / math.Min / math.Max restated.  Parity unpinned by the reference.
"""
from __future__ import annotations

import math

import numpy as np

from .scene_py import PyScene


# ----------------------------------------------------------- Go math (scalar)
def go_min(x, y):
    if x == -math.inf or y == -math.inf:
        return -math.inf
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if x == 0 and x == y:
        return x if math.copysign(1, x) < 0 else y
    return x if x < y else y


def go_max(x, y):
    if x == math.inf or y == math.inf:
        return math.inf
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if x == 0 and x == y:
        return y if math.copysign(1, x) < 0 else x
    return x if x > y else y


def go_pow(x: float, y: float) -> float:
    """Go math.Pow for the cases the tracer can reach (x >= 0 or NaN, finite y)."""
    if y == 0 or x == 1:
        return 1.0
    if y == 1:
        return x
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if x == 0:
        return math.inf if y < 0 else 0.0
    if y == 0.5:
        return math.sqrt(x)
    if y == -0.5:
        return 1 / math.sqrt(x)
    yf, yi = math.modf(abs(y))
    a1, ae = 1.0, 0
    if yf != 0:
        if yf > 0.5:
            yf -= 1
            yi += 1
        a1 = math.exp(yf * math.log(x))
    x1, xe = math.frexp(x)
    i = int(yi)
    while i != 0:
        if xe < -(1 << 12) or (1 << 12) < xe:
            ae += xe
            break
        if i & 1 == 1:
            a1 *= x1
            ae += xe
        x1 *= x1
        xe <<= 1
        if x1 < .5:
            x1 += x1
            xe -= 1
        i >>= 1
    if y < 0:
        a1 = 1 / a1
        ae = -ae
    return math.ldexp(a1, ae)


# ------------------------------------------------------------- vector (numpy)
def _cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _norm(a):
    mag = np.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
    return (a[0] / mag, a[1] / mag, a[2] / mag)


def _s_norm(a):
    mag = math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
    return (a[0] / mag, a[1] / mag, a[2] / mag)


def _s_len(a):
    return math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])


def _s_sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _s_add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def _s_scale(a, s):
    return (s * a[0], s * a[1], s * a[2])


def _s_dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _s_cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


class NpOracle:
    def __init__(self, scene: PyScene, chunk: int = 256):
        self.sc = scene
        self.chunk = chunk
        self.cam_pos = tuple(scene.cam_pos)
        d = scene.cam_dir
        up = (0.0, 1.0, 0.0)
        c = _s_cross(d, up)
        if c == (0.0, 0.0, 0.0):
            raise ValueError("camera dir parallel to global up")
        self.fwd = _s_norm(d)
        self.left = _s_norm(c)
        self.up = _s_cross(self.left, self.fwd)
        self.tris = []
        for m in scene.meshes:
            V = m.vertices
            P1, P2, P3 = V[m.face_v[:, 0]], V[m.face_v[:, 1]], V[m.face_v[:, 2]]
            self.tris.append((P1, P2, P3))

    # ---- object.go:63-110 for a batch of rays against one object, brute force
    def _object_hits(self, oi, O, D):
        mi, pos = self.sc.objects[oi]
        m = self.sc.meshes[mi]
        P1, P2, P3 = self.tris[mi]
        O = [O[:, k] - pos[k] for k in range(3)]  # rOrigin.Sub(o.Pos)
        D = [D[:, k] for k in range(3)]
        R = len(O[0])
        ok = np.zeros(R, bool)
        best_face = np.full(R, -1, np.int64)
        best_t = np.zeros(R)
        best_bc = np.zeros((R, 3))
        if len(P1) == 0:
            return ok, best_face, best_t, best_bc, O
        with np.errstate(all="ignore"):
            o = [x[:, None] for x in O]
            d = [x[:, None] for x in D]
            p1 = [P1[None, :, k] for k in range(3)]
            e1 = [P2[None, :, k] - P1[None, :, k] for k in range(3)]
            e2 = [P3[None, :, k] - P1[None, :, k] for k in range(3)]
            neg = [-1.0 * x for x in d]
            c = _cross(e2, neg)
            inc = _dot(e1, c)
            p1or = [o[k] - p1[k] for k in range(3)]
            r2 = _dot(p1or, c) / inc
            r3 = _dot(e1, _cross(p1or, neg)) / inc
            s = r2 + r3
            r1 = 1.0 - r2 - r3
            t = _dot(e1, _cross(e2, p1or)) / inc
            hit = (inc != 0.0) & (0.0 <= r2) & (r2 <= 1.0) & (0.0 <= s) & (s <= 1.0) & \
                (r1 >= 0.0) & (r2 >= 0.0) & (r3 >= 0.0) & (t >= 0.0)
            ip = [o[k] + t * d[k] for k in range(3)]
            dx = [o[k] - ip[k] for k in range(3)]
            dist = np.sqrt(dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2])
            dist = np.where(hit, dist, np.inf)
        ok = hit.any(axis=1)
        f = np.argmin(dist, axis=1)
        rows = np.arange(R)
        best_face = np.where(ok, f, -1)
        best_t = t[rows, f]
        best_bc = np.stack([r1[rows, f], r2[rows, f], r3[rows, f]], axis=1)
        return ok, best_face, best_t, best_bc, O

    def _trace(self, O, D):
        """tracer.go:27-50 for a batch: returns per ray (ok, obj, face, hit(world), normal)."""
        R = len(O)
        ok = np.zeros(R, bool)
        obj = np.full(R, -1, np.int64)
        face = np.full(R, -1, np.int64)
        hitw = np.zeros((R, 3))
        nrm = np.zeros((R, 3))
        bestd = np.zeros(R)
        for oi, (mi, pos) in enumerate(self.sc.objects):
            m = self.sc.meshes[mi]
            P1, P2, P3 = self.tris[mi]
            for s in range(0, R, self.chunk):
                sl = slice(s, s + self.chunk)
                h, f, t, bc, Oo = self._object_hits(oi, O[sl], D[sl])
                for r in np.nonzero(h)[0]:
                    gi = s + r
                    fi = int(f[r])
                    o = (Oo[0][r], Oo[1][r], Oo[2][r])
                    d = (D[gi, 0], D[gi, 1], D[gi, 2])
                    tt = float(t[r])
                    ip = _s_add(o, _s_scale(d, tt))
                    if len(m.normals):
                        n1, n2, n3 = (tuple(m.normals[m.face_n[fi, k]]) for k in range(3))
                        b = bc[r]
                        nv = _s_norm(_s_add(_s_add(_s_scale(n1, float(b[0])), _s_scale(n2, float(b[1]))),
                                            _s_scale(n3, float(b[2]))))
                    else:
                        nv = _s_norm(_s_cross(_s_sub(tuple(P2[fi]), tuple(P1[fi])),
                                              _s_sub(tuple(P3[fi]), tuple(P1[fi]))))
                    w = _s_add(ip, pos)
                    dd = _s_len(_s_sub(w, self.cam_pos))
                    if not ok[gi] or dd < bestd[gi]:
                        ok[gi] = True
                        bestd[gi] = dd
                        obj[gi] = oi
                        face[gi] = fi
                        hitw[gi] = w
                        nrm[gi] = nv
        return ok, obj, face, hitw, nrm

    def frame(self, W: int, H: int, tan_half_fov: float, shade: bool = True):
        """Full framebuffer, pixel (i, j) at i*H + j (worker/sequential/main.go:21-28)."""
        i = np.repeat(np.arange(W), H)
        j = np.tile(np.arange(H), W)
        hw, hh = W // 2, H // 2
        phw = tan_half_fov
        phh = phw * float(H) / float(W)
        si = phw * ((hw - i).astype(np.float64) - 0.5) / float(hw)
        sj = phh * ((hh - j).astype(np.float64) - 0.5) / float(hh)
        cp, f, l, u = self.cam_pos, self.fwd, self.left, self.up
        base = [cp[k] + f[k] for k in range(3)]
        p = [(base[k] + si * l[k]) + sj * u[k] for k in range(3)]
        dv = _norm([p[k] - cp[k] for k in range(3)])
        D = np.stack(dv, axis=1)
        O = np.tile(np.array(cp, np.float64), (len(i), 1))
        ok, obj, face, hitw, nrm = self._trace(O, D)
        n = W * H
        rgb = np.zeros((n, 3))
        if shade:
            for px in np.nonzero(ok)[0]:
                rgb[px] = self._phong(int(obj[px]), int(face[px]), tuple(hitw[px]), tuple(nrm[px]))
        return dict(valid=ok.astype(np.uint8), face=np.where(ok, face, -1).astype(np.int32),
                    obj=np.where(ok, obj, -1).astype(np.int32), rgb=rgb)

    def _phong(self, oi, fi, hit, normal):
        mi, _ = self.sc.objects[oi]
        m = self.sc.meshes[mi]
        mt = m.materials[m.face_mat[fi]]
        ka, kd, ks, ns = tuple(mt[0:3]), tuple(mt[3:6]), tuple(mt[6:9]), float(mt[9])
        col = [float(x) for x in ka]
        for lpos, lcol in self.sc.lights:
            ldir = _s_norm(_s_sub(lpos, hit))
            origin = _s_add(hit, _s_scale(ldir, 0.0001))
            sok, _, _, shit, _ = self._trace(np.array([origin]), np.array([ldir]))
            if not sok[0] or _s_len(_s_sub(lpos, hit)) < _s_len(_s_sub(tuple(shit[0]), hit)):
                refl = _s_sub(_s_scale(normal, 2 * _s_dot(ldir, normal)), ldir)
                camdir = _s_norm(_s_sub(self.cam_pos, hit))
                dfac = go_max(_s_dot(ldir, normal), 0.0)
                sfac = go_pow(go_max(_s_dot(refl, camdir), 0.0), ns)
                for k in range(3):
                    dk = go_max(0.0, go_min(dfac * float(kd[k]), 1.0)) * lcol[k]
                    col[k] = go_min(col[k] + dk, 1.0)
                for k in range(3):
                    sk = go_max(0.0, go_min(sfac * float(ks[k]), 1.0)) * lcol[k]
                    col[k] = go_min(col[k] + sk, 1.0)
        return col
