"""BASELINE.json configs[3] input: a synthetic 1,000,000-triangle OBJ.

UV sphere of radius 1.2 centred at the origin (placed like suzanne by scene.json's object
position): `stacks` x `slices` cells (default 500 x 1000), every cell emitted as two
explicit `f` triangles, so the file holds exactly 2 * stacks * slices faces.  The pole
cells give zero-area triangles: legal, and never hit (their Möller–Trumbore incidence
is exactly 0).  Per-vertex unit normals (`vn`), coordinates written with `%.6f` like
Blender so the loaders' float32 parse is the same on every path.  Deterministic: the
`seed` only perturbs nothing unless --jitter is given (kept for the configs[3] recipe,
seed = 1234).

usage: python tools/gen_sphere_obj.py OUT_DIR [--stacks 500 --slices 1000]
writes OUT_DIR/sphere.obj, OUT_DIR/sphere.mtl and OUT_DIR/scene.json (a copy of the
reference's example/scene.json with the model replaced).
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(ROOT, "tests", "golden", "example")


def sphere_arrays(stacks: int, slices: int, radius: float = 1.2, seed: int = 1234, jitter: float = 0.0):
    rng = np.random.default_rng(seed)
    th = np.linspace(0.0, np.pi, stacks + 1)          # polar angle, rows 0..stacks
    ph = np.linspace(0.0, 2.0 * np.pi, slices + 1)    # azimuth, columns 0..slices (seam duplicated)
    T, P = np.meshgrid(th, ph, indexing="ij")
    n = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], axis=-1).reshape(-1, 3)
    if jitter:
        n = n + rng.normal(scale=jitter, size=n.shape)
        n /= np.linalg.norm(n, axis=1, keepdims=True)
    v = radius * n
    idx = np.arange((stacks + 1) * (slices + 1)).reshape(stacks + 1, slices + 1)
    a, b = idx[:-1, :-1], idx[:-1, 1:]
    c, d = idx[1:, :-1], idx[1:, 1:]
    f1 = np.stack([a, c, d], axis=-1).reshape(-1, 3)
    f2 = np.stack([a, d, b], axis=-1).reshape(-1, 3)
    faces = np.empty((2 * stacks * slices, 3), np.int64)
    faces[0::2] = f1
    faces[1::2] = f2
    return v, n, faces


def write(out_dir: str, stacks: int = 500, slices: int = 1000, seed: int = 1234, jitter: float = 0.0) -> str:
    os.makedirs(out_dir, exist_ok=True)
    v, n, f = sphere_arrays(stacks, slices, seed=seed, jitter=jitter)
    obj = os.path.join(out_dir, "sphere.obj")
    with open(obj, "w") as fh:
        fh.write(f"# synthetic UV sphere {stacks}x{slices}, {len(f)} triangles (tools/gen_sphere_obj.py)\n")
        fh.write("mtllib sphere.mtl\no Sphere\n")
        fh.write("".join(f"v {x:.6f} {y:.6f} {z:.6f}\n" for x, y, z in v))
        fh.write("".join(f"vn {x:.4f} {y:.4f} {z:.4f}\n" for x, y, z in n))
        fh.write("usemtl Material\ns 1\n")
        f1 = f + 1
        fh.write("".join(f"f {a}//{a} {b}//{b} {c}//{c}\n" for a, b, c in f1))
    with open(os.path.join(out_dir, "sphere.mtl"), "w") as fh:
        fh.write(open(os.path.join(EXAMPLE, "suzanne.mtl")).read())
    scene = json.load(open(os.path.join(EXAMPLE, "scene.json")))
    scene["objs"][0]["model"] = "sphere.obj"
    with open(os.path.join(out_dir, "scene.json"), "w") as fh:
        json.dump(scene, fh, indent=1)
    return os.path.join(out_dir, "scene.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--stacks", type=int, default=500)
    ap.add_argument("--slices", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--jitter", type=float, default=0.0)
    a = ap.parse_args()
    print(write(a.out_dir, a.stacks, a.slices, a.seed, a.jitter))


if __name__ == "__main__":
    main()
