"""Generate the gob wire fixtures (tests/golden/gob/*.gob) — TEST INFRASTRUCTURE ONLY.

The bytes a reference master would send to a worker, written by the Go-gob encoder
restatement tests/golden/gob_go.py (no Go toolchain here: PARITY UNPINNED against a real
Go encoder; the encoder itself is pinned by the encoding/gob documentation's own vectors in
tests/test_gob.py).  Each scene gives:
  <name>_state.gob  MasterState.state of Register (master/registrar.go:30-50): gob(Environment)
  <name>_diff.gob   WorkOrder.diff of one frame (master/main.go:260-263): gob(EnvMutables)
Scenes: the reference's example/ (suzanne, 3 lights), and the four-object synthetic scene of
tests/scenes.py (suzanne twice, a cube without vertex normals, a sphere; 4 lights) whose diff
also carries an object whose id links to no mesh (LinkTo leaves its mesh nil).

    python tests/golden/make_gob.py
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import gob_go as G  # noqa: E402
from oracle.scene_py import load_scene  # noqa: E402

OUT = os.path.join(HERE, "gob")
SCENE = os.path.join(HERE, "example", "scene.json")


def master_side(sc, model_names):
    """The master's Environment for a PyScene (environment.go:162-234): object i gets id
    i + 1; one mesh per model path; lights NewRGB(u8); camera NewCamera(pos, dir, fov)."""
    meshes = {model_names[k]: m for k, m in enumerate(sc.meshes)}
    paths = {i + 1: model_names[mi] for i, (mi, _) in enumerate(sc.objects)}
    objects = [(pos, i + 1) for i, (_, pos) in enumerate(sc.objects)]
    cam = (sc.cam_pos, G.norm(sc.cam_dir), sc.fov)  # Camera.MarshalBinary sends forward = dir.Norm()
    return meshes, paths, objects, list(sc.lights), cam


def write(name: str, state: bytes, diff: bytes) -> None:
    os.makedirs(OUT, exist_ok=True)
    for suffix, data in (("state", state), ("diff", diff)):
        with open(os.path.join(OUT, f"{name}_{suffix}.gob"), "wb") as fh:
            fh.write(data)
        print(f"{name}_{suffix}.gob: {len(data)} bytes")


def main() -> None:
    from scenes import multi_object_scene

    sc = load_scene(SCENE)
    meshes, paths, objects, lights, cam = master_side(sc, ["suzanne.obj"])
    write("example", G.register_state(meshes, paths), G.work_order_diff(objects, lights, cam))

    ms = multi_object_scene(sc.meshes[0])
    names = ["suzanne.obj", "cube.obj", "sphere.obj"]
    meshes, paths, objects, lights, cam = master_side(ms, names)
    objects.append(((0.0, 5.0, -3.0), 99))  # an id with no path: linked to no mesh
    write("multi", G.register_state(meshes, paths), G.work_order_diff(objects, lights, cam))


if __name__ == "__main__":
    main()
