"""Generate the committed golden vectors from the oracle (tests/golden/*.npz).

The reference (Go) cannot be built or run here, and ships no golden vectors, so these
fixtures come from the C restatement (oracle/rt_oracle.c), which must first agree
bit-for-bit with the independent numpy restatement (oracle/np_oracle.py) on every pixel
that numpy also traces.  Inputs: tests/golden/example/ = the reference's example/
scene (scene.json, suzanne.obj, suzanne.mtl, byte-identical data files).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.np_oracle import NpOracle  # noqa: E402
from oracle.oracle import Oracle, go_tan  # noqa: E402
from oracle.scene_py import load_scene  # noqa: E402

SCENE = os.path.join(HERE, "example", "scene.json")


def main() -> None:
    sc = load_scene(SCENE)
    orc = Oracle(sc)
    npo = NpOracle(sc)
    # 64x48: full planes, cross-checked against numpy on every pixel
    r = orc.frame(64, 48)
    q = npo.frame(64, 48, go_tan(sc.fov / 2))
    assert np.array_equal(r["valid"], q["valid"]) and np.array_equal(r["face"], q["face"])
    assert np.array_equal(r["rgb"], q["rgb"]), "C and numpy restatements disagree"
    np.savez_compressed(os.path.join(HERE, "suzanne_64x48.npz"), W=64, H=48, valid=r["valid"], face=r["face"],
                        obj=r["obj"], rgb=r["rgb"], rgb8=r["rgb8"])
    # 320x240 (configs[0] size): hit pixels only; numpy cross-check on the same frame
    r = orc.frame(320, 240, nthreads=8)
    q = npo.frame(320, 240, go_tan(sc.fov / 2))
    assert np.array_equal(r["valid"], q["valid"]) and np.array_equal(r["face"], q["face"])
    assert np.array_equal(r["rgb"], q["rgb"]), "C and numpy restatements disagree"
    hit = np.nonzero(r["valid"])[0].astype(np.uint32)
    np.savez_compressed(os.path.join(HERE, "suzanne_320x240.npz"), W=320, H=240, hit_index=hit,
                        face=r["face"][hit], rgb=r["rgb"][hit], rgb8=r["rgb8"][hit],
                        primary_rays=r["stats"]["primary_rays"], shadow_rays=r["stats"]["shadow_rays"])
    print("wrote golden fixtures:", int(len(hit)), "hits at 320x240")


if __name__ == "__main__":
    main()
