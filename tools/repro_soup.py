"""Trace one vertex-light soup (tests/scenes.py) with the given options and compare with the
R-tree oracle: python tools/repro_soup.py SEED OPTS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import distributed_raytracer_amd as rt
    from oracle.oracle import Oracle
    from scenes import gpu_env, soup_scene
    seed, opts = int(sys.argv[1]), int(sys.argv[2])
    ctx = rt.Context(0)
    sc = soup_scene(seed, vertex_light=True)
    env = gpu_env(ctx, sc)
    ctx.set_options(opts)
    ctx.profile_enable(True)
    fb = rt.draw(env, 64, 48)
    p = ctx.profile_read()
    ref = Oracle(sc, culling="rtree").frame(64, 48, nthreads=8)
    ok = all(np.array_equal(getattr(fb, k), ref[k]) for k in ("valid", "rgb"))
    print(f"seed {seed} opts {opts}: equal={ok} redo_items={p['redo_items']} hits={int(fb.valid.sum())}", flush=True)


if __name__ == "__main__":
    main()
