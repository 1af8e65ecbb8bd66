"""Where do the cycles go?  Times the frame kernels on controlled variants of the
suzanne scene (1 GPU): the camera turned away (every ray misses: raygen, root test and
outputs only), the default view, and a close-up (mesh fills the screen).

usage (GPU box): python tools/cost_probe.py [--repeat N] [--views default,away] [--opts default,static]
Each (view, options) pair is timed N times (interleaved); the minimum is reported.
"""
import argparse
import time
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--views", default="")
    ap.add_argument("--opts", default="")
    a = ap.parse_args()
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    base = env.mutable()
    cam = base.cam
    views = {
        "default": cam,
        "away": rt.Camera.new(cam.pos, tuple(-np.asarray(cam.forward)), cam.fov),
        "closeup": rt.Camera.new(tuple(np.asarray(cam.pos) + 0.6 * (np.array([1.0, 1.0, -1.0]) - np.asarray(cam.pos))),
                                 tuple(np.array([1.0, 1.0, -1.0]) - np.asarray(cam.pos)), cam.fov),
    }
    opts = {"default": 0, "static": rt._lib.MIRT_OPT_STATIC_SCHEDULE, "no_frustum": rt._lib.MIRT_OPT_NO_FRUSTUM,
            "split": rt._lib.MIRT_OPT_SPLIT_KERNELS}
    if a.views:
        views = {k: views[k] for k in a.views.split(",")}
    if a.opts:
        opts = {k: opts[k] for k in a.opts.split(",")}
    sh = FrameSharder(ctx, 1920, 1080, 0, 1, 64)
    out = {}
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for _ in range(a.repeat):
            for vname, c in views.items():
                mut = rt.EnvMutables(base.objects, base.lights, c)
                frame = mut.to_frame()
                for oname, o in opts.items():
                    ctx.set_options(o)
                    for _ in range(5):
                        sh.render(frame)
                    torch.cuda.synchronize()
                    # steady-state frame time without profiling events
                    t0 = time.perf_counter()
                    for _ in range(50):
                        sh.render(frame)
                    torch.cuda.synchronize()
                    wall = (time.perf_counter() - t0) / 50 * 1e6
                    ctx.profile_enable(True)
                    for _ in range(30):
                        sh.render(frame)
                    torch.cuda.synchronize()
                    ctx.profile_enable(False)
                    p = ctx.profile_read()
                    n = max(p["launches"], 1)
                    prev = out.get(f"{vname}/{oname}", {})
                    best = lambda key, v: round(min(v, prev.get(key, v)), 1)
                    out[f"{vname}/{oname}"] = {
                        "wall_us": best("wall_us", wall),
                        "primary_us": best("primary_us", p["primary_ms_sum"] / n * 1e3),
                        "shadow_us": best("shadow_us", p["shadow_ms_sum"] / n * 1e3),
                        "frame_us": best("frame_us", p["frame_ms_sum"] / n * 1e3),
                        "hits": p["hits"] // n,
                        "prim_nodes": p["primary_node_visits"] // n, "prim_leaves": p["primary_leaf_visits"] // n,
                        "prim_tests": p["primary_tri_tests"] // n, "shadow_tests": p["shadow_tri_tests"] // n}
            ctx.set_options(0)
    for k, v in out.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
