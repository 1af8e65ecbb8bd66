"""Where do the cycles go?  Times the frame kernels on controlled variants of the
suzanne scene (1 GPU): the camera turned away (every ray misses: raygen, root test and
outputs only), the default view, and a close-up (mesh fills the screen).

usage (GPU box): python tools/cost_probe.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
            "dyn_primary": rt._lib.MIRT_OPT_DYNAMIC_PRIMARY,
            "one_kernel": rt._lib.MIRT_OPT_ONE_KERNEL}
    sh = FrameSharder(ctx, 1920, 1080, 0, 1, 64)
    out = {}
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for vname, c in views.items():
            mut = rt.EnvMutables(base.objects, base.lights, c)
            frame = mut.to_frame()
            for oname, o in opts.items():
                ctx.set_options(o)
                for _ in range(5):
                    sh.render(frame)
                torch.cuda.synchronize()
                ctx.profile_enable(True)
                for _ in range(30):
                    sh.render(frame)
                torch.cuda.synchronize()
                ctx.profile_enable(False)
                p = ctx.profile_read()
                n = max(p["launches"], 1)
                out[f"{vname}/{oname}"] = {
                    "primary_us": round(p["primary_ms_sum"] / n * 1e3, 1),
                    "shadow_us": round(p["shadow_ms_sum"] / n * 1e3, 1),
                    "frame_us": round(p["frame_ms_sum"] / n * 1e3, 1),
                    "hits": p["hits"] // n,
                    "prim_nodes": p["primary_node_visits"] // n, "prim_leaves": p["primary_leaf_visits"] // n,
                    "prim_tests": p["primary_tri_tests"] // n, "shadow_tests": p["shadow_tri_tests"] // n}
            ctx.set_options(0)
    for k, v in out.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
