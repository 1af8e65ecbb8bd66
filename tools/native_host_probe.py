"""Host cost per frame of the native frame driver (mirt_trace_frame) on one GPU: the
world = 1 tiled rehearsal (packed rgbv tiles + unpack, no RCCL peers) with the camera
turned away (the GPU side nearly empty, so the frame interval is the host's enqueue cost)
and with the default view; FrameSharder's world = 1 path beside it.

usage (GPU box): python tools/native_host_probe.py [--frames 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--size", default="1920x1080")
    a = ap.parse_args()
    import numpy as np
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder, NativeFrameGroup
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    mut = env.mutable()
    c = mut.cam
    views = {"away": rt.EnvMutables(mut.objects, mut.lights,
                                    rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov)).to_frame(),
             "default": mut.to_frame()}
    W, H = (int(x) for x in a.size.split("x"))
    drivers = {"native_tiled32": lambda: NativeFrameGroup(ctx, W, H, 0, 1, 32, inflight=a.inflight),
               "native_whole": lambda: NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=a.inflight),
               "torch_whole": lambda: FrameSharder(ctx, W, H, 0, 1, inflight=a.inflight)}
    for dname, make in drivers.items():
        d = make()
        for vname, fr in views.items():
            for _ in range(20):
                d.render(fr)
            d.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                d.render(fr)
            t1 = time.perf_counter()
            d.flush()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"driver": dname, "view": vname, "inflight": a.inflight, "size": a.size,
                              "host_enqueue_us": round((t1 - t0) / a.frames * 1e6, 1),
                              "frame_interval_us": round((t2 - t0) / a.frames * 1e6, 1)}), flush=True)
        if hasattr(d, "close"):
            d.close()
        ctx.set_grid()


if __name__ == "__main__":
    main()
