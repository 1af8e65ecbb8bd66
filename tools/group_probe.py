"""Frames of the native group (mirt_trace_frame) on one GPU for profiling:
  MIRT_GROUP_REHEARSE=8 rocprofv3 --kernel-trace --stats -- python3 tools/group_probe.py --tile 32
usage: python tools/group_probe.py [--tile 32|0] [--inflight 4] [--frames 200] [--view default|away]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--view", default="default", choices=("default", "away"))
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--host-output", action="store_true", help="the root copies every frame to pinned host memory (the bench's D2H)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    mut = env.mutable()
    if a.view == "away":
        c = mut.cam
        mut = rt.EnvMutables(mut.objects, mut.lights, rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov))
    fr = mut.to_frame()
    W, H = (int(x) for x in a.size.split("x"))
    g = NativeFrameGroup(ctx, W, H, 0, 1, a.tile or None, inflight=a.inflight, batch=a.batch, host_output=a.host_output)
    for _ in range(20):
        g.render(fr)
    g.flush()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    calls = []
    for _ in range(a.frames):
        c0 = time.perf_counter()
        g.render(fr)
        calls.append(time.perf_counter() - c0)
    t1 = time.perf_counter()
    g.flush()
    torch.cuda.synchronize()
    print(json.dumps({"tile": a.tile, "inflight": a.inflight, "batch": a.batch, "view": a.view, "size": a.size,
                      "rehearse": os.environ.get("MIRT_GROUP_REHEARSE", "1"), "host_output": a.host_output,
                      "frame_interval_us": round((time.perf_counter() - t0) / a.frames * 1e6, 1),
                      "host_enqueue_us": round((t1 - t0) / a.frames * 1e6, 1),
                      "call_us_p10_50_90": [round(float(np.percentile(calls, q)) * 1e6, 1) for q in (10, 50, 90)]}))
    g.close()


if __name__ == "__main__":
    main()
