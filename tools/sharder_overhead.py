"""FrameSharder vs a bare enqueue loop (same frames, streams, buffers, launch shape):
is the sharder's per-frame host work on the critical path?  Also times the host cost
per render() with the camera turned away (GPU nearly idle).

usage (GPU box): python tools/sharder_overhead.py [--inflight 4]
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
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--frames", type=int, default=300)
    a = ap.parse_args()
    import numpy as np
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder, trace_tiles_device
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    mut = env.mutable()
    c = mut.cam
    views = {"default": mut.to_frame(),
             "away": rt.EnvMutables(mut.objects, mut.lights,
                                    rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov)).to_frame()}
    W, H = 1920, 1080
    F = a.inflight
    side = torch.cuda.Stream()
    res = {}
    with torch.cuda.stream(side):
        sh = FrameSharder(ctx, W, H, 0, 1, inflight=F)
        for rep in range(2):
            for vname, frame in views.items():
                # sharder
                for _ in range(20):
                    sh.render(frame)
                sh.flush()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.frames):
                    sh.render(frame)
                t1 = time.perf_counter()
                sh.flush()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                r1 = ((t1 - t0) / a.frames * 1e6, (t2 - t0) / a.frames * 1e6)
                # bare loop on the sharder's own streams and buffers
                streams = sh.streams or [torch.cuda.current_stream()]
                for k in range(20):
                    trace_tiles_device(ctx, frame, W, H, sh._mine_c, sh.frames[k % F], streams[k % F].cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(a.frames):
                    trace_tiles_device(ctx, frame, W, H, sh._mine_c, sh.frames[k % F], streams[k % F].cuda_stream)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                r2 = ((t1 - t0) / a.frames * 1e6, (t2 - t0) / a.frames * 1e6)
                res[f"{vname}/sharder"] = min(res.get(f"{vname}/sharder", (1e9, 1e9)), r1, key=lambda x: x[1])
                res[f"{vname}/bare"] = min(res.get(f"{vname}/bare", (1e9, 1e9)), r2, key=lambda x: x[1])
    for k, (enq, tot) in res.items():
        print(json.dumps({"case": k, "inflight": F, "host_enqueue_us": round(enq, 1), "frame_interval_us": round(tot, 1)}))


if __name__ == "__main__":
    main()
