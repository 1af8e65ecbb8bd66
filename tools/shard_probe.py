"""Per-rank trace time at N GPUs, rehearsed on one GPU: for world = 1, 2, 4, 8 the
frame is cut into the interleaved 64x64 tiles of FrameSharder and each rank's tile set
is traced on its own (steady state, back-to-back frames, no events).  The maximum over
ranks is the compute part of an N-GPU frame; the gather (overlapped with the next
frame) is not included.  Reports the implied compute-only speedup.

usage (GPU box): python tools/shard_probe.py [--frames 100] [--tile 64]
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
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import alloc_planes, assign, plan_tiles, pixels_of, trace_tiles_device
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    frame = env.mutable().to_frame()
    W, H = a.width, a.height
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    base = None
    with torch.cuda.stream(stream):
        for world in (int(x) for x in a.worlds.split(",")):
            tiles = [(0, 0, W, H)] if world == 1 else plan_tiles(W, H, a.tile)
            per = []
            for r in range(world):
                mine = assign(tiles, world, r)
                planes = alloc_planes(pixels_of(mine), dev)
                for _ in range(10):
                    trace_tiles_device(ctx, frame, W, H, mine, planes, stream.cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.frames):
                    trace_tiles_device(ctx, frame, W, H, mine, planes, stream.cuda_stream)
                torch.cuda.synchronize()
                us = (time.perf_counter() - t0) / a.frames * 1e6
                ctx.profile_enable(True)
                for _ in range(20):
                    trace_tiles_device(ctx, frame, W, H, mine, planes, stream.cuda_stream)
                torch.cuda.synchronize()
                ctx.profile_enable(False)
                p = ctx.profile_read()
                n = max(p["launches"], 1)
                per.append({"rank": r, "wall_us": round(us, 1), "kernel_us": round(p["frame_ms_sum"] / n * 1e3, 1),
                            "hits": p["hits"] // n, "tiles": len(mine)})
            worst = max(x["wall_us"] for x in per)
            if base is None:
                base = worst
            print(json.dumps({"world": world, "max_wall_us": worst, "mean_wall_us": round(sum(x["wall_us"] for x in per) / world, 1),
                              "compute_speedup": round(base / worst, 2), "ranks": per}), flush=True)


if __name__ == "__main__":
    main()
