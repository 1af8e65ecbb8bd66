"""Frames in flight: F streams, each with its own output planes, frames dealt round-robin
(frame k on stream k % F).  The persistent kernels of consecutive frames then overlap:
one frame's tail (the last heavy workgroups) runs beside the next frame's start.
Reports the steady-state frame interval per (world share, F, launch shape), the minimum
over --repeat interleaved passes: the whole 1080p frame (world 1) or rank 0's tiles of an
N-GPU split (interleaved 64x64 tiles, as FrameSharder deals them).

usage (GPU box): python tools/inflight_probe.py [--world 1,8] [--inflight 1,2,4] [--maxwg 0,256] [--repeat 3]
"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--world", default="1,8")
    ap.add_argument("--inflight", default="1,2,4")
    ap.add_argument("--grid", default="32", help="min 8x8 blocks per workgroup (mirt_set_grid), comma list")
    ap.add_argument("--maxwg", default="0", help="max workgroups per frame (mirt_set_grid; 0 = 2 per CU), comma list")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--tiled", action="store_true", help="world 1 as 64x64 tiles too (default: one tile)")
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--view", default="default", choices=("default", "away"))
    a = ap.parse_args()
    import numpy as np
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import _tiles_c, alloc_planes, assign, plan_tiles, pixels_of, trace_tiles_device
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    mut = env.mutable()
    if a.view == "away":  # every block culled: the GPU side is nearly empty
        c = mut.cam
        mut = rt.EnvMutables(mut.objects, mut.lights, rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov))
    frame = mut.to_frame()
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    ints = lambda s: [int(x) for x in s.split(",")]
    configs = list(itertools.product(ints(a.world), ints(a.inflight), ints(a.grid), ints(a.maxwg)))
    best = {}
    for _ in range(a.repeat):
        for world, F, g, mw in configs:
            tiles = [(0, 0, W, H)] if world == 1 and not a.tiled else assign(plan_tiles(W, H, a.tile), world, 0)
            ctx.set_grid(g, mw)
            streams = [torch.cuda.Stream(dev) for _ in range(F)]
            planes = [alloc_planes(pixels_of(tiles), dev, packed=world > 1) for _ in range(F)]
            tc = _tiles_c(tiles)

            def run(n):
                for k in range(n):
                    trace_tiles_device(ctx, frame, W, H, tc, planes[k % F], streams[k % F].cuda_stream)

            run(4 * F + 10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(a.frames)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / a.frames * 1e6
            key = (world, F, g, mw)
            best[key] = min(us, best.get(key, us))
    for (world, F, g, mw), us in best.items():
        print(json.dumps({"world": world, "inflight": F, "min_blocks_per_wg": g, "max_wg": mw,
                          "frame_interval_us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
