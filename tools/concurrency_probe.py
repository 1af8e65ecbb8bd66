"""Does splitting one frame into k concurrent calls (interleaved 64x64 tiles, one stream
each) shorten the frame?  The persistent kernels of the calls interleave on the chip, so
one call's tail can fill with another call's work.  Times frames of the default view,
1 GPU, for k = 1, 2, 4 with the split kernels and with the one-launch kernel.

usage (GPU box): python tools/concurrency_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import alloc_planes, assign, plan_tiles, pixels_of, trace_tiles_device
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    frame = env.mutable().to_frame()
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    res = {}
    for oname, o in (("one_kernel", 0), ("split", rt._lib.MIRT_OPT_SPLIT_KERNELS)):
        ctx.set_options(o)
        for k in (1, 2, 4):
            tiles = [(0, 0, W, H)] if k == 1 else plan_tiles(W, H, 64)
            parts = [assign(tiles, k, r) for r in range(k)]
            planes = [alloc_planes(pixels_of(p), dev) for p in parts]
            streams = [torch.cuda.Stream(dev) for _ in range(k)]
            main = torch.cuda.current_stream(dev)

            def one():
                ev = torch.cuda.Event()
                ev.record(main)
                for r in range(k):
                    streams[r].wait_event(ev)
                    trace_tiles_device(ctx, frame, W, H, parts[r], planes[r], streams[r].cuda_stream)
                for r in range(k):
                    e = torch.cuda.Event()
                    e.record(streams[r])
                    main.wait_event(e)

            for _ in range(10):
                one()
            torch.cuda.synchronize()
            print("warm", oname, k, flush=True)
            best = None
            for _ in range(3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(main)
                for _ in range(50):
                    one()
                b.record(main)
                torch.cuda.synchronize()
                t = a.elapsed_time(b) / 50 * 1e3
                best = t if best is None else min(best, t)
            res[f"{oname}/k{k}"] = round(best, 1)
            print(oname, k, round(best, 1), flush=True)
    ctx.set_options(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
