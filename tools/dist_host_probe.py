"""Host cost of the N-GPU per-frame sequence, rehearsed on ONE GPU with a world-size-1
RCCL process group: trace rank 0's tiles of an N-way split into a packed rgbv plane,
gather it (torch.distributed "nccl", async), wait, unpack — exactly FrameSharder's world > 1
calls.  Reports host microseconds per frame for each piece and the frame interval, with
the GPU work of one rank's share running meanwhile.

usage (GPU box): python tools/dist_host_probe.py [--share 8] [--frames 300]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share", type=int, default=8)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--inflight", type=int, default=4)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    import torch
    import torch.distributed as dist
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd import _lib as L
    from distributed_raytracer_amd.framebuffer import (DevicePlanes, _tiles_c, alloc_planes, assign, pixels_of,
                                                       plan_tiles, trace_tiles_device)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    frame = env.mutable().to_frame()
    W, H = 1920, 1080
    F = a.inflight
    mine = assign(plan_tiles(W, H, 32), a.share, 0)
    cap = pixels_of(mine)
    tc = _tiles_c(mine)
    offs = (C.c_uint64 * len(mine))(*[sum(t[2] * t[3] for t in mine[:i]) for i in range(len(mine))])
    dev = torch.device("cuda", 0)
    streams = [ctx.stream_create() for _ in range(F)]
    packed = [alloc_planes(cap, dev, packed=True) for _ in range(F)]
    gathered = [torch.empty(cap, dtype=torch.int32, device=dev) for _ in range(F)]
    fbs = [alloc_planes(W * H, dev) for _ in range(F)]
    cucum = {"trace": 0.0, "gather": 0.0, "wait_unpack": 0.0}

    def run(n, timing):
        pend = None
        for k in range(n):
            s = streams[k % F]
            t0 = time.perf_counter()
            trace_tiles_device(ctx, frame, W, H, tc, packed[k % F], s.cuda_stream)
            t1 = time.perf_counter()
            with torch.cuda.stream(s):
                w = dist.gather(packed[k % F].rgbv, [gathered[k % F]], dst=0, async_op=True)
            t2 = time.perf_counter()
            if pend is not None:
                pk, pw = pend
                ps = streams[pk % F]
                with torch.cuda.stream(ps):
                    pw.wait()
                src = DevicePlanes(rgbv=gathered[pk % F]).outputs()
                L.check(L.lib().mirt_unpack_tiles_at_async(ctx.handle, W, H, tc, offs, len(mine), C.byref(src),
                                                           C.byref(fbs[pk % F].outputs()), C.c_void_p(ps.cuda_stream)))
            t3 = time.perf_counter()
            pend = (k, w)
            if timing:
                cucum["trace"] += t1 - t0
                cucum["gather"] += t2 - t1
                cucum["wait_unpack"] += t3 - t2
        torch.cuda.synchronize()

    run(20, False)
    t0 = time.perf_counter()
    run(a.frames, True)
    dt = (time.perf_counter() - t0) / a.frames * 1e6
    out = {"share": a.share, "inflight": F, "frame_interval_us": round(dt, 1)}
    out.update({f"host_{k}_us": round(v / a.frames * 1e6, 1) for k, v in cucum.items()})
    # the trace alone (no collective) for comparison
    t0 = time.perf_counter()
    for k in range(a.frames):
        trace_tiles_device(ctx, frame, W, H, tc, packed[k % F], streams[k % F].cuda_stream)
    torch.cuda.synchronize()
    out["trace_only_interval_us"] = round((time.perf_counter() - t0) / a.frames * 1e6, 1)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
