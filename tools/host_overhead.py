"""Host enqueue cost vs device time per frame (1 GPU): python tools/host_overhead.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    frame = env.mutable().to_frame()
    sh = FrameSharder(ctx, 1920, 1080, 0, 1, 64)
    out = {}
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for prof in (False, True):
            ctx.profile_enable(prof)
            for _ in range(5):
                sh.render(frame)
            torch.cuda.synchronize()
            n = 200
            t0 = time.perf_counter()
            for _ in range(n):
                sh.render(frame)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            p = ctx.profile_read() if prof else None
            out["prof" if prof else "noprof"] = {
                "host_enqueue_us": round((t1 - t0) / n * 1e6, 1),
                "wall_us": round((t2 - t0) / n * 1e6, 1),
                "device_frame_us": round(p["frame_ms_sum"] / max(p["launches"], 1) * 1e3, 1) if p else None}
            ctx.profile_enable(False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
