"""Where the host time after a burst of frames goes (the bench's timed-region end): a burst of
frames through the native group as bench.py runs it (8 in flight, host output), then the host
wait, then variants of the device-wide synchronize, each timed on the host:
  python tools/sync_probe.py [--frames 20] [--reps 5]
  variant "device":  mirt_group_wait, then hipDeviceSynchronize (torch.cuda.synchronize)
  variant "twice":   mirt_group_wait, hipDeviceSynchronize twice (the second one's cost)
Use MIRT_LIB to compare library builds (before round 6's end, mirt_group_wait left the streams'
completion round trips to the device-wide synchronize)."""
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
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    hip = C.CDLL("libamdhip64.so")
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    fr = env.mutable().to_frame()
    g = NativeFrameGroup(ctx, 1920, 1080, 0, 1, None, inflight=8, batch=1, host_output=True)
    out = {}
    try:
        for _ in range(5):
            g.render(fr)
        g.wait()
        torch.cuda.synchronize()
        for variant in ("device", "twice", "device"):
            res = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                for _ in range(a.frames):
                    g.render(fr)
                t0 = time.perf_counter()
                g.wait()
                t1 = time.perf_counter()
                t2 = time.perf_counter()
                hip.hipDeviceSynchronize()
                t3 = time.perf_counter()
                if variant == "twice":
                    hip.hipDeviceSynchronize()
                t4 = time.perf_counter()
                res.append([(t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t4 - t3) * 1e6])
            out.setdefault(variant, []).append([round(float(x), 1) for x in np.median(np.array(res), axis=0)])
    finally:
        g.close()
    print(json.dumps({"frames": a.frames, "lib": os.environ.get("MIRT_LIB", "libmirt.so"),
                      "columns": ["group_wait_us", "-", "device_sync_us",
                                                      "second_device_sync_us"], **out}))


if __name__ == "__main__":
    main()
