"""LDS triangle streaming (configs[3]) window statistics per frame, from a -DMIRT_DIAG=1 build
(MIRT_LIB; built by `make -C distributed_raytracer_amd/csrc OUT=../libmirt_diag.so OBJ=obj_diag EXTRA=-DMIRT_DIAG=1`): leaves served through the per-wave LDS windows and window reloads (8 KB each),
hence the window's hit rate.
  MIRT_LIB=distributed_raytracer_amd/libmirt_diag.so python tools/stream_window.py /tmp/sphere1m/scene.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    scene = sys.argv[1] if len(sys.argv) > 1 else "/tmp/sphere1m/scene.json"
    W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (3840, 2160)
    ctx = rt.Context(0)
    env = rt.Environment.from_file(scene, ctx)
    fr = env.mutable().to_frame()
    g = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=1)
    g.render(fr)
    g.wait()
    torch.cuda.synchronize()
    ctx.debug_counters()
    n = 3
    for _ in range(n):
        g.render(fr)
    g.wait()
    torch.cuda.synchronize()
    c = ctx.debug_counters() / n
    served, reloads = float(c[23]), float(c[31])
    tris = int(os.environ.get("STREAM_TRIS", "24"))  # the build's MIRT_STREAM_TRIS
    out = {"scene": scene, "width": W, "height": H, "frames": n,
           "primary_leaves_per_frame": float(c[6]), "shadow_leaves_per_frame": float(c[14]),
           "window_leaves_served_per_frame": served, "window_reloads_per_frame": reloads,
           "window_hit_rate": (served - reloads) / served if served else None,
           "window_faces": tris + 1, "reload_bytes_per_frame": reloads * (tris + 1) * 72,
           "note": f"wave-level counts (one per wave per leaf); a reload copies {tris + 1} faces x 72 B into the "
                   f"wave's LDS slice"}
    print(json.dumps(out))
    g.close()


if __name__ == "__main__":
    main()
