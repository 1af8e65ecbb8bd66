"""Wave-level stage counts of the triangle test per frame (a -DMIRT_DIAG=1 build, MIRT_LIB):
  MIRT_LIB=distributed_raytracer_amd/libmirt_diag.so python tools/diag_stages.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    fr = env.mutable().to_frame()
    g = NativeFrameGroup(ctx, 1920, 1080, 0, 1, None, inflight=1)
    g.render(fr)
    g.wait()
    torch.cuda.synchronize()
    ctx.debug_counters()
    n = 4
    for _ in range(n):
        g.render(fr)
    g.wait()
    torch.cuda.synchronize()
    c = ctx.debug_counters() / n
    # stage 2: waves with a lane the divide-free classification leaves undecided (they run the
    # r2 / r3 divides); stage 3: waves with a lane inside the triangle (they run the t divide)
    names = ["tests", "past the pre-rejects", "take the r2/r3 divides", "inside (t divide)", "hits", "node visits",
             "leaves", "reach t pre-test"]
    for base, kind in ((0, "primary"), (8, "shadow")):
        print(kind, "  ".join(f"{nm}={c[base + i]:.0f}" for i, nm in enumerate(names)))
    print("k_trace: ready-wait spins", c[17], " idle spins", c[18], " shadow items", c[19], " primary blocks", c[20],
          " culled blocks", c[21])
    print("shadow light-table classifications", c[22], " skipped by the wave", c[22] - c[8])
    print("box gates", c[24], " further far planes", c[25], " near planes", c[26], " waves with a failing box", c[27],
          " nearest redo", c[28], " segment redo", c[29],
          " object gates skipped (block certificate)", c[30])
    g.close()


if __name__ == "__main__":
    main()
