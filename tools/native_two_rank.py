"""Two ranks of the native multi-GPU frame (mirt_group, RCCL send/recv gather) on
whatever GPUs the box has (ranks share a GPU when there are fewer).  Launch:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29561 tools/native_two_rank.py
Rank 0 checks every framebuffer against a single-GPU draw of the same camera."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import NativeFrameGroup
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    ctx = rt.Context(dev)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    W, H = 320, 240
    base = env.mutable()
    c = base.cam
    cams = [c, rt.Camera.new(tuple(np.asarray(c.pos) + np.array([0.7, 0.3, 0.0])), c.forward, c.fov)]
    muts = [rt.EnvMutables(base.objects, base.lights, cm) for cm in cams]
    frames = [m.to_frame() for m in muts]
    try:
        g = NativeFrameGroup(ctx, W, H, rank, world, 32, inflight=2)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: native group failed: {e}", flush=True)
        dist.destroy_process_group()
        return
    order = [0, 1, 1, 0, 0, 1]
    for q in order:
        g.render(frames[q])
    g.flush()
    torch.cuda.synchronize()
    if rank == 0:
        ok = True
        for k in range(len(order) - 2, len(order)):
            ref = rt.draw(env, W, H, muts[order[k]])
            got = g.frames[k % 2]
            ok &= np.array_equal(got.valid.cpu().numpy(), ref.valid) and np.array_equal(got.rgb8.cpu().numpy(), ref.rgb8)
        print(f"native two-rank frames bit-exact: {ok}", flush=True)
    dist.barrier()
    g.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
