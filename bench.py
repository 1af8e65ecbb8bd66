"""Benchmark: Mrays/s + ms/frame of the trace worker on suzanne.obj 1920x1080.

A "step" is one full frame of tracer.Trace semantics over example/scene.json
(BASELINE.json configs[1]): primary ray per pixel, one shadow ray per light per hit
(3 lights), Phong, uint8 packing — everything worker/sequential's draw loop does per
frame.  Inputs (mesh, frame params) are resident on the GPU before timing; outputs stay
in HBM.  With N GPUs (torchrun, one process per GPU) the same frame is split into
interleaved 32x32 tiles and the packed tiles are gathered to rank 0 over RCCL and
unpacked into the framebuffer inside the timed region (strong scaling: total work is
one frame whatever N is).

Frames are pipelined (--inflight F, default 4): frame k runs on stream k % F with its own
buffers, so frame k+1's kernel starts while frame k's last workgroups finish, as the
reference master keeps several frames in flight.  ms_per_step is therefore the frame
INTERVAL at steady state (throughput); frame_latency_ms is one frame rendered alone
(render, gather, unpack, host sync) with the same launch shape.

Prints ONE JSON line on rank 0 (contract in the task statement).  Fields beyond the
contract: frames_in_flight, frame_latency_ms, primary_mrays_s, rays_per_frame, hits,
ms_kernels, parity, roofline_fp64_valu, cpu_baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
SCENE = os.path.join(ROOT, "tests", "golden", "example", "scene.json")
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"] if os.path.exists(
    os.path.join(ROOT, "BASELINE.json")) else "Mrays/sec + ms/frame, suzanne.obj 1920x1080"
BYTES_PER_TRI_TEST = 72  # fp64 P1, E1, E2 read per ray-triangle test
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X spec, vector FP64 (FMA = 2 flops)
HOST_CORES = 16  # the GPU box's CPU share for one GPU (os.cpu_count() shows the whole machine)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tile", type=int, default=8, help="multi-GPU deal unit: tile width (pixels)")
    ap.add_argument("--tile-h", type=int, default=0,
                    help="tile height; 0 = full-height column strips (contiguous in the column-major framebuffer)")
    ap.add_argument("--scene", default=SCENE)
    ap.add_argument("--bounces", type=int, default=0,
                    help="configs[4] reflection EXTENSION: bounces per primary hit (0 = the reference)")
    # defaults measured on one MI355X (tools/batch_sweep.sh): the whole 1080p frame runs
    # best as 8 in flight, 2 per launch; a rank's 1/N share needs more frames per launch
    # (each workgroup then owns enough blocks to hide its heaviest block's chain)
    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
    ap.add_argument("--batch", type=int, default=int(os.environ.get("MIRT_BATCH", "4" if multi else "2")),
                    help="frames per k_trace launch (native sharder; 1..min(8, inflight))")
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("MIRT_INFLIGHT", "16" if multi else "8")),
                    help="frames in flight (one stream and one set of buffers each; frame k+1's kernel "
                         "starts while frame k's last workgroups finish)")
    ap.add_argument("--grid", default="",
                    help="frame-kernel launch shape 'MIN_BLOCKS_PER_WG,MAX_WORKGROUPS' (mirt_set_grid; "
                         "default: FrameSharder's choice for the frames in flight)")
    ap.add_argument("--sharder", choices=("native", "torch"), default="native",
                    help="per-frame driver: native (libmirt mirt_trace_frame, RCCL called from C) or torch "
                         "(framebuffer.FrameSharder over torch.distributed)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-prefilter", action="store_true", help="ablation: always divide for r2")
    ap.add_argument("--no-octant", action="store_true", help="ablation: generic (sorted) child-box test only")
    ap.add_argument("--split-kernels", action="store_true",
                    help="variant: k_primary then k_shadow (default: one k_trace launch per frame)")
    ap.add_argument("--static-schedule", action="store_true",
                    help="ablation: round-robin work split instead of the dynamic work queues")
    ap.add_argument("--brute-force", action="store_true",
                    help="test every triangle for every ray (the north star's brute force; no BVH culling)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_pmc_traffic.json"),
                    help="per-launch HBM bytes / fp64 flops of the dominant kernel from rocprofv3 --pmc passes (profiles/)")
    a = ap.parse_args()
    # a short run (--steps K) keeps the pipeline shallow: the timed region ends with a drain
    # of up to F frames, so F stays within K / 8 unless set explicitly
    if "--inflight" not in sys.argv and "MIRT_INFLIGHT" not in os.environ:
        a.inflight = max(2, min(a.inflight, a.steps // 8))
    a.batch = max(1, min(a.batch, a.inflight))
    return a


def workload_name(a, W: int, H: int, tris: int, nl: int) -> str:
    """The BASELINE.json config this run measures (configs[1] by default)."""
    model = "suzanne.obj" if os.path.abspath(a.scene) == os.path.abspath(SCENE) else os.path.basename(
        os.path.dirname(os.path.abspath(a.scene))) + f" ({tris} tris)"
    name = f"{model} {W}x{H}, primary + one shadow ray per light ({nl}) + Phong"
    if a.bounces:
        name += f" + {a.bounces}-bounce reflections (configs[4] extension)"
    if model == "suzanne.obj" and W == 1920 and H == 1080 and not a.bounces:
        name += " (BASELINE configs[1])"
    return name


def cpu_baseline(scene_path: str, W: int, H: int) -> dict:
    """SURVEY.md §8(d) CPU baselines, timed on this host: (i) the oracle's faithful variant
    (rtreego-style R-tree, 1 thread, fp64, worker/sequential's serial i/j loop) over one
    full frame — the reported value; (ii) the same code on the box's host cores
    (column-interleaved threads)."""
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    orc = Oracle(load_scene(scene_path), use_rtree=True)
    out = None
    for threads in (1, HOST_CORES):
        t0 = time.perf_counter()
        r = orc.frame(W, H, nthreads=threads)
        dt = time.perf_counter() - t0
        rays = r["stats"]["primary_rays"] + r["stats"]["shadow_rays"]
        v = {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
             "sample": f"one full {W}x{H} frame ({rays} primary+shadow rays), oracle/rt_oracle.c with "
                       f"rtreego-style R-tree culling, {threads} thread(s), {dt:.2f} s",
             "ms_per_frame": round(dt * 1e3, 1)}
        if out is None:
            out = v
        else:
            out["all_cores"] = {k: v[k] for k in ("value", "cores", "ms_per_frame")}
    out["nproc"] = os.cpu_count()
    return out


def parity_check(fb_valid: np.ndarray, fb_rgb8: np.ndarray, scene_path: str, W: int, H: int,
                 bounces: int = 0) -> dict:
    """Parity gate of the timed frame: a 1/16 subsample — every 16th
    column — against the oracle, valid mask and rgb8 bit-exact."""
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    cols = list(range(5, W, 16))
    orc = Oracle(load_scene(scene_path), use_rtree=True)
    orc.set_bounces(bounces)
    ref = orc.trace_tiles(W, H, [(x, 0, 1, H) for x in cols], nthreads=HOST_CORES)
    sub = np.concatenate([np.arange(x * H, (x + 1) * H) for x in cols])
    ok = bool(np.array_equal(fb_valid[sub], ref["valid"]) and np.array_equal(fb_rgb8[sub], ref["rgb8"]))
    return {"columns_checked": len(cols), "bit_exact": ok, "hits": int(fb_valid.sum())}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    # One process per GPU.  MIRT_DIST_BACKEND=gloo (rehearsal of the N>1 path on a box
    # with fewer GPUs than ranks): ranks share GPUs and the gather stages through host.
    backend = os.environ.get("MIRT_DIST_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder, NativeFrameGroup

    W, H = a.width, a.height
    ctx = rt.Context(local)
    opts = (rt._lib.MIRT_OPT_NO_OCTANT if a.no_octant else 0) | (rt._lib.MIRT_OPT_NO_PREFILTER if a.no_prefilter else 0) | (
        rt._lib.MIRT_OPT_BRUTE_FORCE if a.brute_force else 0) | (
        rt._lib.MIRT_OPT_STATIC_SCHEDULE if a.static_schedule else 0) | (rt._lib.MIRT_OPT_SPLIT_KERNELS if a.split_kernels else 0)
    ctx.set_options(opts)
    env = rt.Environment.from_file(a.scene, ctx)
    import dataclasses
    frame = dataclasses.replace(env.mutable(), max_bounces=a.bounces).to_frame()
    tris = sum(len(m.face_v) for m in env.meshes)
    nl = len(env.mutable().lights)
    # native: the per-frame trace + RCCL gather + unpack in libmirt (mirt_trace_frame), one C
    # call per frame; torch: the same sequence through torch.distributed (FrameSharder), used
    # for the gloo rehearsal (RCCL cannot put two ranks on one GPU) and as a fallback
    sharder = a.sharder if not (world > 1 and backend != "nccl") else "torch"
    sh = None
    if sharder == "native":
        try:
            sh = NativeFrameGroup(ctx, W, H, rank, world, a.tile if world > 1 else None, inflight=a.inflight,
                                  tile_h=a.tile_h, batch=a.batch)
        except Exception as e:  # noqa: BLE001 — reported in the JSON line, then the torch path runs
            print(f"native frame group unavailable ({e}); using the torch.distributed sharder", file=sys.stderr)
            sharder = f"torch (native failed: {e})"
    if sh is None:
        # the torch.distributed path was tuned at 4 in flight (one frame per launch)
        sh = FrameSharder(ctx, W, H, rank, world, a.tile, inflight=min(a.inflight, 4), tile_h=a.tile_h)
    if a.grid:
        ctx.set_grid(*(int(x) for x in a.grid.split(",")))
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local]) if backend == "nccl" else dist.barrier()

    # One stream for every frame: frames are serialised on the GPU (no two frames in
    # flight writing the same framebuffer); the host still enqueues ahead of the GPU.
    # The throughput region runs without profiling (its HIP events between the kernels cost
    # ~10 % of a frame); the same frames are then traced again with profiling on, and the
    # per-kernel HIP-event times and device counters (rays, tests) come from that region.
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for _ in range(a.warmup):
            sh.render(frame)
        sh.flush()
        torch.cuda.synchronize(dev)

        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sh.render(frame)  # N > 1: frame k's gather overlaps frame k+1's tracing
        sh.flush()            # the last frame's gather + unpack are inside the timed region
        torch.cuda.synchronize(dev)
        barrier()
        t1 = time.perf_counter()

        ctx.profile_enable(True)
        for _ in range(a.steps):
            sh.render(frame)
        sh.flush()
        torch.cuda.synchronize(dev)
        ctx.profile_enable(False)

        # single-frame latency: one frame alone (render, gather + unpack, host sync), median
        lat = []
        for _ in range(min(a.steps, 20)):
            barrier()
            torch.cuda.synchronize(dev)
            l0 = time.perf_counter()
            sh.render(frame)
            sh.flush()
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - l0)
        latency = float(np.median(lat)) if lat else 0.0
    prof = ctx.profile_read()

    elapsed = t1 - t0
    pl = max(prof["frames"], 1)  # per-frame device counters (a launch may trace several frames)
    counts = torch.tensor([elapsed, latency, prof["primary_rays"] / pl, prof["shadow_rays"] / pl, prof["hits"] / pl,
                           prof["reflection_rays"] / pl], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
    if world > 1:
        tmax = counts[:2].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = counts[2:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed, latency = (float(x) for x in tmax.tolist())
        primary, shadow, hits, refl = (float(x) for x in sums.tolist())
    else:
        primary, shadow, hits, refl = (float(x) for x in counts[2:].tolist())

    if rank == 0:
        steps = a.steps
        ms = elapsed / steps * 1e3
        rays_per_frame = primary + shadow + refl  # per frame, all ranks (device counters)
        launches = max(prof["launches"], 1)
        prim_ms = prof["primary_ms_sum"] / launches
        # the dominant kernel: k_trace (the whole frame, one launch) or, split, k_primary;
        # reflection frames always run split (k_primary, k_shadow, k_reflect)
        one = not a.split_kernels and not a.bounces
        kname = "k_trace" if one else "k_primary"
        k_tests = (prof["primary_tri_tests"] + (prof["shadow_tri_tests"] if one else 0)) / launches
        achieved = k_tests * BYTES_PER_TRI_TEST / (prim_ms / 1e3) / 1e9
        traffic = fp64_flops = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                if tj.get("width") == W and tj.get("height") == H and tj.get("gpus", 1) == world:
                    traffic = tj.get(f"{kname}_hbm_bytes_per_launch")
                    fp64_flops = tj.get(f"{kname}_fp64_flops_per_launch")
            except (OSError, ValueError):
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(rays_per_frame / (ms / 1e3) / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: the reference's own example/scene.json (suzanne.obj, 968 tris, 3 lights), static frame-0 camera"
                     if os.path.abspath(a.scene) == os.path.abspath(SCENE) else
                     f"synthetic: {os.path.relpath(a.scene, ROOT)} ({tris} tris, {nl} lights), the scene's camera"),
            "config": {"workload": workload_name(a, W, H, tris, nl), "width": W, "height": H, "triangles": tris,
                       "lights": nl, "parallelism": f"image tiles x{world}" + (f" ({a.tile}px, RCCL gather)"
                                                                                if world > 1 else ""),
                       "culling": "none (brute force)" if a.brute_force else "exact BVH (packet traversal)"},
            "frames_in_flight": sh.F,
            "frames_per_launch": getattr(sh, "B", 1),
            "sharder": sharder,
            "frame_latency_ms": round(latency * 1e3, 4),
            "primary_mrays_s": round(primary / (ms / 1e3) / 1e6, 3),
            "rays_per_frame": int(rays_per_frame),
            "hits_per_frame": int(hits),
            "tri_tests_per_frame": int((prof["primary_tri_tests"] + prof["shadow_tri_tests"]) / pl),
            "bvh_visits_per_frame": {k: int(prof[k] / pl) for k in (
                "primary_node_visits", "primary_leaf_visits", "shadow_node_visits", "shadow_leaf_visits")},
            "ms_kernels": {("frame_kernel" if one else "primary"): round(prim_ms, 4),
                           "shadow": round(prof["shadow_ms_sum"] / launches, 4),
                           "reflect": round(prof["reflect_ms_sum"] / launches, 4),
                           "frame_device": round(prof["frame_ms_sum"] / launches, 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kname, "bytes_per_unit": BYTES_PER_TRI_TEST,
                         "units_per_launch": int(k_tests),
                         # with frames in flight a launch shares the chip with its neighbours,
                         # so per-launch time overstates the cost: the same bytes per frame
                         # over the steady-state frame interval
                         "chip_rate_gbs": round(k_tests * launches / pl * BYTES_PER_TRI_TEST / (ms / 1e3) / 1e9, 1),
                         "note": "algorithmic bytes = 72 B fp64 triangle record x ray-triangle tests actually "
                                 "performed (device counter); the mesh is LDS-resident so the real bound is fp64 "
                                 "VALU, see DESIGN.md; kernel time = HIP events on the trace stream over a second "
                                 "region of the same frames (the throughput region runs without events)"},
            "roofline_fp64_valu": None if fp64_flops is None else {
                "bound": "fp64-valu", "kernel": kname, "unit": "TFLOP/s", "peak": FP64_VALU_PEAK_TFLOPS,
                "achieved": round(64 * fp64_flops / (prim_ms / 1e3) / 1e12, 3),
                "frac": round(64 * fp64_flops / (prim_ms / 1e3) / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                "flops_per_launch": int(64 * fp64_flops),
                "note": "SQ_INSTS_VALU_FLOPS_FP64 (counts per wave instruction, FMA = 2) x 64 lanes per launch, "
                        "from the committed rocprofv3 pass (profiles/), over this run's HIP-event time of the kernel"},
        }
        if not a.no_parity:
            fr = sh.frame
            line["parity"] = parity_check(fr.valid.cpu().numpy(), fr.rgb8.cpu().numpy(), a.scene, W, H, a.bounces)
        if not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(a.scene, W, H)
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
