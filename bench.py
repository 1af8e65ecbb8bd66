"""Benchmark: Mrays/s + ms/frame of the trace worker on suzanne.obj 1920x1080.

A "step" is one full frame of tracer.Trace semantics over example/scene.json
(BASELINE.json configs[1]): primary ray per pixel, one shadow ray per light per hit
(3 lights), Phong, uint8 packing — everything worker/sequential's draw loop does per
frame — and, as BASELINE.md §3 defines ms/frame, the D2H copy of the assembled rgb8 +
valid framebuffer into pinned host memory (mirt_group_set_host_output; --no-d2h leaves
outputs in HBM).  Inputs (mesh, frame params) are resident on the GPU before timing.
With N GPUs (torchrun, one process per GPU) the same frame is split into interleaved
8-px strips; every rank's strips inside the frame's hit rectangle are gathered to rank 0
over RCCL and unpacked into the framebuffer inside the timed region (strong scaling:
total work is one frame whatever N is).

Frames are pipelined (--inflight F frames in flight, --batch B frames per k_trace
launch): frame k+1's kernel starts while frame k's last workgroups finish, as the
reference master keeps several frames in flight (master/main.go:264-266).  ms_per_step is
the wall time of the K timed frames / K (from an empty pipeline to the last frame in host
memory); device_ms_per_frame the same frames without the D2H; frame_latency_ms one frame
rendered alone (render, [gather, unpack,] D2H, host sync), median of up to 20.

Prints ONE JSON line on rank 0 (contract in the task statement).  Fields beyond the
contract: frames_in_flight, frames_per_launch, device_ms_per_frame, frame_latency_ms,
primary_mrays_s, rays_per_frame, ms_kernels, launches (k_trace launches per region, in
order: warmup, timed, device-only, profiled, latency — the key to the committed rocprofv3
trace), parity, roofs (physical roofs from the committed PMC passes of this command),
cpu_baseline.
"""
from __future__ import annotations

import argparse
import dataclasses
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
VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 4  # wave64 VALU instructions per second at 4 cycles each (fp64 rate)
SIMD_CYCLES_PER_S = 256 * 4 * 2.4e9     # VALU-busy roof: 1024 SIMDs x 2.4 GHz
HOST_CORES = 16  # the GPU box's CPU share for one GPU (os.cpu_count() shows the whole machine)


LDS_RESIDENT_FACES = 1024  # meshes up to this many faces are staged whole into each workgroup's LDS


def scene_tag(path: str) -> str:
    """Which scene a profile was taken on: the scene file's directory and name."""
    p = os.path.abspath(path)
    return os.path.join(os.path.basename(os.path.dirname(p)), os.path.basename(p))


def find_profile(path: str, shape: dict, build_id: str):
    """The committed rocprofv3 summary of THIS command on THIS build (tools/roofline.py): the
    given file, or the newest profiles/*_roofline.json (by tag) whose launch shape equals this
    run's and whose build_id (mirt_build_id() of the library it was taken on: a hash of the
    kernels, their launch code and the compile flags) equals the loaded library's; counters
    from another shape or another build are never cited.  Returns (profile, path, why-not)."""
    import glob
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "*_roofline.json")), reverse=True)
    stale = None
    for c in cands:
        pj = load_profile(c, shape)
        if not pj:
            continue
        if pj.get("build_id") != build_id:
            stale = stale or os.path.relpath(c, ROOT)
            continue
        return pj, c, None
    why = ("no committed PMC profile of this command's shape" if stale is None else
           f"the newest profile of this shape ({stale}) was taken on another build (build_id differs from {build_id})")
    return None, None, why


def roofline_block(pj, pj_path, kname, ms, dev_ms, achieved, k_tests, frames_per_launch, launch_ms,
                   mesh_lds_resident, alg_kernel=None, launch_ms_mean=None, why_not=None, tests_per_frame=None):
    """`roofline` of the bench line: the PHYSICAL binding roof of the frame kernel.  The
    kernels are fp64 VALU code whose mesh sits in LDS (suzanne) or streams from L2/HBM
    (configs[3]); the committed PMC passes of this exact command (profiles/) show the VALU as
    the binding unit (HBM at ~10%), so achieved = VALU-busy SIMD cycles per frame (4 x
    SQ_ACTIVE_INST_VALU of the frame kernel, the numerator of rocprof's VALUBusy) /
    ms_per_step (the headline frame interval, measured live), against 1,024 SIMDs x 2.4 GHz.
    `issue` keeps the instruction count (SQ_INSTS_VALU) at the fp64 issue rate; traffic = HBM
    bytes per frame from the PMC passes ((2 FETCH_SIZE + WRITE_SIZE) x 1024); the north
    star's algorithmic HBM figure (72 B x ray-triangle tests / launch duration) is kept as
    `algorithmic`.  Without a committed profile of this command the algorithmic figure is the
    roofline (and says so)."""
    per_launch_bytes = k_tests * BYTES_PER_TRI_TEST
    # the launch duration: the rocprofv3 kernel-trace average of the TIMED region's launches when
    # the committed profile of this command is of this build (the profiled region's HIP events
    # bracket launches slowed by the profiling itself, 1.7x in r05j); the HIP-event median of
    # the profiled region otherwise, and always as a cross-check
    # (only where one launch of the profiled kernel is the unit: a reflection frame's figure spans
    # all its kernels, whose per-kernel launches the profile averages separately)
    timed_ns = ((pj or {}).get("avg_ns_by_region") or {}).get("timed") if alg_kernel in (None, kname) else None
    hip_median_achieved = achieved
    if timed_ns:
        launch_src = (f"rocprofv3 kernel-trace average of the timed region's launches "
                      f"({os.path.relpath(pj_path, ROOT)}, same build)")
        launch_ms_used = timed_ns / 1e6
        achieved = per_launch_bytes / (launch_ms_used / 1e3) / 1e9
    else:
        launch_src = "MEDIAN HIP-event duration of the profiled region's launches (no profile of this build)"
        launch_ms_used = launch_ms
    alg = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4),
           "kind": "algorithmic (north star): 72 B fp64 triangle record x ray-triangle tests performed "
                   "(device counter) per launch / " + launch_src + (
                       "; the mesh is LDS-resident, so these bytes are LDS reads, not HBM traffic"
                       if mesh_lds_resident else "; the mesh is HBM-resident (scalar loads through L2/MALL)"),
           "kernel": alg_kernel or kname, "bytes_per_unit": BYTES_PER_TRI_TEST, "units_per_launch": int(k_tests),
           "frames_per_launch": round(frames_per_launch, 3), "launch_ms": round(launch_ms_used, 4),
           "hip_event_median_launch_ms": round(launch_ms, 4),
           "achieved_on_hip_event_median": round(hip_median_achieved, 1),
           "launch_ms_mean": None if launch_ms_mean is None else round(launch_ms_mean, 4),
           "achieved_on_mean": None if not launch_ms_mean else round(per_launch_bytes / (launch_ms_mean / 1e3) / 1e9, 1)}
    if tests_per_frame is not None:
        # frames in flight overlap, so a launch's duration is not a frame's cost: the same bytes per
        # FRAME over the device-only frame interval (the timed frames without the D2H)
        pf = tests_per_frame * BYTES_PER_TRI_TEST / (dev_ms / 1e3) / 1e9
        alg["per_frame"] = {"bytes_per_frame": int(tests_per_frame * BYTES_PER_TRI_TEST),
                            "interval_ms": round(dev_ms, 4), "achieved": round(pf, 1),
                            "frac": round(pf / HBM_PEAK_GBS, 4),
                            "note": "72 B x tests per frame / device_ms_per_frame (the timed frames' interval, "
                                    "outputs left in HBM): not inflated by the overlap of frames in flight"}
    if not pj or "sq_insts_valu_per_launch" not in pj:
        out = dict(alg)
        out["kernel"], out["kernels"] = kname, alg["kernel"]  # the dominant kernel names the shape
        out["traffic"] = None
        out["note"] = (why_not or "no committed PMC profile of this command's shape") + ": algorithmic roofline only"
        return out
    fpl = pj["frames_per_launch"]
    valu = pj["sq_insts_valu_per_launch"] / fpl
    hbm = pj.get("hbm_bytes_per_launch")
    issue = {"valu_insts_per_frame": int(valu),
             "issue_frac_4cyc": round(valu / (ms / 1e3) / VALU_ISSUE_PER_S, 4),
             "note": "wave64 VALU instructions per frame / ms_per_step against one instruction per 4 cycles per "
                     "SIMD (fp64 rate); fp32 and integer ops issue in 2 on CDNA4's SIMD-32"}
    common = {"traffic": int(hbm / fpl) if hbm is not None else None,
              "traffic_unit": "HBM bytes per frame (PMC: (2 FETCH_SIZE + WRITE_SIZE) x 1024)", "kernel": kname,
              "interval_ms": round(ms, 4), "source": os.path.relpath(pj_path, ROOT), "issue": issue, "algorithmic": alg}
    if "valu_busy_simd_cycles_per_launch" in pj:
        busy = pj["valu_busy_simd_cycles_per_launch"] / fpl
        peak = SIMD_CYCLES_PER_S
        out = {"bound": "valu", "achieved": round(busy / (ms / 1e3) / 1e9, 2), "peak": round(peak / 1e9, 1),
               "unit": "G VALU-busy SIMD-cycles/s", "frac": round(busy / (ms / 1e3) / peak, 4),
               "kind": "physical: VALU-busy SIMD cycles of " + kname + " per frame (4 x SQ_ACTIVE_INST_VALU, the "
                       "committed PMC pass of this command) / ms_per_step, against 1024 SIMDs x 2.4 GHz",
               "valu_busy_cycles_per_frame": int(busy), "lane_utilization": pj.get("valu_lane_utilization"),
               "device_interval_frac": round(busy / (dev_ms / 1e3) / peak, 4)}
        out.update(common)
        return out
    out = {"bound": "valu", "achieved": round(valu / (ms / 1e3) / 1e9, 2), "peak": round(VALU_ISSUE_PER_S / 1e9, 1),
           "unit": "G wave64-VALU-inst/s", "frac": issue["issue_frac_4cyc"],
           "kind": "physical: SQ_INSTS_VALU of " + kname + " per frame (committed PMC pass of this command) / "
                   "ms_per_step, against 1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction",
           "device_interval_frac": round(valu / (dev_ms / 1e3) / VALU_ISSUE_PER_S, 4)}
    out.update(common)
    return out


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
    # None = the measured default for the run (see resolve_shape)
    ap.add_argument("--batch", type=int, default=None, help="frames per k_trace launch (1..min(8, inflight))")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight (one stream and one set of buffers each)")
    ap.add_argument("--grid", default="",
                    help="frame-kernel launch shape 'MIN_BLOCKS_PER_WG,MAX_WORKGROUPS' (mirt_set_grid; "
                         "default: NativeFrameGroup's choice for the frames in flight)")
    ap.add_argument("--sharder", choices=("native", "torch"), default="native",
                    help="per-frame driver: native (libmirt mirt_trace_frame, RCCL called from C) or torch "
                         "(framebuffer.FrameSharder over torch.distributed)")
    ap.add_argument("--camera", choices=("static", "orbit"), default="static",
                    help="static: the scene's frame-0 camera every frame; orbit: a camera that changes every "
                         "frame (the scene camera orbited about the first object, --orbit-deg per frame, "
                         "NewCamera per frame), as the reference master issues frames while the camera moves")
    ap.add_argument("--orbit-deg", type=float, default=1.0, help="orbit step per frame (degrees)")
    ap.add_argument("--lights", choices=("static", "orbit"), default="static",
                    help="static: the scene's lights every frame; orbit: every light moves every frame (orbited "
                         "about the first object by --light-deg per frame), as EnvMutables diffs may carry "
                         "(environment.go:65-69): a new light-table key every frame")
    ap.add_argument("--light-deg", type=float, default=2.0, help="light orbit step per frame (degrees)")
    ap.add_argument("--no-d2h", action="store_true", help="leave the assembled frames in HBM (no host output)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-prefilter", action="store_true", help="ablation: always divide for r2")
    ap.add_argument("--no-octant", action="store_true", help="ablation: generic (sorted) child-box test only")
    ap.add_argument("--reflect-chains", action="store_true",
                    help="variant (--bounces): reflections as per-pixel chains in one kernel (k_reflect) instead of "
                         "level by level with rays packed in block order (k_bounce / k_pack / k_shadow)")
    ap.add_argument("--no-box-gate", action="store_true",
                    help="ablation: without the reference's face/object Box.Intersect (brute-force semantics)")
    ap.add_argument("--no-light-table", action="store_true",
                    help="ablation: shadow segments without the fp32 light-table pre-classification")
    ap.add_argument("--views", action="store_true",
                    help="experiment: per-frame view tables instead of the BVH walk (DESIGN.md §4.8)")
    ap.add_argument("--split-kernels", action="store_true",
                    help="variant: k_primary then k_shadow (default: one k_trace launch per frame)")
    ap.add_argument("--static-schedule", action="store_true",
                    help="ablation: round-robin work split instead of the dynamic work queues")
    ap.add_argument("--lds-stream", action="store_true",
                    help="(the default since round 5: meshes beyond the LDS stream each leaf's triangles "
                         "through a per-wave LDS window; accepted for older command lines)")
    ap.add_argument("--no-lds-stream", action="store_true",
                    help="ablation: meshes beyond the LDS read straight from HBM with scalar loads "
                         "(MIRT_OPT_NO_LDS_STREAM; same results)")
    ap.add_argument("--brute-force", action="store_true",
                    help="test every triangle for every ray (the north star's brute force; no BVH culling)")
    ap.add_argument("--box", type=int, default=0,
                    help="measure the box drop-in instead (mirt_box_trace_tile, DESIGN.md §5.4): one worker process "
                         "with N device entries (entry i on device i %% devices present) serving the reference "
                         "master's BulkTrace orders, --inflight frames in flight, from the native caller "
                         "worker_c/box_bench (one thread per order, as gRPC serves each in a goroutine)")
    ap.add_argument("--box-workers", type=int, default=1,
                    help="--box: the master's partition into this many rectangles per frame (master/main.go:54-91)")
    ap.add_argument("--profile-json", default="",
                    help="per-launch counters of the dominant kernel from rocprofv3 passes of this command "
                         "(tools/roofline.py writes it; used only when its launch shape equals this run's); "
                         "default: the newest profiles/*_roofline.json whose shape matches")
    a = ap.parse_args()
    resolve_shape(a)
    return a


def resolve_shape(a) -> None:
    """Frames in flight F and frames per launch B.  Measured on one MI355X: the whole 1080p frame
    runs best as 8 in flight x 1 per launch on 4 streams, each frame's D2H fused into the next
    launch on its stream (round 5: 300 frames 0.056 vs 0.060 ms at 4 x 1 with the
    copy kernel between the traces, profiles/r05_ab_fused_copy.txt; earlier shapes:
    profiles/r02_shape_sweep.txt);
    a rank's 1/N share needs more frames per launch (each workgroup then owns enough blocks
    to hide its heaviest block's chain).  An unset batch keeps at least two launches' worth of
    batch slots so launches overlap."""
    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
    F = a.inflight if a.inflight is not None else int(os.environ.get("MIRT_INFLIGHT", "16" if multi else "8"))
    B = a.batch if a.batch is not None else int(os.environ.get("MIRT_BATCH", "4" if multi else "1"))
    F = max(1, min(F, 32))
    if a.split_kernels or a.bounces:
        B = 1  # one frame per launch on those paths
    B = max(1, min(B, F, 8))
    if a.batch is None and F // B < 2 and F >= 2:
        B = max(1, F // 2)
    a.inflight, a.batch = F, B


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


def host_threads() -> int:
    """CPUs this process may run on (the box's share; os.cpu_count() shows the machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(scene_path: str, W: int, H: int) -> dict:
    """SURVEY.md §8(d) / BASELINE.md §2 CPU baselines, timed on this host:
    (i) the oracle's faithful variant (rtreego-style R-tree, 1 thread, fp64,
        worker/sequential's serial i/j loop) over one full frame — the reported value;
    (ii) the same code on all the host cores this process is allotted (the box's share for
        one GPU, 16; column-interleaved threads), and again at os.cpu_count() (`nproc`)
        threads, the whole shared machine, as SURVEY.md §8(d) words it (`threads_<nproc>`);
    (iii) brute force (every triangle, no culling), 1 thread, on every 64th column of the
        frame (a bounded sample), scaled to the full frame."""
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    sc = load_scene(scene_path)
    orc = Oracle(sc, use_rtree=True)
    out = None
    # the box allots HOST_CORES CPUs per GPU; os.cpu_count() shows the whole, shared machine,
    # so the all-cores variant runs on the allotted cores (sched_getaffinity if smaller)
    allc = max(1, min(host_threads(), HOST_CORES))
    # ... and at `nproc` threads as SURVEY.md §8(d) / BASELINE.md §2 word it (on the shared box
    # these threads contend with other tenants for the machine's cores: an upper bound, not a share)
    nproc = max(1, os.cpu_count() or 1)
    reps = 3  # the host is shared: every variant is timed three times, median and spread reported
    for threads in sorted({1, allc, nproc}):
        dts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = orc.frame(W, H, nthreads=threads)
            dts.append(time.perf_counter() - t0)
        dt = float(np.median(dts))
        rays = r["stats"]["primary_rays"] + r["stats"]["shadow_rays"]
        v = {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
             "sample": f"one full {W}x{H} frame ({rays} primary+shadow rays), oracle/rt_oracle.c with "
                       f"rtreego-style R-tree culling, {threads} thread(s), median of {reps} runs {dt:.2f} s",
             "ms_per_frame": round(dt * 1e3, 1), "repeats": reps,
             "spread_mrays_s": [round(rays / max(dts) / 1e6, 4), round(rays / min(dts) / 1e6, 4)]}
        if out is None:
            out = v
        else:
            out[f"threads_{threads}"] = {k: v[k] for k in ("value", "cores", "ms_per_frame", "repeats", "spread_mrays_s")}
            if threads == nproc:
                out[f"threads_{threads}"]["note"] = ("variant (ii) at nproc (BASELINE.md §2): the whole shared "
                                                     "machine, whose other CPUs serve other jobs' GPUs")
    cols = list(range(0, W, 64))
    brute = Oracle(sc, use_rtree=False)
    t0 = time.perf_counter()
    r = brute.trace_tiles(W, H, [(x, 0, 1, H) for x in cols], nthreads=1)
    dt = time.perf_counter() - t0
    rays = r["stats"]["primary_rays"] + r["stats"]["shadow_rays"]
    out["brute_force_1_thread"] = {
        "value": round(rays / dt / 1e6, 4), "cores": 1,
        "ms_per_frame": round(dt * 1e3 * W / len(cols), 1),
        "sample": f"every 64th column ({len(cols)} x {H} px, {rays} rays) in {dt:.2f} s, scaled x{W / len(cols):.0f}"}
    out["nproc"] = os.cpu_count()
    out["affinity_cpus"] = host_threads()
    return out


def orbit_cameras(cam_pos, cam_dir, fov, center, n: int, step_deg: float):
    """n cameras orbiting `center` about the world y axis from the scene camera's position,
    each looking at the center: (pos, forward, fov) for NewCamera (camera.go:35-44), which
    normalises the forward itself.  Frame data only — the reference's camera motion code is
    out of scope."""
    import math
    c = np.asarray(center, np.float64)
    r = np.asarray(cam_pos, np.float64) - c
    out = []
    for k in range(n):
        a = math.radians(step_deg * k)
        ca, sa = math.cos(a), math.sin(a)
        p = c + np.array([ca * r[0] + sa * r[2], r[1], -sa * r[0] + ca * r[2]])
        out.append((tuple(p), tuple(c - p), fov))
    return out


def orbit_lights(lights, center, n: int, step_deg: float):
    """n light sets: every light of the scene rotated about the world y axis through `center`
    by step_deg x k in frame k (positions only; colours kept).  Frame data only."""
    import math
    c = np.asarray(center, np.float64)
    out = []
    for k in range(n):
        a = math.radians(step_deg * k)
        ca, sa = math.cos(a), math.sin(a)
        ls = []
        for lt in lights:
            r = np.asarray(lt.pos, np.float64) - c
            ls.append(dataclasses.replace(lt, pos=tuple(float(x) for x in
                                                        c + np.array([ca * r[0] + sa * r[2], r[1], -sa * r[0] + ca * r[2]]))))
        out.append(ls)
    return out


def parity_check(fb_valid: np.ndarray, fb_rgb8: np.ndarray, scene_path: str, W: int, H: int,
                 bounces: int = 0, camera=None, lights=None, fb_rgb=None) -> dict:
    """Parity gate of the timed frames: EVERY pixel of the last timed
    frame against the oracle (R-tree restatement, 16 threads), valid mask and rgb8
    bit-exact; with the D2H on, the frame checked is the host copy.  fb_rgb: the fp64
    colour plane of the same frame's inputs (north_star's bound: within 1e-5 per channel;
    checked bit-exact as well)."""
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    sc = load_scene(scene_path)
    if camera is not None or lights is not None:  # a moving camera's / moving lights' last timed frame
        import copy
        sc = copy.copy(sc)
        if camera is not None:
            sc.cam_pos, sc.cam_dir, sc.fov = tuple(map(float, camera[0])), tuple(map(float, camera[1])), float(camera[2])
        if lights is not None:
            sc.lights = [(tuple(lt.pos), tuple(lt.col)) for lt in lights]
    orc = Oracle(sc, use_rtree=True)
    orc.set_bounces(bounces)
    ref = orc.frame(W, H, nthreads=HOST_CORES)
    ok = bool(np.array_equal(fb_valid, ref["valid"]) and np.array_equal(fb_rgb8, ref["rgb8"]))
    out = {"pixels_checked": W * H, "bit_exact": ok, "hits": int(fb_valid.sum())}
    if fb_rgb is not None:
        d = float(np.abs(fb_rgb - ref["rgb"]).max()) if fb_rgb.shape == ref["rgb"].shape else float("inf")
        out["rgb_f64"] = {"bit_exact": bool(np.array_equal(fb_rgb, ref["rgb"])), "max_abs_diff": d,
                          "within_1e-5": bool(d <= 1e-5)}
        out["bit_exact"] = bool(ok and out["rgb_f64"]["bit_exact"])
    return out


def load_profile(path: str, shape: dict):
    """The committed rocprofv3 summary of THIS command (tools/roofline.py), if its launch
    shape matches; counters from another shape are never mixed in."""
    if not os.path.exists(path):
        return None
    try:
        pj = json.load(open(path))
    except (OSError, ValueError):
        return None
    ps = pj.get("shape", {})
    # the same shape both ways: a profile of a variant (a key this run lacks, e.g. moving lights)
    # is never cited for the plain command
    if any(ps.get(k) != v for k, v in shape.items()) or any(k not in shape for k in ps):
        return None
    return pj


def box_main(a) -> None:
    """--box N: the box drop-in under the reference master's traffic.  The
    native caller worker_c/box_bench keeps --inflight frames in flight, each frame's
    --box-workers rectangles (master/main.go:54-91) served concurrently by mirt_box_trace_tile
    into host buffers (rgb8: what TraceResults carries); ms_per_step = wall time / frames.  The
    last frame, assembled as the master draws it, is checked against the oracle (rgb8, every
    pixel)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "worker_c", "box_bench")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} is missing: run __graft_entry__.build()")
    W, H = a.width, a.height
    F = a.inflight
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "frame.bin")
        cmd = [exe, a.scene, str(W), str(H), str(a.box), str(a.box_workers), str(F), str(a.steps), str(a.warmup), out]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            raise SystemExit(f"box_bench failed ({p.returncode}): {p.stderr[-2000:]}")
        r = json.loads(p.stdout.strip().splitlines()[-1])
        rgb8 = np.fromfile(out, np.uint8).reshape(W * H, 3)
        timers = [ln for ln in p.stderr.splitlines() if ln.startswith("box_timers")]
    ms = r["ms_per_frame"]
    line = {
        "metric": METRIC, "value": round(r["rays_per_frame"] / (ms / 1e3) / 1e6, 3), "unit": "Mrays/s", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: the reference's own example/scene.json, static frame-0 camera",
        "config": {"workload": f"box drop-in: {os.path.basename(a.scene)} {W}x{H} served as the reference master's "
                               f"BulkTrace orders ({r['orders_per_frame']} per frame) by one worker process of "
                               f"{a.box} device entries",
                   "width": W, "height": H, "box_entries": a.box, "master_workers": a.box_workers,
                   "orders_per_frame": r["orders_per_frame"], "transport": {1: "rccl", 2: "device copies", 3: "host"}.get(
                       r["transport"], r["transport"]), "devices_present": r["devices"],
                   "outputs": "rgb8 into the caller's host buffer (TraceResults colours)"},
        "frames_in_flight": F, "rays_per_frame": r["rays_per_frame"], "hits_per_frame": r["hits_per_frame"],
        "caller": "worker_c/box_bench (native threads, one per order)",
    }
    if timers:  # MIRT_BOX_TIMERS=1: host time per phase of an order (warmup orders included)
        line["box_timers"] = timers[-1]
    if not a.no_parity:
        from oracle.oracle import Oracle
        from oracle.scene_py import load_scene
        ref = Oracle(load_scene(a.scene), use_rtree=True).frame(W, H, nthreads=HOST_CORES)
        line["parity"] = {"pixels_checked": W * H, "bit_exact": bool(np.array_equal(rgb8, ref["rgb8"])),
                          "frame": "last timed frame, orders assembled on the host as master/main.go:164-176 draws them"}
    print(json.dumps(line), flush=True)


def main():
    a = parse()
    if a.box:
        return box_main(a)
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
        # a collective that never completes (a rank that died before joining) fails the run
        # after MIRT_DIST_TIMEOUT_S instead of hanging it
        import datetime
        to = datetime.timedelta(seconds=int(os.environ.get("MIRT_DIST_TIMEOUT_S", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=to)
        else:
            dist.init_process_group(backend, timeout=to)

    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder, NativeFrameGroup

    W, H = a.width, a.height
    ctx = rt.Context(local)
    opts = (rt._lib.MIRT_OPT_NO_OCTANT if a.no_octant else 0) | (rt._lib.MIRT_OPT_NO_PREFILTER if a.no_prefilter else 0) | (
        rt._lib.MIRT_OPT_BRUTE_FORCE if a.brute_force else 0) | (
        rt._lib.MIRT_OPT_STATIC_SCHEDULE if a.static_schedule else 0) | (rt._lib.MIRT_OPT_SPLIT_KERNELS if a.split_kernels else 0) | (
        rt._lib.MIRT_OPT_VIEWS if a.views else 0) | (rt._lib.MIRT_OPT_NO_LIGHT_TABLE if a.no_light_table else 0) | (
        rt._lib.MIRT_OPT_REFLECT_CHAINS if a.reflect_chains else 0) | (rt._lib.MIRT_OPT_NO_BOX_GATE if a.no_box_gate else 0) | (
        rt._lib.MIRT_OPT_LDS_STREAM if a.lds_stream else 0) | (rt._lib.MIRT_OPT_NO_LDS_STREAM if a.no_lds_stream else 0)
    ctx.set_options(opts)
    env = rt.Environment.from_file(a.scene, ctx)
    import dataclasses
    base = dataclasses.replace(env.mutable(), max_bounces=a.bounces)
    cams = [None]
    lsets = [None]
    nseq = max(a.steps, a.warmup) if (a.camera == "orbit" or a.lights == "orbit") else 1
    if a.camera == "orbit":
        c = base.cam
        cams = orbit_cameras(c.pos, c.forward, c.fov, base.objects[0].pos, nseq, a.orbit_deg)
    if a.lights == "orbit":
        lsets = orbit_lights(base.lights, base.objects[0].pos, nseq, a.light_deg)
    seq = []
    for k in range(nseq):
        m = base
        if a.camera == "orbit":
            m = dataclasses.replace(m, cam=rt.Camera.new(*cams[k]))
        if a.lights == "orbit":
            m = dataclasses.replace(m, lights=lsets[k])
        seq.append(m.to_frame())

    def frame_at(k):
        return seq[k % len(seq)]
    tris = sum(len(m.face_v) for m in env.meshes)
    nl = len(env.mutable().lights)
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local]) if backend == "nccl" else dist.barrier()

    # native: the per-frame trace + RCCL gather + unpack (+ D2H) in libmirt (mirt_trace_frame),
    # one C call per frame; torch: the same sequence through torch.distributed (FrameSharder),
    # used for the gloo rehearsal (RCCL cannot put two ranks on one GPU).  The choice is
    # collective: if any rank cannot create the native group, every rank uses torch.
    sharder = a.sharder if not (world > 1 and backend != "nccl") else "torch"
    d2h = not a.no_d2h and sharder == "native"

    def native_group(host_output: bool):
        # N > 1: every host wait of the group is deadline-bounded, so a rank whose transfers never
        # arrive fails the run (MIRT_E_TIMEOUT / MIRT_E_PEER naming it) instead of hanging it
        return NativeFrameGroup(ctx, W, H, rank, world, a.tile if world > 1 else None, inflight=a.inflight,
                                tile_h=a.tile_h, batch=a.batch, host_output=host_output and rank == 0,
                                timeout_ms=int(os.environ.get("MIRT_GROUP_TIMEOUT_MS", "60000")) if world > 1 else 0)

    sh = None
    err = ""
    if sharder == "native":
        try:
            sh = native_group(d2h)
        except Exception as e:  # noqa: BLE001 — reported in the JSON line, then the torch path runs
            err = str(e)
    if world > 1 and sharder == "native":
        ok = torch.tensor([0.0 if sh is None else 1.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() < 1.0:
            sh = None
            err = err or "another rank could not create its native group"
    if sharder == "native" and sh is None:
        print(f"native frame group unavailable ({err}); using the torch.distributed sharder", file=sys.stderr)
        sharder, d2h = f"torch (native failed: {err})", False
    if sh is None:
        # the torch.distributed path was tuned at 4 in flight (one frame per launch)
        sh = FrameSharder(ctx, W, H, rank, world, a.tile, inflight=min(a.inflight, 4), tile_h=a.tile_h)
    if a.grid:
        ctx.set_grid(*(int(x) for x in a.grid.split(",")))

    def finish():
        """The enqueued frames are done (gathers, unpacks and D2H included): a host wait on
        the group's completion events (hipEventSynchronize, or within the group's deadline at
        N > 1); the torch.cuda.synchronize() that follows brackets the steps.  Waiting on the
        events first keeps the runtime's blocking device-wide wait, which had returned ~120 us
        after the last kernel ended (rocprofv3 HIP trace), out of the measured
        time.  The torch.distributed sharder: torch's stream waits for its streams."""
        if isinstance(sh, NativeFrameGroup):
            # the host wait covers every batch, gathers included: torch's stream has nothing
            # left to wait for (a flush here only cost ~20-40 us of host time)
            sh.wait()
        else:
            sh.flush()

    # launches per region (the key that partitions the rocprofv3 kernel trace of this command)
    launches = {}

    def count(region, n_frames, batched=True):
        per = a.batch if (batched and hasattr(sh, "B")) else 1
        launches[region] = launches.get(region, 0) + (n_frames + per - 1) // per

    stream = torch.cuda.Stream(dev)
    host_last = None
    with torch.cuda.stream(stream):
        for k in range(a.warmup):
            sh.render(frame_at(k))
        finish()
        count("warmup", a.warmup)
        torch.cuda.synchronize(dev)

        # timed region: K frames from an empty pipeline to the last one in host memory
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        last = None
        for k in range(a.steps):
            last = sh.render(frame_at(k))  # N > 1: frame k's gather overlaps frame k+1's tracing
        finish()                     # the last frame's gather + unpack (+ D2H) are inside the timed region
        torch.cuda.synchronize(dev)
        barrier()
        t1 = time.perf_counter()
        count("timed", a.steps)
        if d2h and rank == 0:
            # the D2H'd frame (checked against the oracle below): views of the pinned planes
            # now, copied after the device-only region (which leaves host output off), so the
            # GPU does not idle through a host copy (33 MB at 4K) between the two regions
            host_last = sh.host_frame(last, copy=False)

        # the same frames without the D2H (device-resident outputs)
        dev_elapsed = None
        if d2h:
            if rank == 0:
                sh.set_host_output(False)
            barrier()
            torch.cuda.synchronize(dev)
            d0 = time.perf_counter()
            for k in range(a.steps):
                sh.render(frame_at(k))
            finish()
            torch.cuda.synchronize(dev)
            barrier()
            dev_elapsed = time.perf_counter() - d0
            count("device_only", a.steps)
            if host_last is not None:
                host_last = tuple(x.copy() for x in host_last)
            if rank == 0:
                sh.set_host_output(True)

        # profiled region: HIP events around every k_trace launch + device counters
        ctx.profile_enable(True)
        for k in range(a.steps):
            sh.render(frame_at(k))
        finish()
        torch.cuda.synchronize(dev)
        ctx.profile_enable(False)
        count("profiled", a.steps)

        # single-frame latency: one frame alone (render, gather + unpack, D2H, host sync), median
        lat = []
        for k in range(min(a.steps, 20)):
            barrier()
            torch.cuda.synchronize(dev)
            l0 = time.perf_counter()
            sh.render(frame_at(k))
            finish()
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - l0)
        count("latency", min(a.steps, 20), batched=False)
        latency = float(np.median(lat)) if lat else 0.0
    prof = ctx.profile_read()

    elapsed = t1 - t0
    pl = max(prof["frames"], 1)  # per-frame device counters (a launch may trace several frames)
    counts = torch.tensor([elapsed, latency, dev_elapsed or 0.0, prof["primary_rays"] / pl, prof["shadow_rays"] / pl,
                           prof["hits"] / pl, prof["reflection_rays"] / pl], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
    if world > 1:
        tmax = counts[:3].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = counts[3:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed, latency, dev_elapsed_max = (float(x) for x in tmax.tolist())
        dev_elapsed = dev_elapsed_max if dev_elapsed is not None else None
        primary, shadow, hits, refl = (float(x) for x in sums.tolist())
    else:
        primary, shadow, hits, refl = (float(x) for x in counts[3:].tolist())

    if rank == 0:
        steps = a.steps
        ms = elapsed / steps * 1e3
        rays_per_frame = primary + shadow + refl  # per frame, all ranks (device counters)
        nlaunch = max(prof["launches"], 1)
        prim_ms = prof["primary_ms_sum"] / nlaunch
        # the algorithmic roofline's launch time: the median launch (a mean counts the odd launch
        # that queued behind an overlapped frame: 665 us against a 191 us rocprof average, r03z)
        prim_med = prof["primary_ms_median"] or prim_ms
        # the dominant kernel: k_trace (the whole frame, one launch); split frames: k_primary;
        # reflection frames: k_shadow (level 0 and each bounce level: the most time per frame,
        # profiles/r03config4_kernel_stats.csv), or k_reflect on the chain path (2.67 of 3.81 ms)
        one = not a.split_kernels and not a.bounces
        kname = "k_trace" if one else (("k_reflect" if a.reflect_chains else "k_shadow") if a.bounces else "k_primary")
        if a.bounces:
            # the algorithmic figure over all the frame's kernels: the reflection levels' tests are
            # counted with the shadow rays' (one statistic), so the whole frame's tests / its time
            k_tests = (prof["primary_tri_tests"] + prof["shadow_tri_tests"]) / nlaunch
            alg_ms = prof["frame_ms_median"] or prof["frame_ms_sum"] / nlaunch
            alg_mean = prof["frame_ms_sum"] / nlaunch
            alg_kernel = ("k_primary + k_shadow + k_reflect" if a.reflect_chains else
                          "k_primary + k_pack + k_bounce + k_shadow (levels 0..bounces) + k_refl_fold")
        else:
            k_tests = (prof["primary_tri_tests"] + (prof["shadow_tri_tests"] if one else 0)) / nlaunch
            alg_ms, alg_kernel, alg_mean = prim_med, kname, prim_ms
        achieved = k_tests * BYTES_PER_TRI_TEST / (alg_ms / 1e3) / 1e9
        shape = {"width": W, "height": H, "gpus": world, "inflight": a.inflight, "batch": a.batch,
                 "steps": steps, "warmup": a.warmup, "d2h": d2h, "kernel": kname,
                 "scene": scene_tag(a.scene), "bounces": a.bounces, "options": opts, "camera": a.camera}
        if a.lights != "static":
            shape["lights"] = a.lights
        build_id = rt._lib.lib().mirt_build_id().decode()
        pj, pj_path, why_not = find_profile(a.profile_json, shape, build_id)
        frames_per_launch = pl / nlaunch
        dev_ms = dev_elapsed / steps * 1e3 if dev_elapsed else ms
        line = {
            "metric": METRIC,
            # value: BASELINE.md §3 / SURVEY.md §8(d) Mrays/s = rays per frame / ms per frame with
            # the D2H of the assembled frame into host memory (ms_per_step); the device-resident
            # rate (outputs left in HBM) is device_mrays_s
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
            "data": ("synthetic: the reference's own example/scene.json (suzanne.obj, 968 tris, 3 lights), " + (
                         "static frame-0 camera" if a.camera == "static" else
                         f"camera orbiting the object {a.orbit_deg} deg per frame (a new camera every frame)")
                     if os.path.abspath(a.scene) == os.path.abspath(SCENE) else
                     f"synthetic: {os.path.relpath(a.scene, ROOT)} ({tris} tris, {nl} lights), the scene's camera") + (
                     f"; lights orbiting the object {a.light_deg} deg per frame (a new light set every frame)"
                     if a.lights == "orbit" else ""),
            "config": {"workload": workload_name(a, W, H, tris, nl), "width": W, "height": H, "triangles": tris,
                       "lights": nl, "parallelism": f"image tiles x{world}" + (f" ({a.tile}px, RCCL gather)"
                                                                                if world > 1 else ""),
                       "culling": "none (brute force)" if a.brute_force else "exact BVH (packet traversal)",
                       "d2h": "rgb8 + valid to pinned host memory inside the timed region" if d2h else "none (HBM)",
                       "scene": scene_tag(a.scene), "bounces": a.bounces, "options": opts, "camera": a.camera,
                       "light_motion": a.lights},
            "frames_in_flight": getattr(sh, "F", a.inflight),
            "frames_per_launch": getattr(sh, "B", 1),
            "sharder": sharder,
            "value_basis": "rays_per_frame / ms_per_step; ms_per_step includes the D2H of the assembled rgb8 + "
                           "valid frame into pinned host memory (BASELINE.md §3)" if d2h else
                           "rays_per_frame / ms_per_step (outputs left in HBM: --no-d2h)",
            "device_ms_per_frame": round(dev_ms, 4),
            "device_mrays_s": round(rays_per_frame / (dev_ms / 1e3) / 1e6, 3),
            "frame_latency_ms": round(latency * 1e3, 4),
            "primary_mrays_s": round(primary / (dev_ms / 1e3) / 1e6, 3),
            "rays_per_frame": int(rays_per_frame),
            "hits_per_frame": int(hits),
            "tri_tests_per_frame": int((prof["primary_tri_tests"] + prof["shadow_tri_tests"]) / pl),
            "bvh_visits_per_frame": {k: int(prof[k] / pl) for k in (
                "primary_node_visits", "primary_leaf_visits", "shadow_node_visits", "shadow_leaf_visits")},
            "ms_kernels": {("frame_kernel" if one else "primary"): round(prim_ms, 4),
                           "shadow": round(prof["shadow_ms_sum"] / nlaunch, 4),
                           "reflect": round(prof["reflect_ms_sum"] / nlaunch, 4),
                           "frame_device": round(prof["frame_ms_sum"] / nlaunch, 4)},
            "launches": launches,
            "redo_items": int(prof.get("redo_items", 0)),
            "light_cache": ctx.light_cache_stats(),
            "build_id": build_id,
            "roofline": roofline_block(pj, pj_path, kname, ms, dev_ms, achieved, k_tests, frames_per_launch,
                                       alg_ms, mesh_lds_resident=tris <= LDS_RESIDENT_FACES, alg_kernel=alg_kernel,
                                       launch_ms_mean=alg_mean, why_not=why_not,
                                       tests_per_frame=(prof["primary_tri_tests"] + prof["shadow_tri_tests"]) / pl),
        }
        # north_star prices its target as bytes/tri-test x tris x rays: the work
        # a brute-force sweep would do.  Culling removes almost all of it, so this "effective"
        # rate is far above any physical peak and says nothing about kernel quality; it is kept
        # as a figure, not as a target met.  `roofline` counts the tests actually performed and
        # `roofs` the physical limits.
        bf_bytes = BYTES_PER_TRI_TEST * float(tris) * rays_per_frame
        line["brute_force_equivalent"] = {
            "definition": "72 B x triangles x rays per frame (the work a brute-force sweep would do) / device ms "
                          "per frame: an effective rate, not a bandwidth",
            "effective_tb_s": round(bf_bytes / (dev_ms / 1e3) / 1e12, 1)}
        if pj:
            # physical roofs over the frame interval (counters of this exact command, profiles/)
            per_frame = lambda x: x / pj["frames_per_launch"]  # noqa: E731
            iv = ms / 1e3  # the headline frame interval (ms_per_step)
            valu = per_frame(pj["sq_insts_valu_per_launch"])
            line["roofs"] = {
                "source": os.path.relpath(pj_path, ROOT),
                "frame_interval_ms": round(ms, 4),
                "valu_issue_frac": round(valu / iv / VALU_ISSUE_PER_S, 4),
                "valu_insts_per_frame": int(valu),
                "salu_insts_per_frame": int(per_frame(pj["sq_insts_salu_per_launch"])),
                "fp64_tflops": round(64 * per_frame(pj["fp64_flops_per_launch"]) / iv / 1e12, 3),
                "fp64_frac": round(64 * per_frame(pj["fp64_flops_per_launch"]) / iv / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                "hbm_bytes_per_frame": int(per_frame(pj["hbm_bytes_per_launch"])),
                "hbm_frac": round(per_frame(pj["hbm_bytes_per_launch"]) / iv / 1e9 / HBM_PEAK_GBS, 4),
                "output_bytes_per_frame": W * H * 4,
            }
        if not a.no_parity and rank == 0:
            if host_last is not None:
                rgb8, valid = host_last
            else:
                fr = sh.frame
                rgb8, valid = fr.rgb8.cpu().numpy(), fr.valid.cpu().numpy()
            # the fp64 colour of the last timed frame's inputs: the timed frames write rgb8 + valid
            # (what BulkTrace returns), so the same frame is traced once more through the frame
            # group with the device fp64 rgb plane on, after every timed region
            g2 = NativeFrameGroup(ctx, W, H, 0, 1, None, inflight=1, with_rgb=True)
            try:
                g2.render(frame_at(a.steps - 1))
                g2.wait()
                g2.flush()
                torch.cuda.synchronize(dev)
                rgb64 = g2.frames[0].rgb.cpu().numpy()
            finally:
                g2.close()
            count("parity_rgb", 1, batched=False)  # (the launches key partitions the kernel trace)
            line["launches"] = launches
            line["parity"] = parity_check(valid, rgb8, a.scene, W, H, a.bounces,
                                          cams[(a.steps - 1) % len(cams)] if a.camera == "orbit" else None,
                                          lsets[(a.steps - 1) % len(lsets)] if a.lights == "orbit" else None,
                                          fb_rgb=rgb64)
            line["parity"]["frame"] = "host copy (D2H)" if host_last is not None else "device framebuffer"
            line["parity"]["rgb_f64"]["frame"] = ("device fp64 rgb plane of the last timed frame's inputs, traced "
                                                  "again through the frame group with the plane on")
        if not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(a.scene, W, H)
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
