"""Per-wave timeline of one frame (MIRT_OPT_TIMELINE): when waves start and end, the
shader clock they ran at, work items per wave, per-XCD spread.

usage (GPU box): python tools/timeline.py [--width W --height H --frames N --static]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(rec: np.ndarray) -> dict:
    out = {}
    for kern, name in ((0, "primary"), (1, "shadow")):
        r = rec[rec[:, 0] == kern].astype(np.float64)
        if not len(r):
            continue
        t0 = r[:, 2].min()
        start = (r[:, 2] - t0) * 10.0  # 100 MHz ticks -> ns
        end = (r[:, 3] - t0) * 10.0
        life = end - start
        clk_ghz = (r[:, 5] - r[:, 4]) / np.maximum(life, 1.0)
        items = (r[:, 7].astype(np.uint64) >> np.uint64(32)).astype(np.float64)
        xcc = (r[:, 7].astype(np.uint64) & np.uint64(0xffff)).astype(np.int64)
        staged = np.where(r[:, 6] > 0, (r[:, 6] - t0) * 10.0, np.nan)
        q = lambda a: [round(float(np.percentile(a, p)) / 1e3, 2) for p in (0, 10, 50, 90, 100)]
        out[name] = {
            "waves": int(len(r)),
            "span_us": round(float(end.max()) / 1e3, 2),
            "start_us_p0_10_50_90_100": q(start),
            "end_us_p0_10_50_90_100": q(end),
            "mean_life_frac_of_span": round(float(life.mean() / end.max()), 3),
            "staged_us_p50_100": [round(float(np.nanpercentile(staged, p)) / 1e3, 2) for p in (50, 100)]
            if np.isfinite(staged).any() else None,
            "shader_clock_ghz_median": round(float(np.median(clk_ghz)), 3),
            "items_per_wave_p0_50_100": [int(np.percentile(items, p)) for p in (0, 50, 100)],
            "per_xcc_end_us_max": {int(x): round(float(end[xcc == x].max()) / 1e3, 2) for x in np.unique(xcc)},
        }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--static", action="store_true")
    ap.add_argument("--opts", type=int, default=0, help="extra MIRT_OPT_* bits")
    ap.add_argument("--save", default="")
    ap.add_argument("--view", default="default", choices=("default", "away"))
    ap.add_argument("--phase", action="store_true",
                    help="library built with -DMIRT_PHASE_TIMING=1 (MIRT_LIB): cycles per primary phase")
    a = ap.parse_args()
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import FrameSharder
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    mut = env.mutable()
    if a.view == "away":
        c = mut.cam
        mut = rt.EnvMutables(mut.objects, mut.lights, rt.Camera.new(c.pos, tuple(-np.asarray(c.forward)), c.fov))
    frame = mut.to_frame()
    sh = FrameSharder(ctx, a.width, a.height, 0, 1, 64)
    opts = rt._lib.MIRT_OPT_TIMELINE | (rt._lib.MIRT_OPT_STATIC_SCHEDULE if a.static else 0) | a.opts
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        ctx.set_options(0)
        for _ in range(3):
            sh.render(frame)
        torch.cuda.synchronize()
        ctx.set_options(opts)
        res = []
        for _ in range(a.frames):
            sh.render(frame)
            torch.cuda.synchronize()
            rec = ctx.debug_timeline()
            if a.phase:
                r = rec[rec[:, 0] == 0].astype(np.float64)
                items = (r[:, 7].astype(np.uint64) >> np.uint64(32)).astype(np.float64)
                res.append({"primary_cycles_per_block": {
                    "raygen_trace": round(float(r[:, 4].sum() / items.sum())),
                    "outputs_hits": round(float(r[:, 5].sum() / items.sum())),
                    "between_blocks": round(float(r[:, 6].sum() / items.sum()))},
                    "wave_life_cycles_per_block": round(float(((r[:, 3] - r[:, 2]) * 10 * 2.17).sum() / items.sum()))})
            else:
                res.append(summarize(rec))
            if a.save:
                np.save(a.save, rec)
        ctx.set_options(0)
    for r in res[-2:]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
