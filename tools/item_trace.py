"""Per-work-item timeline of one k_trace frame (diagnostic build, MIRT_ITEM_TRACE):
how long primary blocks and shadow items take on one wave, and what the last
workgroups were doing.  Build the library first (on the CPU host):
  make -C distributed_raytracer_amd/csrc EXTRA='-DMIRT_ITEM_TRACE=1 -DMIRT_PHASE_TIMING=1' OBJ=obj_item OUT=../libmirt_item.so
usage (GPU box): MIRT_LIB=distributed_raytracer_amd/libmirt_item.so python tools/item_trace.py [--world 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(rec: np.ndarray) -> dict:
    r = rec.astype(np.float64)
    t0 = r[:, 2].min()
    start = (r[:, 2] - t0) / 100.0  # 100 MHz ticks -> us
    end = (r[:, 3] - t0) / 100.0
    dur = end - start
    kind = rec[:, 0]
    wg = rec[:, 1]
    tests = r[:, 6]
    nodes = (rec[:, 7] & 0xffffffff).astype(np.float64)
    hits = (rec[:, 7] >> 32).astype(np.float64)
    q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 50, 90, 99, 100)] if len(a) else []
    prim = kind == 0
    culled = prim & (nodes == 1) & (tests == 0)
    prim_hit = prim & (hits > 0)
    prim_miss = prim & ~culled & (hits == 0)
    sh = kind == 1
    out = {
        "span_us": round(float(end.max()), 2),
        "items": int(len(rec)),
        "primary_culled": {"n": int(culled.sum()), "dur_us_p0_50_90_99_100": q(dur[culled])},
        "primary_miss": {"n": int(prim_miss.sum()), "dur_us_p0_50_90_99_100": q(dur[prim_miss])},
        "primary_hit": {"n": int(prim_hit.sum()), "dur_us_p0_50_90_99_100": q(dur[prim_hit]),
                         "tests_p50_100": [float(np.percentile(tests[prim_hit], p)) for p in (50, 100)] if prim_hit.any() else []},
        "primary_hit_phase_kcycles_raygen_trace_p50_100": [
            [round(float(np.percentile((rec[prim_hit, 5] & 0xffffffff).astype(np.float64), p)) / 1e3, 1) for p in (50, 100)],
            [round(float(np.percentile((rec[prim_hit, 5] >> 32).astype(np.float64), p)) / 1e3, 1) for p in (50, 100)],
            [round(float(np.percentile(r[prim_hit, 4], p)) / 1e3, 1) for p in (50, 100)]] if prim_hit.any() else [],
        "first_item_start_us_per_wg_p0_50_100": q(np.array([start[wg == w].min() for w in np.unique(wg)])),
        "shadow": {"n": int(sh.sum()), "dur_us_p0_50_90_99_100": q(dur[sh]),
                   "tests_p50_100": [float(np.percentile(tests[sh], p)) for p in (50, 100)] if sh.any() else []},
        "sum_item_us": {"primary": round(float(dur[prim].sum()), 1), "shadow": round(float(dur[sh].sum()), 1)},
    }
    # per workgroup: end time, busy wave-time; the latest workgroups' last items
    wgs = np.unique(wg)
    wend = np.array([end[wg == w].max() for w in wgs])
    wbusy = np.array([dur[wg == w].sum() for w in wgs])
    out["wg_end_us_p0_50_90_100"] = q(wend)
    out["wg_busy_wave_us_p0_50_90_100"] = q(wbusy)
    late = wgs[np.argsort(wend)[-3:]]
    out["latest_wgs"] = []
    for w in late:
        m = wg == w
        order = np.argsort(start[m])
        items = [[int(kind[m][i]), round(float(start[m][i]), 1), round(float(dur[m][i]), 1), int(tests[m][i]),
                  int(hits[m][i])] for i in order if dur[m][i] > 2.0]
        out["latest_wgs"].append({"wg": int(w), "end_us": round(float(end[m].max()), 1),
                                  "busy_wave_us": round(float(dur[m].sum()), 1),
                                  "items_over_2us[kind,start,dur,tests,hits]": items[-12:]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--save", default="")
    a = ap.parse_args()
    import torch
    import distributed_raytracer_amd as rt
    from distributed_raytracer_amd.framebuffer import alloc_planes, assign, plan_tiles, pixels_of, trace_tiles_device
    ctx = rt.Context(0)
    env = rt.Environment.from_file(os.path.join(ROOT, "tests", "golden", "example", "scene.json"), ctx)
    frame = env.mutable().to_frame()
    W, H = 1920, 1080
    tiles = [(0, 0, W, H)] if a.world == 1 else assign(plan_tiles(W, H, 64), a.world, a.rank)
    planes = alloc_planes(pixels_of(tiles), torch.device("cuda", 0))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(5):
            trace_tiles_device(ctx, frame, W, H, tiles, planes, s.cuda_stream)
        torch.cuda.synchronize()
        ctx.set_options(rt._lib.MIRT_OPT_TIMELINE)
        for k in range(3):
            trace_tiles_device(ctx, frame, W, H, tiles, planes, s.cuda_stream)
            torch.cuda.synchronize()
            rec = ctx.debug_timeline(1 << 18)
            res = analyse(rec)
            if a.save:
                np.save(a.save, rec)
        ctx.set_options(0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
