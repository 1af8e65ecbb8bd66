"""Condense a tools/profile_cmd.sh run (gpurun_out/prof_<tag>) into the files bench.py and
the judge read:

  python tools/roofline.py r02

  profiles/<tag>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary of the command (verbatim)
  profiles/<tag>_roofline.json     per k_trace launch, for the launches of each bench region:
                                   mean duration (kernel trace), HBM bytes, VALU/SALU/FP64 counts
                                   (PMC passes of the same command), the launch shape

The bench line of the trace pass names how many k_trace launches each region made, in
order (warmup, timed, device_only, profiled, latency); the k_trace dispatches of every pass
are split the same way, so the profiled region's mean duration here is the denominator of
the bench's `roofline.achieved` (HIP events around the same launches) and `frac` follows
from this file.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
in KiB from separate passes and gfx950's FETCH_SIZE counts half the bytes of wide streaming
reads, so hbm = (2 FETCH_SIZE + WRITE_SIZE) x 1024 (an upper bound for narrower reads).
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_trace"
ORDER = ("warmup", "timed", "device_only", "profiled", "latency")


def bench_line(log: str) -> dict:
    for ln in reversed(open(log).read().splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    raise SystemExit(f"no bench JSON line in {log}")


def regions(dispatches, launches: dict):
    """dispatch ids (submission order) -> region name, by the bench's launch counts."""
    names = [r for r in ORDER if launches.get(r)]
    total = sum(launches[r] for r in names)
    if len(dispatches) != total:
        raise SystemExit(f"{len(dispatches)} {KERNEL} dispatches but the bench reports {total} launches {launches}")
    out, i = {}, 0
    for r in names:
        for d in dispatches[i:i + launches[r]]:
            out[d] = r
        i += launches[r]
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    line = bench_line(os.path.join(src, "trace.log"))
    launches = line["launches"]
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats_avg = None
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if KERNEL in r["Name"]:
            stats_avg = float(r["AverageNs"])
    # kernel trace: duration per region
    rows = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    reg = regions([int(r["Dispatch_Id"]) for r in rows], launches)
    dur = collections.defaultdict(list)
    for r in rows:
        dur[reg[int(r["Dispatch_Id"])]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {
        "tag": tag,
        "command": "python3 bench.py " + open(os.path.join(src, "args.txt")).read().split("args:", 1)[1].strip(),
        "kernel": KERNEL,
        "shape": {"width": line["config"]["width"], "height": line["config"]["height"], "gpus": line["n_gpus"],
                  "inflight": line["frames_in_flight"], "batch": line["frames_per_launch"], "steps": line["steps"],
                  "warmup": line["warmup"], "d2h": line["config"].get("d2h", "").startswith("rgb8"),
                  "kernel": line["roofline"]["kernel"]},
        "frames_per_launch": line["roofline"]["frames_per_launch"],
        "launches": launches,
        "stats_avg_ns_all_launches": stats_avg,
        "avg_ns_by_region": {k: sum(v) / len(v) for k, v in dur.items()},
        "launch_count_by_region": {k: len(v) for k, v in dur.items()},
        "trace_pass_bench": {k: line.get(k) for k in ("ms_per_step", "device_ms_per_frame", "frame_latency_ms", "value")},
        "trace_pass_roofline": line["roofline"],
    }
    # PMC passes: per-launch counters, averaged over the timed and profiled regions
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("pmc_fetch", "pmc_write", "pmc_sq"):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        pl = bench_line(os.path.join(src, f"{p}.log"))
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(per)
        preg = regions(ids, pl["launches"])
        for d in ids:
            if preg[d] in ("timed", "profiled"):
                for n, v in per[d].items():
                    ctr[preg[d]][n].append(v)
    c = {}
    for region in ("timed", "profiled"):
        for n, v in ctr[region].items():
            c.setdefault(n, []).extend(v)
    mean = {n: sum(v) / len(v) for n, v in c.items()}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        out["fetch_kib_per_launch"] = mean["FETCH_SIZE"]
        out["write_kib_per_launch"] = mean["WRITE_SIZE"]
        out["hbm_bytes_per_launch"] = int((2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024)
    for n, key in (("SQ_INSTS_VALU", "sq_insts_valu_per_launch"), ("SQ_INSTS_SALU", "sq_insts_salu_per_launch"),
                   ("SQ_INSTS_VALU_FLOPS_FP64", "fp64_flops_per_launch"), ("SQ_INSTS_LDS", "sq_insts_lds_per_launch"),
                   ("SQ_INSTS_SMEM", "sq_insts_smem_per_launch"), ("SQ_WAVES", "sq_waves_per_launch"),
                   ("SQ_WAVE_CYCLES", "sq_wave_cycles_per_launch"), ("SQ_BUSY_CYCLES", "sq_busy_cycles_per_launch"),
                   ("GRBM_GUI_ACTIVE", "grbm_gui_active_per_launch")):
        if n in mean:
            out[key] = mean[n]
    # the bench's roofline recomputed from this file (what the judge checks)
    prof_ns = out["avg_ns_by_region"].get("profiled")
    if prof_ns:
        units = line["roofline"]["units_per_launch"]
        ach = units * line["roofline"]["bytes_per_unit"] / (prof_ns * 1e-9) / 1e9
        out["roofline_from_trace"] = {"achieved_gbs": round(ach, 1), "frac": round(ach / 8000.0, 4),
                                      "bench_frac": line["roofline"]["frac"],
                                      "note": "72 B x tests per launch (bench device counter) / mean kernel-trace "
                                              "duration of the profiled region's launches"}
    json.dump(out, open(os.path.join(dst, f"{tag}_roofline.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
