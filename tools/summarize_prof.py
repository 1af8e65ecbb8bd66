"""Condense a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>_*.

  python tools/summarize_prof.py r01 [--width 1920 --height 1080 --gpus 1]

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_summary.json       per kernel: avg duration, HBM bytes per launch from
                                    the PMC passes, VALU/LDS instruction counts, clock
  profiles/<tag>_pmc_traffic.json   k_primary HBM bytes per launch (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and
WRITE_SIZE are in KiB and come from separate passes; on gfx950 FETCH_SIZE reads half the
bytes of wide coalesced streaming reads, so the read side is doubled
(hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024, an upper bound for narrower accesses).
GRBM_GUI_ACTIVE is summed over the 8 XCDs: clock = GRBM_GUI_ACTIVE / 8 / duration.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    for k in ("k_primary", "k_shadow", "k_trace", "k_reflect", "k_rays", "k_unpack", "k_debug_fp64"):
        if k in name:
            return k + ("<nopre>" if "false>" in name and k != "k_shade" else "")
    return name.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--traffic-out", default="", help="merge the traffic keys into this json (default: <tag>_pmc_traffic.json)")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    kern = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        kern[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                  "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_f64"):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (p, r["Dispatch_Id"])
            if p == "pmc_sq" and key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    summary = {"tag": a.tag, "width": a.width, "height": a.height, "gpus": a.gpus, "kernels": {}}
    for k, d in kern.items():
        c = {n: sum(v) / len(v) for n, v in ctr.get(k, {}).items()}
        e = dict(d)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fetch_kib"] = c["FETCH_SIZE"]
            e["write_kib"] = c["WRITE_SIZE"]
            e["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                  "SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                  "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_SALU"):
            if n in c:
                e[n] = c[n]
        if "GRBM_GUI_ACTIVE" in c and dur.get(k):
            e["clock_ghz_est"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (sum(dur[k]) / len(dur[k])) / 1e9, 3)
        summary["kernels"][k] = e
    json.dump(summary, open(os.path.join(dst, f"{a.tag}_summary.json"), "w"), indent=1)
    tout = a.traffic_out or os.path.join(dst, f"{a.tag}_pmc_traffic.json")
    tj = json.load(open(tout)) if a.traffic_out and os.path.exists(tout) else {}
    tj.update({"width": a.width, "height": a.height, "gpus": a.gpus,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; (2*FETCH+WRITE)*1024"})
    tj.setdefault("tags", [])
    if a.tag not in tj["tags"]:
        tj["tags"].append(a.tag)
    for name in ("k_trace", "k_primary", "k_shadow"):
        kp = summary["kernels"].get(name, {})
        if "hbm_bytes_per_launch" in kp:
            tj[f"{name}_hbm_bytes_per_launch"] = kp["hbm_bytes_per_launch"]
            tj[f"{name}_avg_ns"] = kp["avg_ns"]
            tj[f"{name}_fp64_flops_per_launch"] = kp.get("SQ_INSTS_VALU_FLOPS_FP64")
            tj[f"{name}_valu_insts_per_launch"] = kp.get("SQ_INSTS_VALU")
    json.dump(tj, open(tout, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
