"""Per-kernel table from tools/exp_profile.sh output: python tools/pmc_table.py gpurun_out/<dir>"""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for p in ("pmc", "pmc2"):
    f = os.path.join(d, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if (p, r["Dispatch_Id"]) not in seen and p == "pmc":
            seen.add((p, r["Dispatch_Id"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k, c in rows.items():
    if "mirt" not in k:
        continue
    a = {n: sum(v) / len(v) for n, v in c.items()}
    t = sum(dur[k]) / max(len(dur[k]), 1)
    out = {"us": round(t * 1e6, 1)}
    wc = a.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if n in a:
                out[n.replace("SQ_", "").lower() + "_frac"] = round(a[n] / wc, 3)
    for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_WAVES"):
        if n in a:
            out[n] = int(a[n])
    if "GRBM_GUI_ACTIVE" in a and t:
        out["clock_ghz"] = round(a["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 2)
    if "SQ_INSTS_VALU" in a and t:
        out["valu_per_cu_cycle"] = round(a["SQ_INSTS_VALU"] / (256 * t * 2.3e9), 3)
    print(k, json.dumps(out))
