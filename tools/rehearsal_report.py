"""Summarise tools/profile_rehearsal.sh: per kernel, launches / mean duration; k_trace PMC per frame."""
import collections, csv, glob, json, os, sys
D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_rehearsal"
for mode in ("share", "whole"):
    rows = list(csv.DictReader(open(glob.glob(f"{D}/{mode}_trace/**/run_kernel_stats.csv", recursive=True)[0])))
    print(f"== {mode}: kernel stats")
    for r in rows:
        print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:8.2f} total_ms {float(r['TotalDurationNs'])/1e6:8.3f}")
    tr = list(csv.DictReader(open(glob.glob(f"{D}/{mode}_trace/**/run_kernel_trace.csv", recursive=True)[0])))
    kt = sorted([r for r in tr if "k_trace" in r["Kernel_Name"]], key=lambda r: int(r["Start_Timestamp"]))
    if kt:
        span = (int(kt[-1]["End_Timestamp"]) - int(kt[0]["Start_Timestamp"])) / 1e3
        print(f"  k_trace launches {len(kt)}, span {span:.1f} us")
    pm = glob.glob(f"{D}/{mode}_pmc/**/run_counter_collection.csv", recursive=True)
    if pm:
        agg = collections.defaultdict(float); n = collections.Counter()
        for r in csv.DictReader(open(pm[0])):
            if "k_trace" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        print("  k_trace PMC per launch:", {k: round(v / max(n[k], 1)) for k, v in agg.items()})
