"""Per-kernel averages of every counter collected by tools/exp_counters.sh."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "c*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if "mirt" in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    print(k)
    for n in sorted(c):
        print(f"  {n:28s} {sum(c[n]) / len(c[n]):16.0f}")
