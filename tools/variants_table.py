"""Table of tools/variants.sh results: per variant, the bench's device frame interval and
lone-frame latency, and per k_trace launch (one frame, one launch in flight) the PMC counts.
  python tools/variants_table.py gpurun_out/<dir> base nophong ..."""
import collections
import csv
import glob
import json
import os
import sys


def main(d, names):
    cols = None
    for n in names:
        line = None
        for ln in open(os.path.join(d, f"{n}.bench.log")):
            if ln.startswith("{"):
                line = json.loads(ln)
        row = {"variant": n, "dev_ms": line["device_ms_per_frame"], "lat_ms": line["frame_latency_ms"],
               "tests": line["tri_tests_per_frame"]}
        for f in sorted(glob.glob(os.path.join(d, f"{n}.c*", "run_counter_collection.csv"))):
            per = collections.defaultdict(dict)
            for r in csv.DictReader(open(f)):
                if "k_trace" in r["Kernel_Name"]:
                    per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            ids = sorted(per)[1:]  # drop the warmup launch
            for k in per[ids[0]]:
                row[k] = sum(per[i][k] for i in ids) / len(ids)
        if cols is None:
            cols = list(row)
            print(" | ".join(c.replace("SQ_", "") for c in cols))
        print(" | ".join(f"{row.get(c, 0):.4g}" if not isinstance(row.get(c), str) else row[c] for c in cols))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
