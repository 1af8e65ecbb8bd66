"""Concurrency of k_trace launches in a rocprofv3 --kernel-trace CSV:
python tools/trace_overlap.py <kernel_trace.csv>  -> durations, mean concurrency, start gaps."""
import csv
import sys

import numpy as np


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_trace" in r["Kernel_Name"]]
    s = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
    e = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
    o = np.argsort(s)
    s, e = s[o][len(s) // 4:], e[o][len(s) // 4:]  # drop warm-up quarter
    d = (e - s) / 1e3
    span = (e.max() - s.min()) / 1e3
    ev = sorted([(t, 1) for t in s] + [(t, -1) for t in e])
    cur, hist, last = 0, {}, ev[0][0]
    for t, k in ev:
        hist[cur] = hist.get(cur, 0) + (t - last)
        cur += k
        last = t
    tot = sum(hist.values())
    print(f"launches {len(s)} span {span:.1f} us  interval {span / len(s):.2f} us  dur p10/50/90 "
          f"{np.percentile(d, 10):.1f}/{np.percentile(d, 50):.1f}/{np.percentile(d, 90):.1f} us")
    print("concurrency time share:", {k: round(v / tot, 3) for k, v in sorted(hist.items())})
    gaps = np.diff(s) / 1e3
    print(f"start gap p10/50/90 {np.percentile(gaps, 10):.1f}/{np.percentile(gaps, 50):.1f}/{np.percentile(gaps, 90):.1f} us")


if __name__ == "__main__":
    main()
