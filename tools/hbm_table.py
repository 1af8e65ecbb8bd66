"""Per-kernel HBM bytes per frame from tools/hbm_probe.sh's two PMC passes (FETCH_SIZE, WRITE_SIZE),
with MI355X_MICROARCH.md's gfx950 correction (2 x FETCH_SIZE + WRITE_SIZE, KiB):
    python tools/hbm_table.py gpurun_out/hbm_TAG [frame-kernel-name-prefix [regions]]
regions (e.g. warmup=5,timed=20,device_only=20,profiled=20,latency=20, the bench line's `launches`):
also the prefix kernel's fetch and write per launch in each bench region, in dispatch order."""
import collections
import csv
import sys


def main():
    d = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_primary"
    tot = {}
    frames = 0
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        s = collections.defaultdict(float)
        n = collections.defaultdict(set)
        for r in csv.DictReader(open(f"{d}/{c}/run_counter_collection.csv")):
            k = r["Kernel_Name"].split("(")[0].replace("void mirt::", "").replace("mirt::", "")
            s[k] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
        frames = max(len(v) for k, v in n.items() if k.startswith(first))
        tot[c] = {k: v / frames / 1024 for k, v in s.items()}
    print(f"# {d}: MiB per frame over {frames} frames (every launch of the command, all regions)")
    F = W = 0.0
    for k in sorted(tot["FETCH_SIZE"]):
        if not k.startswith("k_"):
            continue
        f, w = tot["FETCH_SIZE"][k], tot["WRITE_SIZE"].get(k, 0.0)
        F += f
        W += w
        print(f"{k:40s} fetch {f:8.1f}  write {w:8.1f}")
    print(f"frame kernels: fetch {F:.1f} write {W:.1f} MiB; HBM (2 fetch + write) {2 * F + W:.1f} MiB = "
          f"{(2 * F + W) * 1048576 / 1e9:.3f} GB per frame")
    if len(sys.argv) > 3:
        regions = [(r.split("=")[0], int(r.split("=")[1])) for r in sys.argv[3].split(",")]
        per = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            by = collections.defaultdict(float)
            for r in csv.DictReader(open(f"{d}/{c}/run_counter_collection.csv")):
                k = r["Kernel_Name"].split("(")[0].replace("void mirt::", "").replace("mirt::", "")
                if k.startswith(first):
                    by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            vals = [by[i] for i in sorted(by)]
            out, k = [], 0
            for name, n in regions:
                v = vals[k:k + n]
                k += n
                out.append(sum(v) / max(len(v), 1) / 1024)
            per[c] = out
        for (name, _), f, w in zip(regions, per["FETCH_SIZE"], per["WRITE_SIZE"]):
            print(f"{first} {name:12s} fetch {f:6.1f} write {w:6.1f} MiB per launch; HBM {2 * f + w:6.1f} MiB")


if __name__ == "__main__":
    main()
