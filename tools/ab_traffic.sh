#!/bin/bash
# HBM traffic per k_trace launch of the driver's command, per library build (two PMC passes:
# FETCH_SIZE and WRITE_SIZE cannot share one on gfx950; MI355X_MICROARCH.md's correction
# (2 FETCH_SIZE + WRITE_SIZE) x 1024).   tools/ab_traffic.sh libA.so libB.so ...
export TMPDIR=/tmp
OUT=gpurun_out/ab_traffic
mkdir -p $OUT
for L in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/$L.$C -o run -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity ${TRAFFIC_ARGS:-} > $OUT/$L.$C.log 2>&1 || { echo "$L $C failed"; exit 1; }
  done
  python3 - "$OUT" "$L" <<'PY'
import csv, sys
out, lib = sys.argv[1], sys.argv[2]
v = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per, frames = {}, set()
    for r in csv.DictReader(open(f"{out}/{lib}.{c}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if any(x in k for x in ("k_trace", "k_primary", "k_shadow", "k_bounce", "k_pack", "k_refl_fold")):
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            if "k_trace" in k or "k_primary" in k:
                frames.add(r["Dispatch_Id"])
    v[c] = sum(per.values()) / max(1, len(frames))  # per frame (one k_trace / k_primary each)
print(lib, "fetch KiB", round(v["FETCH_SIZE"]), "write KiB", round(v["WRITE_SIZE"]),
      "HBM MB", round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024 / 1e6, 2))
PY
done
