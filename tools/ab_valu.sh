#!/bin/bash
# VALU / SALU instructions per k_trace launch (one PMC pass of the driver's command per
# library build; every launch traces the same static frame) and the bench line of each.
#   tools/ab_valu.sh libA.so libB.so@--bench-flag ...   (libs under distributed_raytracer_amd/;
#   text after @: extra bench arguments of that variant)
export TMPDIR=/tmp
OUT=gpurun_out/ab_valu
mkdir -p $OUT
for V in "$@"; do
  L=${V%%@*}; X=""; [[ "$V" == *@* ]] && X=${V#*@}
  N=$L${X// /}
  MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
    SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/$N -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-parity $X > $OUT/$N.log 2>&1 || { echo "$N failed"; tail -5 $OUT/$N.log; exit 1; }
  python3 - "$OUT/$N" "$N" <<'PY'
import csv, collections, json, sys
d, name = sys.argv[1], sys.argv[2]
per = collections.defaultdict(dict)
for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
    if "k_trace" in r["Kernel_Name"]:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
m = {k: sum(v[k] for v in per.values()) / len(per) for k in next(iter(per.values()))}
t = open(d + "/../" + name + ".log").read()
b = json.loads(t[t.index("{"):].splitlines()[0])
print(name, "launches", len(per), {k: round(v / 1e6, 3) for k, v in m.items()},
      "util", round(m["SQ_THREAD_CYCLES_VALU"] / (m["SQ_ACTIVE_INST_VALU"] * 64), 3),
      "ms", b["ms_per_step"], "dev", b["device_ms_per_frame"], "lat", b["frame_latency_ms"])
PY
done
