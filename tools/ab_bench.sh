#!/bin/bash
# A/B of library builds (MIRT_LIB) on one box, interleaved: R rounds of each library, one
# bench line each; prints device ms/frame, ms/frame with the D2H and the lone-frame latency.
#   tools/ab_bench.sh "BENCH ARGS" R libA.so libB.so ...   (libs under distributed_raytracer_amd/)
ARGS=$1; R=$2; shift 2
OUT=gpurun_out/ab_bench.txt
mkdir -p gpurun_out; : > $OUT
for rep in $(seq 1 $R); do for L in "$@"; do
  MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-parity \
    > gpurun_out/ab_one.log 2>&1 || { echo "$L failed"; tail -5 gpurun_out/ab_one.log; exit 1; }
  python3 -c "
import json; t=open('gpurun_out/ab_one.log').read(); d=json.loads(t[t.index('{'):].splitlines()[0])
print($rep, '$L', 'dev', d['device_ms_per_frame'], 'ms', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'k', d['ms_kernels'])" >> $OUT
  tail -1 $OUT
done; done
