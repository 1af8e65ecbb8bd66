#!/bin/bash
# A/B of variants (GPU box), interleaved: the driver command (20 frames), 300 frames, and the N = 8
# rehearsal (root and a trace-only peer, 20 and 200 frames).  A variant is NAME:ENV=V[,ENV=V...]
# (MIRT_LIB=distributed_raytracer_amd/libmirt_x.so selects a library build).
#   bash tools/ab_variants.sh REPS "a:MIRT_LIB=... b:MIRT_NO_X=1" [sections: bench bench300 rehearse]
set -o pipefail
R=${1:-2}; VARIANTS=$2; SECTIONS=${3:-"bench bench300 rehearse"}
OUT=gpurun_out/ab_variants; mkdir -p $OUT; : > $OUT/ab.txt
line() {  # label logfile
  python3 -c "
import json; t=open('$2').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print('$1', d['ms_per_step'], d.get('device_ms_per_frame'), d.get('frame_latency_ms'), d['value'], (d.get('parity') or {}).get('bit_exact'))" >> $OUT/ab.txt
}
envs() { echo "${1#*:}" | tr ',' ' '; }
for rep in $(seq 1 $R); do
  for v in $VARIANTS; do
    n=${v%%:*}; E=$(envs "$v")
    if [[ " $SECTIONS " == *" bench "* ]]; then
      env $E timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_$n.log 2>&1 || { tail -5 $OUT/b_$n.log; exit 1; }
      line "bench20 $n" $OUT/b_$n.log
    fi
    if [[ " $SECTIONS " == *" bench300 "* ]]; then
      env $E timeout -k 10 200 python3 bench.py --gpus 1 --steps 300 --warmup 20 --no-cpu-baseline --no-parity > $OUT/b3_$n.log 2>&1 || { tail -5 $OUT/b3_$n.log; exit 1; }
      line "bench300 $n" $OUT/b3_$n.log
    fi
    if [[ " $SECTIONS " == *" rehearse "* ]]; then
      for fr in 20 200; do
        for rk in 0 3; do
          X=""; [ $rk = 3 ] && X="MIRT_GROUP_REHEARSE_RANK=3 MIRT_GROUP_REHEARSE_NO_UNPACK=1"
          r=$(env $E $X MIRT_GROUP_REHEARSE=8 timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr 2>/dev/null | tail -1) || exit 1
          echo "rehearse8 $n frames=$fr rank=$rk $(echo $r | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["frame_interval_us"], d["host_enqueue_us"])')" >> $OUT/ab.txt
        done
      done
    fi
  done
done
sort -s -k1,2 $OUT/ab.txt
