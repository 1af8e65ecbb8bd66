#!/bin/bash
set -o pipefail
# Cost deal A/B (GPU box): driver command, lone frame, N = 8 / 2 rehearsal and the per-item
# timeline of a lone frame, with the deal on (default) and off (MIRT_NO_DEAL=1).
#   bash tools/ab_deal.sh [reps]
R=${1:-3}
OUT=gpurun_out/ab_deal; mkdir -p $OUT; : > $OUT/ab.txt
line() {  # label logfile
  python3 -c "
import json; t=open('$2').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print('$1', d['ms_per_step'], d.get('device_ms_per_frame'), d.get('frame_latency_ms'), d['value'], (d.get('parity') or {}).get('bit_exact'))" >> $OUT/ab.txt
}
for rep in $(seq 1 $R); do
  for v in on off; do
    E=""; [ $v = off ] && E="MIRT_NO_DEAL=1"
    env $E timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$v.log 2>&1 || { tail -5 $OUT/bench_$v.log; exit 1; }
    line "bench20 $v" $OUT/bench_$v.log
  done
done
for v in on off; do
  E=""; [ $v = off ] && E="MIRT_NO_DEAL=1"
  env $E timeout -k 10 200 python3 bench.py --gpus 1 --steps 300 --warmup 20 --no-cpu-baseline --no-parity > $OUT/bench300_$v.log 2>&1 || exit 1
  line "bench300 $v" $OUT/bench300_$v.log
  for n in 8 2; do
    for fr in 20 200; do
      env $E MIRT_GROUP_REHEARSE=$n timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr 2>/dev/null | sed "s/^/rehearse $v N=$n frames=$fr root /" >> $OUT/ab.txt || exit 1
      env $E MIRT_GROUP_REHEARSE=$n MIRT_GROUP_REHEARSE_RANK=3 MIRT_GROUP_REHEARSE_NO_UNPACK=1 timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr 2>/dev/null | sed "s/^/rehearse $v N=$n frames=$fr peer /" >> $OUT/ab.txt || exit 1
    done
  done
  env $E MIRT_LIB=distributed_raytracer_amd/libmirt_item.so timeout -k 10 120 python3 tools/item_trace.py > $OUT/item_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/item_$v.json')); print('item $v span', d['span_us'], 'wg_end', d['wg_end_us_p0_50_90_100'], 'wg_busy', d['wg_busy_wave_us_p0_50_90_100'])" >> $OUT/ab.txt
done
cat $OUT/ab.txt
