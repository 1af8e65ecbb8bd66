#!/bin/bash
# Driver command (3 runs) + the N-rank rehearsal table, one box.
#   bash tools/measure_round.sh TAG
TAG=${1:-r05}
OUT=gpurun_out/measure_$TAG; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1
  python3 -c "
import json,sys; t=open('$OUT/bench_$i.log').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print('bench', $i, d['ms_per_step'], d['device_ms_per_frame'], d['frame_latency_ms'], d['value'], d['parity']['bit_exact'])"
done
timeout -k 10 400 bash tools/rehearse_group.sh > $OUT/rehearse.txt 2>&1 || exit 1
grep -o '"rehearse": "[0-9]*", "frame_interval_us": [0-9.]*' $OUT/rehearse.txt
