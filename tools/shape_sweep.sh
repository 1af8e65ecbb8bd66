#!/bin/bash
# Launch-shape sweep of the bench (frames in flight F x frames per launch B) at a given
# run length; one JSON summary line per shape on stdout:  tools/shape_sweep.sh 20 5 [bench args]
STEPS=${1:-20}; WARM=${2:-5}; shift 2 || true
for fb in ${SHAPES:-2,1 2,2 4,1 4,2 4,4 8,2 8,4 8,8 16,4 16,8}; do
  F=${fb%,*}; B=${fb#*,}
  LOG=/tmp/sweep_${F}_${B}.log
  timeout -k 10 120 python3 bench.py --steps "$STEPS" --warmup "$WARM" --inflight "$F" --batch "$B" \
    --no-cpu-baseline --no-parity "$@" > "$LOG" 2>&1 || { echo "F=$F B=$B failed"; tail -3 "$LOG"; exit 1; }
  python3 -c "
import json, sys
d = json.loads([l for l in open('$LOG').read().splitlines() if l.startswith('{')][-1])
print(json.dumps({'F': $F, 'B': $B, 'steps': $STEPS, 'ms_per_step': d['ms_per_step'],
                  'device_ms': d['device_ms_per_frame'], 'latency_ms': d['frame_latency_ms'],
                  'launch_ms': d['roofline'].get('launch_ms', d['roofline'].get('algorithmic', {}).get('launch_ms'))}))"
done
