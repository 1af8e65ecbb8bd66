#!/bin/bash
# A/B library builds on one bench command (GPU box), alternating, REPS times:
#   tools/ab_config.sh OUT "bench args" libA.so libB.so ...   (paths relative to the repo)
set -u
OUT=$1; ARGS=$2; shift 2
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in $(seq 1 ${REPS:-2}); do for L in "$@"; do
  MIRT_LIB=$L timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-parity > /tmp/ab.log 2>&1 || { tail -5 /tmp/ab.log; exit 1; }
  python3 -c "
import json; t=open('/tmp/ab.log').read(); d=json.loads(t[t.index('{'):].splitlines()[0])
print($rep, '$L', d['ms_per_step'], d['device_ms_per_frame'], d['frame_latency_ms'])" >> "$OUT"
done; done
cat "$OUT"
