#!/bin/bash
# A/B of environment variants of the bench on one box:
#   tools/ab_env.sh "STEPS" "label:ENV=v ENV2=v|label2:..." [bench args]
# one JSON summary line per variant (ms_per_step, device ms, latency, launch ms, counters).
STEPS=$1; SPECS=$2; shift 2
IFS='|' read -ra VARS <<< "$SPECS"
for v in "${VARS[@]}"; do
  label=${v%%:*}; envs=${v#*:}
  LOG=/tmp/ab_$label.log
  env $envs timeout -k 10 150 python3 bench.py --steps "$STEPS" --warmup 5 --no-cpu-baseline --no-parity "$@" \
    > "$LOG" 2>&1 || { echo "$label failed"; tail -3 "$LOG"; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$LOG').read().splitlines() if l.startswith('{')][-1])
print(json.dumps({'v': '$label', 'F': d['frames_in_flight'], 'B': d['frames_per_launch'], 'ms': d['ms_per_step'],
                  'dev_ms': d['device_ms_per_frame'], 'lat_ms': d['frame_latency_ms'], 'launch_ms': d['roofline'].get('launch_ms', d['roofline'].get('algorithmic', {}).get('launch_ms')),
                  'tests': d['tri_tests_per_frame'], 'visits': d['bvh_visits_per_frame']}))"
done
