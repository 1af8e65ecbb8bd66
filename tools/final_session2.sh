#!/bin/bash
# Last check of the round's final build: GPU suite, smoke, the driver command three times, the
# 500-frame and configs[3]/configs[4] lines, and the driver command's profile.  TAG = profile tag.
set -u
TAG=${1:-r04f}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
[ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
PROF_TAG=$TAG tools/gpu_session.sh $OUT tests smoke bench bench500 config3 config4 profile || exit 1
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/driver_$k.log 2>&1 || exit 1
done
echo final done
