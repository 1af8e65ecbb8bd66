#!/bin/bash
# Round-end measurement session on one GPU box: the GPU suite, the bench lines of the README
# table, three driver-command runs, and the profiles of the driver, configs[3] and configs[4]
# commands (tools/profile_cmd.sh / profile_configs.sh).   tools/final_session.sh TAG
set -u
TAG=${1:-r04d}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
[ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
PROF_TAG=$TAG tools/gpu_session.sh $OUT tests bench bench500 orbit brute config3 config4 profile || exit 1
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/driver_$k.log 2>&1 || exit 1
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json --width 3840 --height 2160 \
  --lights orbit --no-cpu-baseline > $OUT/config3_lights_orbit.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --lights orbit --no-cpu-baseline > $OUT/lights_orbit.log 2>&1 || exit 1
tools/profile_configs.sh $TAG config4 config3 > $OUT/profile_configs.log 2>&1 || exit 1
echo final done
