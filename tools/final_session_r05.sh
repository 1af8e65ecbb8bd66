#!/bin/bash
# Round 5's final-build measurements (GPU box), two calls:
#   bash tools/final_session_r05.sh main     GPU suite, smoke, the driver command (+3 repeats), 500 frames,
#                                            configs[3], configs[4], the driver command's profile
#   bash tools/final_session_r05.sh extra    the N-rank rehearsal table, configs[3]/[4] profiles
set -u
TAG=${TAG:-r05f}
OUT=gpurun_out/final_$TAG; mkdir -p $OUT
case ${1:-main} in
  main)
    [ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
    PROF_TAG=$TAG tools/gpu_session.sh $OUT tests smoke bench bench500 config3 config4 profile || exit 1
    for k in 1 2 3; do
      timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/driver_$k.log 2>&1 || exit 1
    done ;;
  extra)
    timeout -k 10 500 bash tools/rehearse_group.sh > $OUT/rehearse.log 2>&1 || exit 1
    cp gpurun_out/rehearse.txt $OUT/rehearse.txt
    timeout -k 10 600 tools/profile_configs.sh $TAG config3 config4 > $OUT/profile_configs.log 2>&1 || exit 1 ;;
esac
echo "final $1 done"
