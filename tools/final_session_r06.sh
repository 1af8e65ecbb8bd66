#!/bin/bash
# Round 6's final-build measurements (GPU box), in parts (each one gpurun call):
#   main     GPU suite, smoke, the driver command x3, 500 frames, the driver command's profile
#   motion   --camera orbit and --lights orbit lines and their profiles (static vs moving frames)
#   config3  configs[3] profiles (LDS streaming, the default, and --no-lds-stream), then their
#            lines (so they cite their own PMC), and the stream window's hit rate (DIAG build)
#   config4  configs[4] profile, then its line; the box lines; the N-rank rehearsal
# Every GPU step runs under its own timeout; the part stops at the first crash or timeout.
set -u
TAG=${TAG:-r06}
OUT=gpurun_out/final_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
sphere() { [ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1; }
C3="--gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json --width 3840 --height 2160 --no-cpu-baseline"
C4="--gpus 1 --steps 20 --warmup 5 --width 3840 --height 2160 --bounces 4 --no-cpu-baseline"
case ${1:-lines} in
  profiles)  # first call: every PMC profile (tools/roofline.py condenses them locally, then commit)
    sphere
    step profile 900 tools/profile_cmd.sh $TAG
    step profile_orbit 900 tools/profile_cmd.sh ${TAG}orbit --gpus 1 --steps 20 --warmup 5 --camera orbit --no-cpu-baseline
    step profile_lights 900 tools/profile_cmd.sh ${TAG}lights --gpus 1 --steps 20 --warmup 5 --lights orbit --no-cpu-baseline ;;
  profiles_configs)
    sphere
    step profile_config3 1200 tools/profile_cmd.sh ${TAG}config3 $C3 --no-parity
    step profile_config3ns 1200 tools/profile_cmd.sh ${TAG}config3ns $C3 --no-parity --no-lds-stream
    step profile_config4 1200 tools/profile_cmd.sh ${TAG}config4 $C4 --no-parity ;;
  lines)  # after the profiles are committed: the lines cite them (same build id)
    step tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
    step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
    for k in 1 2 3; do step driver_$k 300 python3 bench.py --gpus 1 --steps 20 --warmup 5; done
    step bench500 300 python3 bench.py --gpus 1 --no-cpu-baseline
    step orbit 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --camera orbit --no-cpu-baseline
    step lights 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --lights orbit --no-cpu-baseline
    step orbit500 300 python3 bench.py --gpus 1 --camera orbit --no-cpu-baseline ;;
  lines_configs)
    sphere
    step config3 600 python3 bench.py $C3
    step config3ns 600 python3 bench.py $C3 --no-lds-stream
    step config4 600 python3 bench.py $C4
    step stream_window 300 env MIRT_LIB=distributed_raytracer_amd/libmirt_diag.so python3 tools/stream_window.py /tmp/sphere1m/scene.json ;;
  box)
    for spec in 1:1:8:20 1:1:8:300 1:1:16:300 8:1:8:20 8:1:8:300 1:8:8:20 1:8:8:300; do
      IFS=: read -r e wk f st <<< "$spec"
      for rep in 1 2; do
        step box_e${e}_w${wk}_f${f}_s${st}_$rep 300 python3 bench.py --box $e --box-workers $wk --inflight $f --steps $st --warmup 20
      done
    done ;;
  rehearse)
    step rehearse 900 bash tools/rehearse_group.sh
    cp gpurun_out/rehearse.txt $OUT/rehearse.txt ;;
esac
echo "final $1 done"
