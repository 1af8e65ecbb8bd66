#!/bin/bash
# One gpurun session: GPU tests, the driver's bench command, a launch-shape sweep and the
# profile of the driver's command.  Stops at the first step that crashes, hangs or times
# out (rc other than 0 / 1); a step whose tests merely fail lets the session go on.
#   tools/gpu_session.sh OUTDIR [steps...]   steps: tests bench bench500 orbit orbit500 brute config3 config4
#                                             sweep profile profile_orbit smoke
set -u
OUT=${1:-gpurun_out/session}; shift
mkdir -p "$OUT"
STEPS=${*:-"tests bench sweep profile"}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    tests) step tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    bench) step bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench500) step bench500 300 python3 bench.py --gpus 1 --no-cpu-baseline ;;
    orbit) step orbit 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --camera orbit --no-cpu-baseline ;;
    orbit500) step orbit500 300 python3 bench.py --gpus 1 --camera orbit --no-cpu-baseline ;;
    brute) step brute 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --brute-force --no-cpu-baseline ;;
    config3) [ -f /tmp/sphere1m/scene.json ] || python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null
      step config3 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json \
      --width 3840 --height 2160 --no-cpu-baseline ;;
    config4) step config4 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --width 3840 --height 2160 --bounces 4 \
      --no-cpu-baseline ;;
    sweep) step sweep 900 tools/shape_sweep.sh 20 5 ;;
    profile) step profile 900 tools/profile_cmd.sh ${PROF_TAG:-r03} ;;
    profile_orbit) step profile_orbit 900 tools/profile_cmd.sh ${PROF_TAG:-r03}orbit --gpus 1 --steps 20 --warmup 5 \
      --camera orbit --no-cpu-baseline ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
