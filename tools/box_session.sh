#!/bin/bash
# Round 6: the box drop-in on the GPU box.  Its tests, then bench.py --box lines for boxes of 1
# and 8 entries (device 0 repeated: copy transport) serving the master's orders for 1 and 8
# workers, beside the frame group's driver line.   tools/box_session.sh OUTDIR
set -u
OUT=${1:-gpurun_out/box}; mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
[ -n "${NO_TESTS:-}" ] || run tests 600 python3 -u -m pytest tests/test_box.py tests/test_c_worker.py tests/test_group_emulated.py -m gpu -x -v \
  --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
SPECS=${BOX_SPECS:-1:1:8 1:1:16 8:1:8 1:8:8 8:8:8}
for spec in $SPECS; do
  IFS=: read -r e wk f <<< "$spec"
  run box_e${e}_w${wk}_f${f} 300 python3 bench.py --box $e --box-workers $wk --inflight $f --steps ${BOX_STEPS:-300} --warmup 20
done
run driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo "box session done"
