#!/bin/bash
# Bench + rocprofv3 kernel trace + two PMC passes (stall / instruction mix) for one build.
# usage (GPU box): bash tools/exp_profile.sh <outdir> [extra bench args]
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-parity $*"
timeout -k 10 200 $B --steps 30 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo "bench failed rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B --steps 10 --warmup 2 \
  > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$OUT/pmc" -o run -- $B --steps 3 --warmup 1 \
  > "$OUT/pmc.log" 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc2" -o run -- $B --steps 3 --warmup 1 > "$OUT/pmc2.log" 2>&1 || { echo "pmc2 failed rc=$?"; exit 1; }
echo "profile ok"
