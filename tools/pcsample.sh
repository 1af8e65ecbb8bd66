#!/bin/bash
# PC sampling of the bench (rocprofv3 beta): instruction-level hotspots of k_trace.
#   tools/pcsample.sh OUTDIR [method] [bench args]
set -u
OUT=gpurun_out/$1; shift
M=${1:-stochastic}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 -L > "$OUT/list.txt" 2>&1 || true
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 --output-format csv -d "$OUT/pc" -o run -- python3 bench.py --no-cpu-baseline --no-parity --steps 200 "$@" \
  > "$OUT/pc.log" 2>&1
echo "rc=$?"
ls -R "$OUT" | head -20
