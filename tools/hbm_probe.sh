#!/bin/bash
# HBM probe: FETCH_SIZE and WRITE_SIZE passes of one bench command (GPU box)
set -u
TAG=$1; shift; OUT=gpurun_out/hbm_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 bench.py "$@" > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -3 $OUT/$c.log; exit 1; }
  echo "$c ok"
done
