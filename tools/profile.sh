#!/bin/bash
# Profiling recipe (run on the GPU box through gpurun).  Kernel trace + stats in one
# pass, then one --pmc pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950; never combine --pmc with runtime/sys traces).  Output under
# gpurun_out/prof_$TAG; summaries are copied into profiles/ by tools/summarize_prof.py.
set -u
TAG=${1:-r01}
W=${W:-1920}; H=${H:-1080}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BENCH="bench.py --steps ${STEPS:-500} --warmup 20 --no-cpu-baseline --no-parity --width $W --height $H ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH \
  > "$OUT/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace pass ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH \
  > "$OUT/pmc_fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
echo "fetch pass ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH \
  > "$OUT/pmc_write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "write pass ok"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $BENCH > "$OUT/pmc_sq.log" 2>&1 || { echo "sq pass failed rc=$?"; exit 1; }
echo "sq pass ok"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
  SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU \
  --output-format csv -d "$OUT/pmc_f64" -o run -- python3 $BENCH > "$OUT/pmc_f64.log" 2>&1 || { echo "f64 pass failed rc=$?"; exit 1; }
echo "f64 pass ok"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
echo done
