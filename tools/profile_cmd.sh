#!/bin/bash
# Profile ONE bench command exactly as given (default: the driver's round-end command) on
# the GPU box: a rocprofv3 --kernel-trace --stats pass, then one --pmc pass per counter
# group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; --pmc is never combined
# with runtime/sys traces).  Output under gpurun_out/prof_$TAG; tools/roofline.py condenses
# it into profiles/${TAG}_roofline.json + profiles/${TAG}_kernel_stats.csv.
#   tools/profile_cmd.sh r02 [bench args...]
set -u
TAG=${1:-r02}
shift || true
ARGS=${*:-"--gpus 1 --steps 20 --warmup 5"}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py $ARGS \
    > "$OUT/$name.log" 2>&1 || { echo "$name pass failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "$name pass ok"
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_sq --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
# VALU busy cycles and lane utilisation (VALUBusy / VALUUtilization), the instruction mix
run pmc_valu --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 \
  SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32
run pmc_active --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_CVT \
  SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32
echo "args: $ARGS" > "$OUT/args.txt"
echo done
