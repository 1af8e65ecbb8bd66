#!/bin/bash
# Instruction mix / cache counters per kernel (separate --pmc passes, no traces).
# usage (GPU box): bash tools/exp_counters.sh <outdir> [extra bench args]
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-parity --steps 3 --warmup 1 $*"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES" \
           "SQ_INSTS_VALU_TRANS_F SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_MUL_F SQ_INSTS_VALU_ADD_F SQ_INSTS_VALU_INT SQ_INSTS_VALU_CVT" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/c$i" -o run -- $B > "$OUT/c$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo "counters ok"
