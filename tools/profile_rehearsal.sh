#!/bin/bash
# Kernel trace + PMC of the N-rank rehearsal (root share of an N-way deal on one GPU) and of the
# whole frame at the same frame count, for per-frame work and occupancy comparisons.
#   bash tools/profile_rehearsal.sh [N] [frames] [F] [B]
N=${1:-8}; FR=${2:-200}; F=${3:-16}; B=${4:-4}
OUT=gpurun_out/prof_rehearsal; mkdir -p $OUT
export TMPDIR=/tmp
for mode in share whole; do
  if [ $mode = share ]; then E="MIRT_GROUP_REHEARSE=$N"; ARGS="--tile 8 --inflight $F --batch $B --frames $FR";
  else E="MIRT_GROUP_REHEARSE=1"; ARGS="--tile 0 --inflight 4 --batch 1 --frames $FR"; fi
  env $E timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${mode}_trace -o run -- python3 tools/group_probe.py $ARGS > $OUT/${mode}_trace.log 2>&1 || exit 1
  env $E timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/${mode}_pmc -o run -- python3 tools/group_probe.py $ARGS > $OUT/${mode}_pmc.log 2>&1 || exit 1
done
echo done
