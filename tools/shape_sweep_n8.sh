#!/bin/bash
# N-rank rehearsal (root and a peer) over launch shapes: frames in flight F x frames per launch B
# [x workgroup factor W: a launch gets W x CUs / (F / B) workgroups, MIRT_WG_FACTOR, default 4]
# (DESIGN.md §5.1).  usage: bash tools/shape_sweep_n8.sh "16x4 32x8x2" [N] [frames...]
set -o pipefail
SHAPES=${1:-"16x4 16x8 24x8 32x8"}
N=${2:-8}
FRAMES=${3:-"20 200"}
OUT=gpurun_out/shape_sweep_n$N.txt; : > $OUT
for s in $SHAPES; do
  IFS=x read F B W <<< "$s"; W=${W:-4}
  for fr in $FRAMES; do
    for rk in 0 3; do  # root (with the unpack of every region) and a peer (trace only)
      NU=""; [ $rk != 0 ] && NU="MIRT_GROUP_REHEARSE_NO_UNPACK=1"
      r=$(env $NU MIRT_WG_FACTOR=$W MIRT_GROUP_REHEARSE=$N MIRT_GROUP_REHEARSE_RANK=$rk timeout -k 10 120 \
        python3 tools/group_probe.py --tile 8 --inflight $F --batch $B --frames $fr 2>/dev/null | tail -1) || exit 1
      echo "N=$N F=$F B=$B W=$W frames=$fr rank=$rk $(echo $r | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["frame_interval_us"], d["host_enqueue_us"])')" >> $OUT
    done
  done
done
cat $OUT
