#!/bin/bash
# N-rank rehearsal (root and a peer) over launch shapes: frames in flight F x frames per launch B
# (DESIGN.md §5.1).  usage: bash tools/shape_sweep_n8.sh "16x4 32x8" [N] [frames...]
SHAPES=${1:-"16x4 16x8 24x8 32x8"}
N=${2:-8}
FRAMES=${3:-"20 200"}
OUT=gpurun_out/shape_sweep_n$N.txt; : > $OUT
for s in $SHAPES; do F=${s%x*}; B=${s#*x}
  for fr in $FRAMES; do
    for rk in 0 3; do  # root (with the unpack of every region) and a peer (trace only)
      echo "== N=$N F=$F B=$B frames=$fr rank=$rk" >> $OUT
      NU=""; [ $rk != 0 ] && NU="MIRT_GROUP_REHEARSE_NO_UNPACK=1"
      env $NU MIRT_GROUP_REHEARSE=$N MIRT_GROUP_REHEARSE_RANK=$rk timeout -k 10 120 python3 tools/group_probe.py --tile 8 \
        --inflight $F --batch $B --frames $fr 2>&1 | grep -v amdgpu.ids >> $OUT || exit 1
    done
  done
done
cat $OUT
