#!/bin/bash
# The N-rank root rehearsal with the root's D2H of every frame (the bench's host output), against
# the same without it and the whole frame at N = 1.  bash tools/rehearse_d2h.sh
set -o pipefail
OUT=gpurun_out/rehearse_d2h.txt; : > $OUT
for fr in 20 200; do
  for n in 1 8 4; do
    for ho in "" "--host-output"; do
      if [ $n = 1 ]; then A="--tile 0 --inflight 4 --batch 1"; E=""; else A="--tile 8 --inflight 16 --batch 4"; E="MIRT_GROUP_REHEARSE=$n"; fi
      r=$(env $E timeout -k 10 120 python3 tools/group_probe.py $A --frames $fr $ho 2>/dev/null | tail -1) || exit 1
      echo "N=$n frames=$fr host_output=${ho:+1} $(echo $r | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["frame_interval_us"], d["host_enqueue_us"])')" >> $OUT
    done
  done
done
cat $OUT
