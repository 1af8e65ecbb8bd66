#!/bin/bash
# N-rank rehearsal (root and a peer) over launch shapes at the driver's 20 frames:
#   tools/rehearse_shapes.sh N    (MIRT_GROUP_REHEARSE=N)
N=${1:-8}
for fb in ${SHAPES:-16,4 16,8 8,8 8,4 12,4 16,2}; do
  F=${fb%,*}; B=${fb#*,}
  for r in 0 3; do
    MIRT_GROUP_REHEARSE=$N MIRT_GROUP_REHEARSE_RANK=$r timeout -k 10 120 python3 tools/group_probe.py --tile 8 \
      --inflight $F --batch $B --frames 20 2>/dev/null | tail -1 | sed "s/^/N=$N rank=$r F=$F B=$B /" || exit 1
  done
done
