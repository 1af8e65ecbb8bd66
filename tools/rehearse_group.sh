#!/bin/bash
# Root and peer rehearsal of the N-rank group on one GPU: MIRT_GROUP_REHEARSE=N
# traces rank 0's (or MIRT_GROUP_REHEARSE_RANK's) share of an N-way deal with the bench's N>1 shape.
OUT=gpurun_out/rehearse.txt; : > $OUT
run() { echo "== $*" >> $OUT; env "$@" >> $OUT 2>&1 || exit 1; }
for n in 8 4 2; do
  for fr in 20 200; do
    run MIRT_GROUP_REHEARSE=$n timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr
    run MIRT_GROUP_REHEARSE=$n MIRT_GROUP_REHEARSE_RANK=3 timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr
    # a peer's own work: its trace into the transfer form, no unpack (only the root unpacks)
    run MIRT_GROUP_REHEARSE=$n MIRT_GROUP_REHEARSE_RANK=3 MIRT_GROUP_REHEARSE_NO_UNPACK=1 timeout -k 10 120 python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr
  done
done
cat $OUT | grep -v amdgpu.ids
