# root per-frame interval at N = 2, 4, 8 (16 in flight, 4 per launch, 8-px strips, the
# group's weighted deal) and a non-root rank's (its share, no unpack) at N = 8: the
# one-GPU stand-in for the multi-GPU frame
for n in 2 4 8; do
  MIRT_GROUP_REHEARSE=$n timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 480 --inflight 16 --batch 4 || exit 1
done
MIRT_GROUP_REHEARSE=8 MIRT_GROUP_REHEARSE_RANK=1 MIRT_GROUP_REHEARSE_NO_UNPACK=1 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 480 --inflight 16 --batch 4 | sed 's/^/rank 1 of 8 /'
MIRT_GROUP_REHEARSE=8 MIRT_GROUP_REHEARSE_RANK=4 MIRT_GROUP_REHEARSE_NO_UNPACK=1 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 480 --inflight 16 --batch 4 | sed 's/^/rank 4 of 8 /'
timeout -k 10 60 python tools/group_probe.py --tile 0 --frames 480 --inflight 8 --batch 2 | sed 's/^/N=1 whole /'
