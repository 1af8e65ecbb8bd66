# root per-frame interval at N = 2, 4, 8 (16 in flight, 4 per launch, 8-px strips) and a
# non-root rank's (no unpack) at N = 8: the one-GPU stand-in for the multi-GPU frame
for n in 2 4 8; do
  MIRT_GROUP_REHEARSE=$n timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 480 --inflight 16 --batch 4 || exit 1
done
MIRT_GROUP_REHEARSE=8 MIRT_GROUP_REHEARSE_NO_UNPACK=1 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 480 --inflight 16 --batch 4 | sed 's/^/non-root /'
timeout -k 10 60 python tools/group_probe.py --tile 0 --frames 480 --inflight 8 --batch 2 | sed 's/^/N=1 whole /'
