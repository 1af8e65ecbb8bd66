# frames per launch x frames in flight: N=1 whole screen and the N=8 root rehearsal (8-px strips)
for cfg in ${CFGS:-"4 1" "8 2" "12 4" "16 4" "16 8" "12 2"}; do set -- $cfg
 timeout -k 10 60 python tools/group_probe.py --tile 0 --frames 320 --inflight $1 --batch $2 || exit 1
 MIRT_GROUP_REHEARSE=8 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 320 --inflight $1 --batch $2 || exit 1
done
