# launch shape around the defaults: frames in flight F, per launch B, workgroup factor WF
for cfg in "8 2 2" "8 2 4" "8 2 8" "12 3 4" "6 2 4" "16 4 2" "16 4 4" "16 4 8" "16 2 4"; do set -- $cfg
 MIRT_WG_FACTOR=$3 timeout -k 10 60 python tools/group_probe.py --tile 0 --frames 320 --inflight $1 --batch $2 | sed "s/^/WF=$3 /" || exit 1
 MIRT_WG_FACTOR=$3 MIRT_GROUP_REHEARSE=8 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 320 --inflight $1 --batch $2 | sed "s/^/WF=$3 /" || exit 1
done
