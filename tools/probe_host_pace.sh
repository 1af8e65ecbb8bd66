# N=8 root rehearsal: frame interval and host enqueue cost per mirt_trace_frame call
for cfg in "4 4 default" "8 4 default" "16 2 default" "4 4 away" "16 2 away"; do set -- $cfg
 MIRT_WG_FACTOR=$2 MIRT_GROUP_REHEARSE=8 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 400 --inflight $1 --view $3 || exit 1
done
