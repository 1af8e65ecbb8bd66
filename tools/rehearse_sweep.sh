for F in 2 4 8; do for WF in 2 4 8; do for MB in 8 32; do
 MIRT_WG_FACTOR=$WF MIRT_MIN_BLOCKS=$MB MIRT_GROUP_REHEARSE=8 timeout -k 10 60 python tools/group_probe.py --tile 8 --frames 300 --inflight $F | sed "s/^/F=$F WF=$WF MB=$MB /" || exit 1
done; done; done
