#!/bin/bash
# Host phases of the N = 8 rehearsal (MIRT_HOST_TIMERS build, libmirt_ht.so): where a frame's
# host time goes, with the default view (GPU busy) and the camera turned away (GPU idle).
#   bash tools/host_probe_n8.sh
set -o pipefail
OUT=gpurun_out/host_n8; mkdir -p $OUT; : > $OUT/host.txt
for view in default away; do
  for rank in 0 3; do
    for fr in 20 200; do
      X=""; [ $rank = 3 ] && X="MIRT_GROUP_REHEARSE_RANK=3 MIRT_GROUP_REHEARSE_NO_UNPACK=1"
      echo "== view=$view rank=$rank frames=$fr" >> $OUT/host.txt
      env $X MIRT_NO_DEAL=1 MIRT_LIB=distributed_raytracer_amd/libmirt_ht.so MIRT_GROUP_REHEARSE=8 timeout -k 10 120 \
        python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr --view $view 2>&1 | grep -v amdgpu.ids >> $OUT/host.txt || exit 1
    done
  done
done
cat $OUT/host.txt
