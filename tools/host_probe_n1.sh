set -o pipefail
for ho in "" "--host-output"; do for fr in 20 200; do
 echo "== host_output=$ho frames=$fr"
 MIRT_LIB=distributed_raytracer_amd/libmirt_ht.so timeout -k 10 120 python3 tools/group_probe.py --tile 0 --inflight 4 --batch 1 --frames $fr $ho 2>&1 | grep -v amdgpu.ids || exit 1
done; done
