# A/B two library builds on one box (GPU box): bash tools/ab_lib.sh libA.so libB.so [reps]
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out; : > gpurun_out/ab_lib.txt
for rep in $(seq 1 $R); do for L in $A $B; do
  MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 300 > gpurun_out/ab.log 2>&1 || exit 1
  python -c "
import json; t=open('gpurun_out/ab.log').read(); d=json.loads(t[t.index('{'):].splitlines()[0]); print($rep, '$L', 'bench', d['ms_per_step'], d['frame_latency_ms'])" >> gpurun_out/ab_lib.txt
  MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 100 python tools/inflight_probe.py --view away --world 1 --inflight 4 --maxwg 256 --repeat 1 | grep world | sed "s/^/$rep $L away /" >> gpurun_out/ab_lib.txt
done; done
cat gpurun_out/ab_lib.txt
