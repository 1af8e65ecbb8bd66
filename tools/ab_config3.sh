#!/bin/bash
# configs[3] A/B (GPU box): kernel variants of the HBM-mesh k_trace, one bench line each.
#   bash tools/ab_config3.sh [reps]
#   default        one-object HBM k_trace (MIRT_HBM1=1)
#   stream         + triangles streamed through each wave's LDS window (--lds-stream)
#   generic        libmirt_h0.so (EXTRA=-DMIRT_HBM1=0): the generic k_trace
#   stream_ns      libmirt_ss0.so + --lds-stream: shadow rays not streamed
R=${1:-2}
OUT=gpurun_out/ab3; mkdir -p $OUT; : > $OUT/ab.txt
[ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
A="--gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json --width 3840 --height 2160 --no-cpu-baseline --no-parity"
for rep in $(seq 1 $R); do
  for v in default stream generic stream_ns; do
    case $v in
      default) L=libmirt.so; X="" ;;
      stream) L=libmirt.so; X="--lds-stream" ;;
      generic) L=libmirt_h0.so; X="" ;;
      stream_ns) L=libmirt_ss0.so; X="--lds-stream" ;;
    esac
    MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 200 python3 bench.py $A $X > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    python3 -c "
import json; t=open('$OUT/$v.log').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print($rep, '$v', d['ms_per_step'], d.get('device_ms_per_frame'), d['value'])" >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
