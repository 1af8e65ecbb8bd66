#!/bin/bash
# configs[3] A/B (GPU box): the HBM-mesh k_trace variants, one bench line each, interleaved.
#   bash tools/ab_config3.sh [reps]
#   hbm         the default: one-object HBM k_trace, leaves read with scalar loads (MIRT_HBM1)
#   stream      + primary rays' leaf triangles streamed through each wave's LDS window (--lds-stream)
#   stream_sh   libmirt_ss1.so (EXTRA=-DMIRT_STREAM_SHADOW=1) + --lds-stream: shadow sweeps stream too
set -o pipefail
R=${1:-2}
OUT=gpurun_out/ab3; mkdir -p $OUT; : > $OUT/ab.txt
[ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
A="--gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json --width 3840 --height 2160 --no-cpu-baseline"
for rep in $(seq 1 $R); do
  for v in hbm stream stream_sh; do
    case $v in
      hbm) L=libmirt.so; X="" ;;
      stream) L=libmirt.so; X="--lds-stream" ;;
      stream_sh) L=libmirt_ss1.so; X="--lds-stream" ;;
    esac
    MIRT_LIB=distributed_raytracer_amd/$L timeout -k 10 300 python3 bench.py $A $X > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    python3 -c "
import json; t=open('$OUT/$v.log').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print($rep, '$v', d['ms_per_step'], d.get('device_ms_per_frame'), d.get('frame_latency_ms'), d['value'], (d.get('parity') or {}).get('bit_exact'))" >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
