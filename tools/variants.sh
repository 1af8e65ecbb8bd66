#!/bin/bash
# Attribute k_trace's time and instructions to its phases with diagnostic builds.
# CPU side (this container):  tools/variants.sh build name:"-DFLAG=1 ..." ...
# GPU box:                    tools/variants.sh run OUTDIR name ...
# Each variant is libmirt_<name>.so (MIRT_LIB); "base" is libmirt.so.  The GPU side runs,
# per variant, the bench (device frame interval, lone-frame latency) and two --pmc passes
# of a short bench (instruction mix and wait cycles per k_trace launch);
# tools/variants_table.py condenses them.
set -u
mode=$1; shift
CSRC=distributed_raytracer_amd/csrc
if [ "$mode" = build ]; then
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    make -s -j8 -C $CSRC OUT=../libmirt_$name.so OBJ=obj_$name EXTRA="$flags" || exit 1
    echo "built libmirt_$name.so ($flags)"
  done
  exit 0
fi
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for name in "$@"; do
  lib=distributed_raytracer_amd/libmirt_$name.so
  [ "$name" = base ] && lib=distributed_raytracer_amd/libmirt.so
  B="python3 bench.py --no-cpu-baseline --no-parity"
  MIRT_LIB=$lib timeout -k 10 120 $B --steps 200 > "$OUT/$name.bench.log" 2>&1 || { echo "$name bench failed"; tail -3 "$OUT/$name.bench.log"; exit 1; }
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    MIRT_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/$name.c$i" -o run -- $B --steps 4 --warmup 1 --inflight 1 \
      > "$OUT/$name.c$i.log" 2>&1 || { echo "$name pmc $i failed rc=$?"; tail -3 "$OUT/$name.c$i.log"; exit 1; }
  done
  echo "$name ok"
done
echo variants done
