#!/bin/bash
# N-rank rehearsal (root and peer of an N-way deal on one GPU, tools/group_probe.py) per variant,
# interleaved: a variant = "name|ENV=... ENV2=...|library" (library relative to the repo).
#   tools/rehearse_variants.sh OUT N "default||distributed_raytracer_amd/libmirt.so" ...
set -u
OUT=$1; N=$2; shift 2
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    IFS='|' read -r name envs lib <<< "$v"
    for fr in ${FRAMES:-20 200}; do
      for rank in 0 3; do
        r=$(env $envs MIRT_LIB=$lib MIRT_GROUP_REHEARSE=$N MIRT_GROUP_REHEARSE_RANK=$rank timeout -k 10 120 \
            python3 tools/group_probe.py --tile 8 --inflight 16 --batch 4 --frames $fr 2>/dev/null | grep '^{') || exit 1
        echo "$rep $name frames=$fr rank=$rank $r" >> "$OUT"
      done
    done
  done
done
cat "$OUT"
