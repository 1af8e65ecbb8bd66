#!/bin/bash
# Profiles of the secondary bench lines (one rocprofv3 trace pass + separate PMC passes each,
# tools/profile_cmd.sh), then their plain bench lines:
#   brute   — the north star's literal loop (--brute-force), configs[1]
#   config3 — BASELINE configs[3]: 1M-triangle sphere at 3840x2160 (HBM-resident mesh)
#   config4 — BASELINE configs[4]: suzanne 3840x2160, 4 bounces (extension)
#   tools/profile_configs.sh TAG [brute] [config3] [config4]
set -u
TAG=${1:-r03}; shift
WHICH=${*:-"brute config3 config4"}
export TMPDIR=/tmp
for w in $WHICH; do
  case $w in
    brute) A="--gpus 1 --steps 20 --warmup 5 --brute-force --no-cpu-baseline --no-parity" ;;
    config3) [ -f /tmp/sphere1m/scene.json ] || timeout -k 10 300 python3 tools/gen_sphere_obj.py /tmp/sphere1m > /dev/null || exit 1
             A="--gpus 1 --steps 20 --warmup 5 --scene /tmp/sphere1m/scene.json --width 3840 --height 2160 --no-cpu-baseline --no-parity" ;;
    config4) A="--gpus 1 --steps 20 --warmup 5 --width 3840 --height 2160 --bounces 4 --no-cpu-baseline --no-parity" ;;
    *) echo "unknown $w"; exit 2 ;;
  esac
  tools/profile_cmd.sh "${TAG}${w}" $A || exit 1
done
echo done
