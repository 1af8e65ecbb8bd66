# bench.py over frames in flight x hardware queues (GPU box): bash tools/bench_sweep.sh
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for rep in 1 2; do
for q in ${QS:-8 16}; do for f in ${FS:-4 6 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 100 python bench.py --no-cpu-baseline --no-parity --steps 300 --inflight $f > gpurun_out/sw.log 2>&1 || exit 1
  python -c "
import json; t=open('gpurun_out/sw.log').read(); d=json.loads(t[t.index('{'):].splitlines()[0]); print($rep, 'q$q', 'F$f', d['ms_per_step'], d['frame_latency_ms'])" >> gpurun_out/sweep.txt
done; done; done
cat gpurun_out/sweep.txt
