mkdir -p gpurun_out; : > gpurun_out/ab.txt
run() { name=$1; shift; timeout -k 10 100 "$@" > gpurun_out/ab.log 2>&1 || exit 1; python -c "
import json; t=open('gpurun_out/ab.log').read(); d=json.loads(t[t.index('{'):].splitlines()[0]); print('$name', d['ms_per_step'], d['frame_latency_ms'], d['frames_in_flight'])" >> gpurun_out/ab.txt; }
run default python bench.py --no-cpu-baseline
run envq16 env GPU_MAX_HW_QUEUES=16 python bench.py --no-cpu-baseline
run steps300 python bench.py --no-cpu-baseline --steps 300
run noparity python bench.py --no-cpu-baseline --no-parity
run sweepcfg env GPU_MAX_HW_QUEUES=16 python bench.py --no-cpu-baseline --no-parity --steps 300 --inflight 8
run default2 python bench.py --no-cpu-baseline
cat gpurun_out/ab.txt
