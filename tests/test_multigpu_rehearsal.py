"""The N>1 bench path on whatever GPUs the box has: bench.py under torch.distributed.run
with 2 ranks (MIRT_DIST_BACKEND=gloo lets both ranks share one GPU; the gather stages
through host memory).  Exercises the tile deal, pipelined gathers, the one-launch unpack
with per-rank offsets and the timed-region flush; the bench's parity gate must report a
bit-exact frame.  (RCCL itself runs at round end on the 8-GPU node.)"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_rank_bench_path_is_bit_exact():
    env = dict(os.environ, MIRT_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--width", "320", "--height", "240", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["parity"]["bit_exact"] and d["hits_per_frame"] == 5820
