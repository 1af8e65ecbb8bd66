"""The bench line's contract (the task's bench.py rules) on the committed
bench lines of this round, and the consistency of the committed profile they cite.  CPU
only: reads profiles/, runs nothing on a GPU."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = ["profiles/r02_bench_driver_cmd.log", "profiles/r02_bench_default.log"]


def _line(path):
    line = None
    for ln in open(os.path.join(ROOT, path)):
        if ln.startswith("{"):
            line = json.loads(ln)
    assert line is not None, f"no JSON line in {path}"
    return line


@pytest.mark.parametrize("path", LINES)
def test_bench_line_contract(path):
    d = _line(path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["unit"] == "Mrays/s" and d["higher_is_better"] is True and d["dtype"] == "f64"
    assert d["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    assert "workload" in d["config"] and "model" not in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1
    # value is the device-resident rate: rays per frame / device ms per frame
    assert abs(d["value"] - d["rays_per_frame"] / d["device_ms_per_frame"] / 1e3) / d["value"] < 2e-3
    assert d["parity"]["bit_exact"] is True and d["parity"]["pixels_checked"] == 1920 * 1080


def test_driver_line_cites_the_committed_profile():
    """The driver-command line's physical roofs come from profiles/r02_roofline.json of the
    same launch shape, and the roofline recomputed from that file is within 5% of the line."""
    d = _line(LINES[0])
    prof = json.load(open(os.path.join(ROOT, "profiles", "r02_roofline.json")))
    assert d["steps"] == prof["shape"]["steps"] and d["warmup"] == prof["shape"]["warmup"]
    assert d["frames_in_flight"] == prof["shape"]["inflight"] and d["frames_per_launch"] == prof["shape"]["batch"]
    assert d["roofs"]["source"] == "profiles/r02_roofline.json"
    assert d["roofs"]["valu_insts_per_frame"] == int(prof["sq_insts_valu_per_launch"] / prof["frames_per_launch"])
    rt = prof["roofline_from_trace"]
    assert abs(rt["frac"] - rt["bench_frac"]) / rt["frac"] < 0.05
