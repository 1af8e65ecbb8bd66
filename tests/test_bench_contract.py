"""The bench line's contract (the task's bench.py rules) on the committed
bench lines of this round, and the consistency of the committed profiles they cite.  CPU
only: reads profiles/, runs nothing on a GPU."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# round 6, final build (profiles/r06i_*): every line ran after its command's profile was committed
TAG = "r06i"
DRIVER = f"profiles/{TAG}_bench_driver_1.log"   # python3 bench.py --gpus 1 --steps 20 --warmup 5
PROFILED = [DRIVER] + [f"profiles/{TAG}_bench_{k}.log" for k in ("driver_2", "driver_3", "orbit", "lights", "config3",
                                                                  "config3ns", "config4", "brute")]
UNPROFILED = [f"profiles/{TAG}_bench_{k}.log" for k in ("bench500", "orbit500")]  # 500 frames: no PMC of that shape
LINES = PROFILED + UNPROFILED


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
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["unit"] == "Mrays/s" and d["higher_is_better"] is True and d["dtype"] == "f64"
    assert d["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    assert "workload" in d["config"] and "model" not in d["config"]
    # value = rays per frame / ms per frame with the D2H
    assert abs(d["value"] - d["rays_per_frame"] / d["ms_per_step"] / 1e3) / d["value"] < 2e-3
    assert abs(d["device_mrays_s"] - d["rays_per_frame"] / d["device_ms_per_frame"] / 1e3) / d["value"] < 2e-3
    assert d["parity"]["bit_exact"] is True and d["parity"]["pixels_checked"] == d["config"]["width"] * d["config"]["height"]
    assert d["parity"]["rgb_f64"]["bit_exact"] is True  # the device fp64 colour plane too
    r = d["roofline"]
    if path in UNPROFILED:  # no PMC of this shape: the algorithmic figure, and it says so
        assert r["bound"] == "hbm" and r["traffic"] is None and "algorithmic roofline only" in r["note"]
        return
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "source", "algorithmic"):
        assert k in r, k
    # the physical roof: VALU-busy SIMD cycles per frame (committed PMC of this command's shape)
    assert r["bound"] == "valu" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert abs(r["achieved"] - r["valu_busy_cycles_per_frame"] / (d["ms_per_step"] * 1e-3) / 1e9) / r["achieved"] < 2e-3
    assert os.path.exists(os.path.join(ROOT, r["source"])) and isinstance(r["traffic"], int) and r["traffic"] > 0
    prof = json.load(open(os.path.join(ROOT, r["source"])))
    assert prof["build_id"] == d["build_id"]  # the profile of this very build
    a = r["algorithmic"]
    assert a["bound"] == "hbm" and a["unit"] == "GB/s" and a["bytes_per_unit"] == 72
    assert ("LDS-resident" in a["kind"]) == (d["config"]["triangles"] <= 1024)


def test_driver_line_cpu_baseline():
    c = _line(DRIVER)["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1


# configs[4] runs 17 kernels per frame: under the kernel trace its ms_per_step is ~20% longer than
# unprofiled, so its line is held to the contract and its shape only
PROFILED_LINES = [p for p in PROFILED if "config4" not in p]


@pytest.mark.parametrize("path", PROFILED_LINES)
def test_line_cites_the_committed_profile_of_its_shape(path):
    """Each line's roofline comes from the profile of its own launch shape, and the fraction
    recomputed from that file (over the profiling run's own ms_per_step) is within 8% of the
    line's: the two are separate runs of the command, and ms_per_step of one build spreads
    by up to ~6% from run to run (the orbit line: 0.0725 and 0.0813 ms in two runs)."""
    d = _line(path)
    r = d["roofline"]
    prof = json.load(open(os.path.join(ROOT, r["source"])))
    sh = prof["shape"]
    assert d["steps"] == sh["steps"] and d["warmup"] == sh["warmup"] and d["n_gpus"] == sh["gpus"]
    assert d["frames_in_flight"] == sh["inflight"] and d["frames_per_launch"] == sh["batch"]
    assert d["config"]["scene"] == sh["scene"] and d["config"]["camera"] == sh["camera"]
    assert d["config"]["bounces"] == sh["bounces"] and d["config"]["options"] == sh["options"]
    assert r["valu_busy_cycles_per_frame"] == int(prof["valu_busy_simd_cycles_per_launch"] / prof["frames_per_launch"])
    rt = prof["roofline_from_trace"]
    assert abs(rt["frac_over_trace_ms_per_step"] - r["frac"]) / r["frac"] < 0.08
    # over the timed region's kernel-trace span (no host tail, no last D2H): higher by ~10-15%
    assert abs(rt["frac_over_timed_kernel_span"] - r["frac"]) / r["frac"] < 0.25


def test_profiles_carry_per_region_kernel_summaries():
    """profiles/<tag>_kernel_regions.csv: every frame kernel's launches per bench region."""
    import csv
    d = _line(DRIVER)
    prof = json.load(open(os.path.join(ROOT, d["roofline"]["source"])))
    rows = list(csv.DictReader(open(os.path.join(ROOT, "profiles", prof["tag"] + "_kernel_regions.csv"))))
    regions = {r["region"]: int(r["launches"]) for r in rows if r["kernel"] == "k_trace"}
    assert regions == {k: v for k, v in d["launches"].items() if v}


@pytest.mark.parametrize("path", PROFILED_LINES)
def test_algorithmic_roofline_uses_the_timed_regions_launches(path):
    """roofline.algorithmic divides the bytes of one launch by the rocprofv3 average of the TIMED
    region's launches from the committed profile of the same build (the profiled region's HIP
    events bracket launches slowed by the profiling itself); the HIP-event median stays as a
    cross-check."""
    d = _line(path)
    a = d["roofline"]["algorithmic"]
    prof = json.load(open(os.path.join(ROOT, d["roofline"]["source"])))
    assert abs(a["launch_ms"] - prof["avg_ns_by_region"]["timed"] / 1e6) < 1e-4
    assert "timed region" in a["kind"] and a["hip_event_median_launch_ms"] > 0
    assert abs(a["achieved"] - a["units_per_launch"] * a["bytes_per_unit"] / (a["launch_ms"] * 1e-3) / 1e9) / a["achieved"] < 2e-3


def test_config_lines_carry_traffic_and_stream_window_counts():
    """configs[3] with and without LDS streaming and configs[4]: each line carries its HBM traffic
    and physical fraction from its own profile, and the stream window's hit rate is counted
    (a -DMIRT_DIAG build, tools/stream_window.py)."""
    t3 = _line(f"profiles/{TAG}_bench_config3.log")["roofline"]["traffic"]
    t3ns = _line(f"profiles/{TAG}_bench_config3ns.log")["roofline"]["traffic"]
    t4 = _line(f"profiles/{TAG}_bench_config4.log")["roofline"]["traffic"]
    assert all(isinstance(t, int) and t > 1e8 for t in (t3, t3ns, t4))
    sw = _line(f"profiles/{TAG}_stream_window.log")
    assert sw["window_leaves_served_per_frame"] > sw["window_reloads_per_frame"] > 0
    assert 0.0 < sw["window_hit_rate"] < 1.0 and sw["window_faces"] == 25


def test_box_lines():
    """The box drop-in's lines (bench.py --box): the contract's metric and unit, bit-exact."""
    for path in (f"profiles/{TAG}_bench_box1.log", f"profiles/{TAG}_bench_box8.log"):
        d = _line(path)
        assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
        assert d["unit"] == "Mrays/s" and d["parity"]["bit_exact"] is True
        assert abs(d["value"] - d["rays_per_frame"] / d["ms_per_step"] / 1e3) / d["value"] < 2e-3
        assert d["config"]["box_entries"] in (1, 8)


def test_in_tree_library_is_the_profiled_build():
    """The library in the tree (built by __graft_entry__.build() from these sources) has the build
    id of the committed profiles the driver's line cites: otherwise a round-end bench of this
    tree could only report the algorithmic figure."""
    import ctypes
    so = os.path.join(ROOT, "distributed_raytracer_amd", "libmirt.so")
    if not os.path.exists(so):
        pytest.skip("libmirt.so not built")
    lib = ctypes.CDLL(so)
    lib.mirt_build_id.restype = ctypes.c_char_p
    prof = json.load(open(os.path.join(ROOT, _line(DRIVER)["roofline"]["source"])))
    assert lib.mirt_build_id().decode() == prof["build_id"] == _line(DRIVER)["build_id"]
