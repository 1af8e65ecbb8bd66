"""The ABI from a caller that is neither Go nor Python: worker_c/mirt_worker (plain C, built by
__graft_entry__.build()) runs the drop-in worker's call sequence — scene -> mirt_create ->
mirt_mesh_upload -> concurrent BulkTrace orders of the master's partition through
mirt_trace_tile -> the master's assembly, then a frame group with library-owned
framebuffers and host output — in a fresh process with no torch and no HIP calls of its own
(the HIP runtime comes through libmirt's RUNPATH).  Its assembled frame must equal the
golden frames bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, SCENE

BIN = os.path.join(ROOT, "worker_c", "mirt_worker")


def _run(W, H, out, workers=4, box=0):
    pre = ["--box", str(box)] if box else []
    return subprocess.run([BIN] + pre + [SCENE, str(W), str(H), str(out), str(workers)], capture_output=True, text=True,
                          timeout=120, env={k: v for k, v in os.environ.items() if not k.startswith("PYTHON")})


def test_c_worker_is_built_and_fails_loudly_without_a_gpu(tmp_path):
    import torch
    assert os.path.exists(BIN), "worker_c/mirt_worker is not built (run __graft_entry__.build())"
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = _run(64, 48, tmp_path / "o.bin")
    assert r.returncode == 2 and "mirt_create" in r.stderr  # MIRT_E_DEVICE, no silent fallback


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,golden,workers", [(64, 48, "suzanne_64x48.npz", 4), (320, 240, "suzanne_320x240.npz", 7)])
def test_c_worker_frames_match_golden(tmp_path, W, H, golden, workers):
    out = tmp_path / "fb.bin"
    r = _run(W, H, out, workers)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group frames equal: yes" in r.stdout
    raw = np.fromfile(out, np.uint8)
    rgb8 = raw[:W * H * 3].reshape(W * H, 3)
    valid = raw[W * H * 3:]
    g = np.load(os.path.join(GOLDEN, golden))
    if "valid" in g:
        assert np.array_equal(valid, g["valid"]) and np.array_equal(rgb8, g["rgb8"])
    else:  # 320x240: hit pixels only
        hit = np.nonzero(valid)[0]
        assert np.array_equal(hit, g["hit_index"].astype(np.int64))
        assert np.array_equal(rgb8[hit], g["rgb8"]) and not rgb8[valid == 0].any()


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,workers,box", [(320, 240, 7, 8), (1920, 1080, 8, 8), (160, 120, 3, 3)])
def test_c_worker_box_serves_the_master_partition(tmp_path, W, H, workers, box):
    """--box N: ONE C worker driving N device entries (mirt_box_*; on a one-GPU box every entry
    is device 0) serves the master's partition (master/main.go:54-91) concurrently; its frame
    equals the one-context frame, and at 320x240 the golden frame."""
    out = tmp_path / "fb.bin"
    r = _run(W, H, out, workers, box)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"box of {box} entries" in r.stdout and "orders equal: yes" in r.stdout
    if (W, H) == (320, 240):
        raw = np.fromfile(out, np.uint8)
        g = np.load(os.path.join(GOLDEN, "suzanne_320x240.npz"))
        rgb8 = raw[:W * H * 3].reshape(W * H, 3)
        assert np.array_equal(rgb8[g["hit_index"].astype(np.int64)], g["rgb8"])


def _run_gob(name, W, H, out, workers=4):
    gob = os.path.join(GOLDEN, "gob")
    return subprocess.run([BIN, "--gob", os.path.join(gob, f"{name}_state.gob"), os.path.join(gob, f"{name}_diff.gob"),
                           str(W), str(H), str(out), str(workers)], capture_output=True, text=True, timeout=120,
                          env={k: v for k, v in os.environ.items() if not k.startswith("PYTHON")})


def test_c_worker_decodes_the_wire_before_the_device(tmp_path):
    """--gob: MasterState.state and a WorkOrder.diff decoded in C (no Go, no Python); without
    a GPU the run gets past the decoding and fails at mirt_create."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = _run_gob("multi", 64, 48, tmp_path / "o.bin")
    assert r.returncode == 2 and "mirt_create" in r.stderr and "gob" not in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H", [("example", 320, 240), ("multi", 160, 120)])
def test_c_worker_from_the_wire_matches_oracle(tmp_path, name, W, H):
    from oracle.oracle import Oracle
    from test_gob import scenes, wire_scene
    out = tmp_path / "fb.bin"
    r = _run_gob(name, W, H, out, 5)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(out, np.uint8)
    ref = Oracle(wire_scene(scenes()[name][0])).frame(W, H)
    assert np.array_equal(raw[W * H * 3:], ref["valid"])
    assert np.array_equal(raw[:W * H * 3].reshape(W * H, 3), ref["rgb8"])
