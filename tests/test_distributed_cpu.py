"""The N>1 path on CPU: world_size-2 gloo.  Each rank traces ITS interleaved tiles
(with the oracle standing in for the GPU kernels — test infrastructure), pads to the
common capacity, gathers with the same gather_packed() the RCCL path uses, and rank 0
assembles the framebuffer with unpack_host (the numpy twin of k_unpack).  The
assembled frame must equal the single-process frame bit-for-bit."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, SCENE


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, tile, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from distributed_raytracer_amd.framebuffer import (assign, gather_packed, packed_capacity, pixels_of,
                                                       plan_tiles, unpack_host)
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tiles = plan_tiles(W, H, tile)
    mine = assign(tiles, world, rank)
    cap = packed_capacity(tiles, world)
    r = Oracle(load_scene(SCENE)).trace_tiles(W, H, mine)
    n = pixels_of(mine)
    rgb = torch.zeros((cap, 3), dtype=torch.float64)
    rgb[:n] = torch.from_numpy(r["rgb"])
    valid = torch.zeros(cap, dtype=torch.uint8)
    valid[:n] = torch.from_numpy(r["valid"])
    got_rgb = gather_packed(rgb, world, rank)
    got_valid = gather_packed(valid, world, rank)
    if rank == 0:
        fb_rgb = np.zeros((W * H, 3))
        fb_valid = np.zeros(W * H, np.uint8)
        for q in range(world):
            tq = assign(tiles, world, q)
            unpack_host(W, H, tq, got_rgb[q].numpy(), fb_rgb)
            unpack_host(W, H, tq, got_valid[q].numpy(), fb_valid)
        np.savez(out_path, rgb=fb_rgb, valid=fb_valid)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 16), (3, 24)])
def test_gloo_tiled_frame_equals_single_frame(tmp_path, oracle, world, tile):
    import torch.multiprocessing as mp
    W, H = 96, 72
    out = str(tmp_path / "fb.npz")
    mp.spawn(_worker, args=(world, _free_port(), W, H, tile, out), nprocs=world, join=True)
    got = np.load(out)
    ref = oracle.frame(W, H)
    assert np.array_equal(got["valid"], ref["valid"])
    assert np.array_equal(got["rgb"], ref["rgb"])


def _fault_worker(rank, world, port, W, H, tile, out_path, mode):
    """Frames 0 and 1 on `world` ranks; at frame 1 the last rank stops answering (never
    sends).  The root must name it within the deadline and skip the frame; the survivors
    regroup from the store, re-deal the tiles among themselves, and frames 2 and 3 must be
    exact.  The oracle stands in for the GPU kernels (test infrastructure)."""
    import sys
    import time
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from distributed_raytracer_amd.framebuffer import (PeerFailure, assign, frame_group_gloo, gather_with_deadline,
                                                       packed_capacity, pixels_of, plan_tiles, unpack_host)
    from oracle.oracle import Oracle
    from oracle.scene_py import load_scene
    store = dist.TCPStore("127.0.0.1", port, world, rank == 0, timeout=__import__("datetime").timedelta(seconds=60))
    orc = Oracle(load_scene(SCENE))
    tiles = plan_tiles(W, H, tile)
    dead = world - 1
    alive = list(range(world))
    epoch = 0
    pg, me, n = frame_group_gloo(store, alive, rank, epoch)
    log = []
    for frame in range(4):
        if rank == dead and frame >= 1:
            if mode == "silent":  # alive but silent: no transfer, no part in the regrouping
                store.wait(["mirt_test_done"], __import__("datetime").timedelta(seconds=120))
            return  # "exit": the process is gone
        mine = assign(tiles, n, me)
        cap = packed_capacity(tiles, n)
        r = orc.trace_tiles(W, H, mine)
        buf = torch.zeros(cap, dtype=torch.uint8)
        buf[:pixels_of(mine)] = torch.from_numpy(r["valid"])
        t0 = time.monotonic()
        try:
            got = gather_with_deadline(pg, buf, me, n, deadline_s=3.0, frame=frame, members=alive)
        except PeerFailure as e:  # the root names the rank; every survivor learns it from the store
            log.append(("failed", frame, e.ranks, round(time.monotonic() - t0, 1)))
            store.set(f"failed_{frame}", ",".join(map(str, e.ranks)))
            got = None
        if frame == 1:  # frame 1's outcome decides the next group (the root wrote it)
            failed = [int(x) for x in store.get(f"failed_{frame}").decode().split(",") if x]
            alive = [q for q in alive if q not in failed]
            epoch += 1
            pg, me, n = frame_group_gloo(store, alive, rank, epoch)
            log.append(("regrouped", frame, alive))
        if rank == 0 and got is not None:
            fb = np.zeros(W * H, np.uint8)
            for q in range(n):
                unpack_host(W, H, assign(tiles, n, q), got[q].numpy(), fb)
            np.save(out_path + f".{frame}.npy", fb)
            log.append(("frame", frame, n))
    if rank == 0:
        import json
        json.dump(log, open(out_path + ".log.json", "w"))
        store.set("mirt_test_done", "1")


@pytest.mark.parametrize("mode", ["silent", "exit"])
def test_gloo_rank_stops_answering_is_named_and_redealt(tmp_path, oracle, mode):
    """f4 fault handling on the N>1 path (master/pool/pool.go:224-260,
    master/main.go:153-161): 3 gloo ranks, rank 2 stops answering at frame 1 — alive but
    silent (the deadline names it) or gone (its closed connection names it)."""
    import json
    import torch.multiprocessing as mp
    W, H = 64, 48
    out = str(tmp_path / "fb")
    mp.spawn(_fault_worker, args=(3, _free_port(), W, H, 16, out, mode), nprocs=3, join=True)
    log = json.load(open(out + ".log.json"))
    assert ["frame", 0, 3] in log
    fails = [e for e in log if e[0] == "failed"]
    assert len(fails) == 1 and fails[0][1] == 1 and fails[0][2] == [2] and fails[0][3] <= 10
    assert ["regrouped", 1, [0, 1]] in log
    assert ["frame", 2, 2] in log and ["frame", 3, 2] in log
    ref = oracle.frame(W, H)["valid"]
    for f in (0, 2, 3):
        assert np.array_equal(np.load(out + f".{f}.npy"), ref), f"frame {f}"
