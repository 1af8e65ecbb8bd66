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
