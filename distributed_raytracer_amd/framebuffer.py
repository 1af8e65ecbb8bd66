"""Image-space sharding of one frame over the GPUs of a box, and framebuffer assembly.

The reference parallelises a frame by recursively bisecting the screen into one
rectangle per worker (master/main.go:54-91) and gathering the per-rectangle results
over gRPC (master/main.go:130-176).  Here one process drives one GPU; the frame is cut
into fixed tiles dealt round-robin to the ranks (interleaved, so the object's pixels
spread evenly — bisection gives 4 of 8 GPUs no hit pixels on suzanne),
every rank traces its tiles into one packed buffer (each tile column-major, the
BulkTrace layout), and a single gather over RCCL (torch.distributed "nccl" backend =
RCCL on ROCm, over xGMI) brings the packed buffers to the root, which scatters them
into the W x H framebuffer with the k_unpack kernel.  The tile plan is a pure function
of (W, H, tile, world), so every rank computes it without communication.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

TileT = Tuple[int, int, int, int]


def plan_tiles(W: int, H: int, tile: int = 64) -> List[TileT]:
    """Raster-order tiles (x, y, w, h) covering W x H; edge tiles are clipped."""
    if W <= 0 or H <= 0 or tile <= 0:
        raise ValueError("W, H and tile must be positive")
    out = []
    for y in range(0, H, tile):
        for x in range(0, W, tile):
            out.append((x, y, min(tile, W - x), min(tile, H - y)))
    return out


def assign(tiles: Sequence[TileT], world: int, rank: int) -> List[TileT]:
    """Interleaved deal: tile k goes to rank k % world."""
    return list(tiles[rank::world])


def pixels_of(tiles: Sequence[TileT]) -> int:
    return int(sum(t[2] * t[3] for t in tiles))


def packed_capacity(tiles: Sequence[TileT], world: int) -> int:
    """Largest per-rank packed size: every rank pads its buffer to this for the gather."""
    return max(pixels_of(assign(tiles, world, r)) for r in range(world))


def master_partition(area: TileT, workers: int, dimension: int = 0, redundancy: int = 1,
                     width_kernel: int = 50, height_kernel: int = 50) -> Tuple[List[TileT], int]:
    """Restatement of the master's recursive bisection partition (master/main.go:54-91):
    returns (rectangles, leftover workers).  Kept for comparison with the interleaved
    plan (tests/test_framebuffer.py); the GPU path does not use it."""
    if workers // redundancy < 2:
        return [area], (workers % redundancy if workers > redundancy else 0)
    x, y, width, height = area
    if width <= width_kernel and height <= height_kernel:
        return [area], workers - redundancy
    elif width <= width_kernel:
        dimension = 1
    elif height <= height_kernel:
        dimension = 0
    if dimension % 2 == 0:
        left = (x, y, width // 2, height)
        right = (x + width // 2, y, width // 2 + width % 2, height)
    else:
        left = (x, y, width, height // 2)
        right = (x, y + height // 2, width, height // 2 + height % 2)
    lp, rem = master_partition(left, workers // 2 + workers % 2, (dimension + 1) % 2, redundancy,
                               width_kernel, height_kernel)
    rp, rem = master_partition(right, workers // 2 + rem, (dimension + 1) % 2, redundancy, width_kernel,
                               height_kernel)
    return lp + rp, rem


def unpack_host(W: int, H: int, tiles: Sequence[TileT], packed: np.ndarray, out: np.ndarray) -> None:
    """numpy twin of k_unpack: packed tile-major planes -> framebuffer (x*H + y).
    `packed`/`out` have the pixel axis first (any trailing channel shape)."""
    off = 0
    for (x, y, w, h) in tiles:
        blk = packed[off:off + w * h].reshape((w, h) + packed.shape[1:])
        fb = out.reshape((W, H) + out.shape[1:])
        fb[x:x + w, y:y + h] = blk
        off += w * h


def gather_packed(buf, world: int, rank: int, root: int = 0, group=None):
    """Gather every rank's packed buffer (same shape on all ranks) to `root`.  The one
    collective of the multi-GPU path: RCCL over xGMI for cuda tensors ("nccl"
    backend), gloo for CPU tensors (tests).  Returns the list on root, None elsewhere."""
    import torch
    import torch.distributed as dist
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device gather: stage through host memory (tests / 1-GPU rehearsals)
        cpu = buf.cpu()
        out = [torch.empty_like(cpu) for _ in range(world)] if rank == root else None
        dist.gather(cpu, out, dst=root, group=group)
        return [t.to(buf.device) for t in out] if out is not None else None
    out = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, out, dst=root, group=group)
    return out


@dataclass
class DevicePlanes:
    """Device tensors of one packed or full-frame output (torch, on the context's GPU)."""
    rgb8: object            # (n, 3) uint8
    valid: object           # (n,)   uint8
    rgb: Optional[object] = None   # (n, 3) float64
    face: Optional[object] = None  # (n,) int32
    raw: Optional[object] = None   # (4n,) uint8: the allocation rgb8 ++ valid live in

    def outputs(self, offset: int = 0) -> L.Outputs:
        def p(t, elem_bytes):
            return None if t is None else t.data_ptr() + offset * elem_bytes
        return L.Outputs(p(self.rgb, 24), p(self.rgb8, 3), p(self.valid, 1), p(self.face, 4), None)


def alloc_planes(n: int, device, with_rgb: bool = False, with_face: bool = False) -> DevicePlanes:
    import torch
    # rgb8 and valid share one allocation so a single gather moves both
    buf = torch.empty(n * 4, dtype=torch.uint8, device=device)
    return DevicePlanes(rgb8=buf[: n * 3].view(n, 3), valid=buf[n * 3:],
                        rgb=torch.empty((n, 3), dtype=torch.float64, device=device) if with_rgb else None,
                        face=torch.empty(n, dtype=torch.int32, device=device) if with_face else None, raw=buf)


def _tiles_c(tiles: Sequence[TileT]):
    arr = (L.Tile * len(tiles))()
    for i, t in enumerate(tiles):
        arr[i] = L.Tile(*t)
    return arr


def trace_tiles_device(ctx, frame_and_keep, W: int, H: int, tiles: Sequence[TileT], planes: DevicePlanes,
                       stream_ptr: Optional[int] = None, stats: bool = False) -> Optional[dict]:
    """Enqueue the trace of `tiles` into `planes` (packed) on `stream_ptr`."""
    fr, _keep = frame_and_keep
    out = planes.outputs()
    st = L.Stats() if stats else None
    L.check(L.lib().mirt_trace_tiles_async(ctx.handle, C.byref(fr), W, H, _tiles_c(tiles), len(tiles),
                                           C.byref(out), C.c_void_p(stream_ptr) if stream_ptr else None,
                                           C.byref(st) if st is not None else None))
    if st is not None:
        return {k: getattr(st, k) for k, _ in L.Stats._fields_}
    return None


def unpack_device(ctx, W: int, H: int, tiles: Sequence[TileT], packed: DevicePlanes, frame: DevicePlanes,
                  stream_ptr: Optional[int] = None) -> None:
    src = packed.outputs()
    dst = frame.outputs()
    L.check(L.lib().mirt_unpack_tiles_async(ctx.handle, W, H, _tiles_c(tiles), len(tiles), C.byref(src),
                                            C.byref(dst), C.c_void_p(stream_ptr) if stream_ptr else None))


class FrameSharder:
    """Per-rank driver: trace my tiles, gather the packed buffers to `root`, unpack there.

    With world == 1 the frame is traced as ONE tile straight into the framebuffer
    (the worker/sequential draw), with no gather and no unpack.

    With world > 1 frames are pipelined: frame k's gather (async on the collective's own
    stream) overlaps frame k+1's tracing, so each rank keeps two packed buffers; frame k
    is unpacked on the root once its gather is done, during render(k+1) or flush().
    All ranks' tiles are unpacked by ONE launch (mirt_unpack_tiles_at_async with the
    per-rank packed offsets).
    """

    def __init__(self, ctx, W: int, H: int, rank: int = 0, world: int = 1, tile: int = 64, root: int = 0,
                 with_rgb: bool = False, group=None):
        import torch
        self.ctx, self.W, self.H = ctx, W, H
        self.rank, self.world, self.root, self.group = rank, world, root, group
        self.device = torch.device("cuda", ctx.device)
        self.with_rgb = with_rgb
        if world == 1:
            self.tiles_all = [(0, 0, W, H)]
        else:
            self.tiles_all = plan_tiles(W, H, tile)
        self.mine = assign(self.tiles_all, world, rank)
        self.cap = packed_capacity(self.tiles_all, world)
        self._pending = None  # (works, gathered buffers) of the frame whose gather is in flight
        self._k = 0
        if world == 1:
            self.packed = None
            self.frame = alloc_planes(W * H, self.device, with_rgb)
        else:
            self.bufs = [alloc_planes(self.cap, self.device, with_rgb) for _ in range(2)]
            self.packed = self.bufs[0]
            self.frame = alloc_planes(W * H, self.device, with_rgb) if rank == root else None
            if rank == root:
                # every rank's tiles at its packed offset r * cap in the gathered buffer
                tl, off = [], []
                for r in range(world):
                    o = r * self.cap
                    for t in assign(self.tiles_all, world, r):
                        tl.append(t)
                        off.append(o)
                        o += t[2] * t[3]
                self._unpack_tiles = _tiles_c(tl)
                self._unpack_offsets = (C.c_uint64 * len(off))(*off)
                self._unpack_n = len(tl)
                self.gathered = [torch.empty(world * self.cap * 4, dtype=torch.uint8, device=self.device)
                                 for _ in range(2)]
                self.gathered_rgb = ([torch.empty((world * self.cap, 3), dtype=torch.float64, device=self.device)
                                      for _ in range(2)] if with_rgb else None)

    def _gather(self, k: int):
        """Issue the gather of packed buffer k % 2 to the root (async with RCCL)."""
        import torch.distributed as dist
        buf = self.bufs[k % 2]
        works = []
        pairs = [(buf.raw, self.gathered[k % 2] if self.rank == self.root else None)]
        if self.with_rgb:
            pairs.append((buf.rgb, self.gathered_rgb[k % 2] if self.rank == self.root else None))
        for src, dst in pairs:
            if src.is_cuda and dist.get_backend(self.group) == "gloo":
                got = gather_packed(src, self.world, self.rank, self.root, self.group)  # synchronous staging
                if dst is not None:
                    for r, g in enumerate(got):
                        dst.view(self.world, -1)[r].copy_(g.reshape(-1))
                continue
            outs = None
            if dst is not None:
                outs = [o.view(src.shape) for o in dst.view(self.world, -1).unbind(0)]
            works.append(dist.gather(src, outs, dst=self.root, group=self.group, async_op=True))
        return works

    def _unpack(self, k: int, stream_ptr: int) -> None:
        # rank r's gathered region is its packed raw buffer [rgb8 (3 cap) | valid (cap)]:
        # make each plane contiguous over the ranks (two strided copies), then one launch
        raw = self.gathered[k % 2].view(self.world, self.cap * 4)
        self._rgb8_all = raw[:, : self.cap * 3].reshape(self.world * self.cap, 3)
        self._valid_all = raw[:, self.cap * 3:].reshape(self.world * self.cap)
        src = DevicePlanes(rgb8=self._rgb8_all, valid=self._valid_all,
                           rgb=self.gathered_rgb[k % 2] if self.with_rgb else None)
        s_out, d_out = src.outputs(), self.frame.outputs()
        L.check(L.lib().mirt_unpack_tiles_at_async(self.ctx.handle, self.W, self.H, self._unpack_tiles,
                                                   self._unpack_offsets, self._unpack_n, C.byref(s_out),
                                                   C.byref(d_out), C.c_void_p(stream_ptr) if stream_ptr else None))

    def render(self, frame_and_keep) -> None:
        """Enqueue one frame on torch's current stream (no host sync)."""
        import torch
        s = torch.cuda.current_stream(self.device).cuda_stream
        if self.world == 1:
            trace_tiles_device(self.ctx, frame_and_keep, self.W, self.H, self.tiles_all, self.frame, s)
            return
        k = self._k
        self._k += 1
        trace_tiles_device(self.ctx, frame_and_keep, self.W, self.H, self.mine, self.bufs[k % 2], s)
        works = self._gather(k)
        self._finish_pending(s)
        self._pending = (k, works)

    def _finish_pending(self, s) -> None:
        if self._pending is None:
            return
        k, works = self._pending
        self._pending = None
        for w in works:
            w.wait()  # the current stream waits for the collective (no host block with RCCL)
        if self.rank == self.root:
            self._unpack(k, s)

    def flush(self) -> None:
        """Complete the frame whose gather is still in flight (unpack on the root)."""
        import torch
        if self.world > 1:
            self._finish_pending(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def last_packed(self):
        return self.bufs[(self._k - 1) % 2] if self.world > 1 else None
