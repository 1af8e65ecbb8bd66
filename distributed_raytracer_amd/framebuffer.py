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
import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

TileT = Tuple[int, int, int, int]


def plan_tiles(W: int, H: int, tile: int = 64, tile_h: Optional[int] = None) -> List[TileT]:
    """Raster-order tiles (x, y, w, h) covering W x H, tile wide and tile_h high (None: square;
    0: full-height column strips, contiguous in the column-major framebuffer); edge tiles
    are clipped."""
    th = tile if tile_h is None else (tile_h or H)
    if W <= 0 or H <= 0 or tile <= 0 or th <= 0:
        raise ValueError("W, H and tile must be positive")
    out = []
    for y in range(0, H, th):
        for x in range(0, W, tile):
            out.append((x, y, min(tile, W - x), min(th, H - y)))
    return out


def skew(world: int) -> int:
    """Row skew of the deal: the smallest s >= sqrt(world) coprime with world (8 -> 3)."""
    s = 1
    while s * s < world or math.gcd(s, world) != 1:
        s += 1
    return s


def assign(tiles: Sequence[TileT], world: int, rank: int) -> List[TileT]:
    """Interleaved deal of a raster tile list (plan_tiles): the tile in column c of tile
    row r goes to rank (c + skew * r) % world, so every rank's tiles are spread over rows
    AND columns (plain k % world puts a rank in the same few columns of every row when the
    row length is a multiple of world's factors).  On the suzanne 1080p hit mask with
    32-pixel tiles the busiest of 8 ranks holds 1.04x the mean hit count (k % world:
    1.07; the master's bisection: 1.37)."""
    if world <= 1:
        return list(tiles)
    cols = sum(1 for t in tiles if t[1] == tiles[0][1]) if tiles else 1
    s = skew(world)
    return [t for k, t in enumerate(tiles) if ((k % cols) + s * (k // cols)) % world == rank]


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


class PeerFailure(RuntimeError):
    """Ranks whose frame transfer did not reach the root before the deadline — the
    torch.distributed counterpart of mirt_group's MIRT_E_PEER (master/pool/pool.go:224-260:
    a worker that stops answering heartbeats is dropped)."""

    def __init__(self, ranks: Sequence[int], frame: int):
        self.ranks, self.frame = sorted(ranks), frame
        super().__init__(f"frame {frame}: no transfer from rank(s) {self.ranks} before the deadline")


def gather_with_deadline(pg, buf, me: int, n: int, deadline_s: float = 5.0, frame: int = 0, root: int = 0,
                         members: Optional[Sequence[int]] = None):
    """Gather `buf` from every rank of process group `pg` (a ProcessGroup used directly:
    ranks 0..n-1, this process is `me`) to `root` with point-to-point transfers — the shape
    of mirt_group's RCCL send/recv group — every receive bounded by one shared deadline.
    On the root: the list of n buffers, or PeerFailure naming each rank whose transfer
    missed the deadline or whose process is gone (`members` maps group ranks to the
    caller's rank numbers; the frame is skipped, as the master skips a frame,
    master/main.go:153-161).  Elsewhere: None, once the send completed or the deadline
    passed."""
    import datetime
    import time
    import torch
    if me != root:
        w = pg.send([buf], root, frame)
        try:  # bounded: a root that gave up on this frame never takes the transfer
            w.wait(datetime.timedelta(seconds=deadline_s))
        except RuntimeError:
            pass
        return None
    out = [torch.empty_like(buf) for _ in range(n)]
    out[root].copy_(buf)
    end = time.monotonic() + deadline_s
    failed, works = [], {}
    for q in range(n):
        if q == root:
            continue
        try:
            works[q] = pg.recv([out[q]], q, frame)
        except RuntimeError:  # the peer's process is gone (connection closed)
            failed.append(q)
    for q, w in works.items():
        left = max(1e-3, end - time.monotonic())
        try:
            ok = w.wait(datetime.timedelta(seconds=left))
        except RuntimeError:  # gloo reports a timed-out wait (or a lost peer) as an error
            ok = False
        if ok is False:
            failed.append(q)
    failed = [members[q] if members is not None else q for q in sorted(failed)]
    if failed:
        raise PeerFailure(failed, frame)
    return out


def frame_group_gloo(store, ranks: Sequence[int], rank: int, epoch: int, timeout_s: float = 30.0):
    """A gloo process group over `ranks` (sorted; this process is `rank`), built straight
    from the shared store: the first group of a frame loop, or after a failure the group of
    the survivors (mirt_group_exclude's counterpart: a new communicator from the store,
    never a collective that would wait for the dead rank).  Returns (group, index of this
    rank in it, group size)."""
    import datetime
    import torch.distributed as dist
    ranks = sorted(ranks)
    me = ranks.index(rank)
    pg = dist.ProcessGroupGloo(dist.PrefixStore(f"mirt_frames_{epoch}", store), me, len(ranks),
                               datetime.timedelta(seconds=timeout_s))
    return pg, me, len(ranks)


@dataclass
class DevicePlanes:
    """Device tensors of one packed or full-frame output (torch, on the context's GPU)."""
    rgb8: Optional[object] = None  # (n, 3) uint8
    valid: Optional[object] = None  # (n,)   uint8
    rgb: Optional[object] = None   # (n, 3) float64
    face: Optional[object] = None  # (n,) int32
    rgbv: Optional[object] = None  # (n,) int32: r | g << 8 | b << 16 | valid << 24 (packed tiles)

    def outputs(self, offset: int = 0) -> L.Outputs:
        if offset == 0 and getattr(self, "_out0", None) is not None:
            return self._out0  # per-frame calls reuse one struct (host time per frame matters)

        def p(t, elem_bytes):
            return None if t is None else t.data_ptr() + offset * elem_bytes
        o = L.Outputs(p(self.rgb, 24), p(self.rgb8, 3), p(self.valid, 1), p(self.face, 4), None, p(self.rgbv, 4))
        if offset == 0:
            self._out0 = o
        return o


def alloc_planes(n: int, device, with_rgb: bool = False, with_face: bool = False,
                 packed: bool = False) -> DevicePlanes:
    """Framebuffer planes rgb8 + valid, or (packed) ONE rgbv word per pixel — the form a
    rank's tiles travel in: one 32-bit store per pixel in the trace kernel and one
    contiguous plane for the gather."""
    import torch
    rgb = torch.empty((n, 3), dtype=torch.float64, device=device) if with_rgb else None
    face = torch.empty(n, dtype=torch.int32, device=device) if with_face else None
    if packed:
        return DevicePlanes(rgbv=torch.empty(n, dtype=torch.int32, device=device), rgb=rgb, face=face)
    return DevicePlanes(rgb8=torch.empty((n, 3), dtype=torch.uint8, device=device),
                        valid=torch.empty(n, dtype=torch.uint8, device=device), rgb=rgb, face=face)


def _tiles_c(tiles):
    """ctypes array of mirt_tile (an already built array is passed through: building one
    costs ~0.3 us per tile of host time, which matters for per-frame calls)."""
    if isinstance(tiles, C.Array):
        return tiles
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

    Frames in flight (`inflight` = F): frame k runs on stream k % F with its own buffers
    (framebuffer k % F; with world > 1, packed buffer and gathered buffer k % F), so the
    persistent trace kernel of frame k+1 starts while frame k's last workgroups finish —
    the frame tail is the largest inefficiency of a single frame — the
    way the reference master keeps several frames in flight (master/main.go:264-266).
    Frames are independent (each may have its own camera); results never change.

    With world > 1 every frame's gather is issued right after its trace (RCCL, async on
    the collective's own stream, which serialises the gathers in issue order on every
    rank), and frame k-1 is completed while frame k is enqueued: its stream waits for its
    gather and, on the root, ONE launch unpacks every rank's tiles (mirt_unpack_tiles_at_async
    with the per-rank packed offsets).  Buffer reuse is stream-ordered: frame k+F traces
    into packed buffer k % F only after stream k % F waited for frame k's gather.
    """

    def __init__(self, ctx, W: int, H: int, rank: int = 0, world: int = 1, tile: int = 64, root: int = 0,
                 with_rgb: bool = False, group=None, inflight: int = 1, tile_h: Optional[int] = None):
        import torch
        self.ctx, self.W, self.H = ctx, W, H
        self.rank, self.world, self.root, self.group = rank, world, root, group
        self.device = torch.device("cuda", ctx.device)
        self.with_rgb = with_rgb
        self.F = max(1, int(inflight))
        if self.F > 1:
            # frames in flight share the chip: at most 2 x CUs x 2 / F workgroups per frame
            # (measured: 4 in flight x 256 workgroups beats 4 x 512 by ~10 %, tools/inflight_probe.py)
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            ctx.set_grid(32, max(1, (4 * cus) // self.F) if self.F > 2 else 0)
        if world == 1:
            self.tiles_all = [(0, 0, W, H)]
        else:
            self.tiles_all = plan_tiles(W, H, tile, tile_h)
        self.mine = assign(self.tiles_all, world, rank)
        self._mine_c = _tiles_c(self.mine)
        self.cap = packed_capacity(self.tiles_all, world)
        self._pending = None  # (k, works) of the frame whose gather is in flight
        self._k = 0
        self._synced = set()  # frame streams that already waited for the current stream (this epoch)
        self._used = set()    # frame streams with frames since the last flush()
        # one stream per frame slot (F == 1: torch's current stream, as before)
        # (each on a hardware queue of its own: HIP shares at most GPU_MAX_HW_QUEUES queues
        # among ordinary streams, and frames whose streams share a queue serialise)
        self.streams = [ctx.stream_create() for _ in range(self.F)] if self.F > 1 else None
        nb = self.F if self.F > 1 else 2  # F == 1: two packed buffers (gather k overlaps trace k+1)
        if world == 1:
            self.packed = None
            self.frames = [alloc_planes(W * H, self.device, with_rgb) for _ in range(self.F)]
        else:
            self.bufs = [alloc_planes(self.cap, self.device, with_rgb, packed=True) for _ in range(nb)]
            self.packed = self.bufs[0]
            self.frames = ([alloc_planes(W * H, self.device, with_rgb) for _ in range(self.F)]
                           if rank == root else None)
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
                self.gathered = [torch.empty(world * self.cap, dtype=torch.int32, device=self.device)
                                 for _ in range(nb)]
                self.gathered_rgb = ([torch.empty((world * self.cap, 3), dtype=torch.float64, device=self.device)
                                      for _ in range(nb)] if with_rgb else None)
        self._nb = nb

    @property
    def frame(self) -> Optional[DevicePlanes]:
        """Framebuffer of the last rendered frame (root only when world > 1; complete
        after flush())."""
        if self.frames is None:
            return None
        return self.frames[(self._k - 1) % self.F] if self._k else self.frames[0]

    def _stream(self, k: int):
        import torch
        return self.streams[k % self.F] if self.streams else torch.cuda.current_stream(self.device)

    def _gather(self, k: int):
        """Issue the gather of packed buffer k to the root (async with RCCL; the current
        stream must be frame k's)."""
        import torch.distributed as dist
        j = k % self._nb
        buf = self.bufs[j]
        works = []
        pairs = [(buf.rgbv, self.gathered[j] if self.rank == self.root else None)]
        if self.with_rgb:
            pairs.append((buf.rgb, self.gathered_rgb[j] if self.rank == self.root else None))
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
        # the gathered rgbv plane is contiguous over the ranks (rank r's packed buffer at
        # pixel r * cap), so one launch expands every rank's tiles into rgb8 + valid
        j = k % self._nb
        s_out = DevicePlanes(rgbv=self.gathered[j], rgb=self.gathered_rgb[j] if self.with_rgb else None).outputs()
        d_out = self.frames[k % self.F].outputs()
        L.check(L.lib().mirt_unpack_tiles_at_async(self.ctx.handle, self.W, self.H, self._unpack_tiles,
                                                   self._unpack_offsets, self._unpack_n, C.byref(s_out),
                                                   C.byref(d_out), C.c_void_p(stream_ptr) if stream_ptr else None))

    def render(self, frame_and_keep) -> None:
        """Enqueue one frame (no host sync).  F == 1: on torch's current stream; F > 1:
        on the sharder's stream k % F (a frame stream's first frame after construction or
        flush() waits for the work already queued on the current stream)."""
        import torch
        k = self._k
        self._k += 1
        sk = self._stream(k)
        if self.streams and (k % self.F) not in self._synced:
            sk.wait_stream(torch.cuda.current_stream(self.device))
            self._synced.add(k % self.F)
            self._used.add(k % self.F)
        if self.world == 1:
            trace_tiles_device(self.ctx, frame_and_keep, self.W, self.H, self._mine_c, self.frames[k % self.F],
                               sk.cuda_stream)
            return
        with torch.cuda.stream(sk):
            trace_tiles_device(self.ctx, frame_and_keep, self.W, self.H, self._mine_c, self.bufs[k % self._nb],
                               sk.cuda_stream)
            works = self._gather(k)
        self._finish_pending()
        self._pending = (k, works)

    def _finish_pending(self) -> None:
        import torch
        if self._pending is None:
            return
        k, works = self._pending
        self._pending = None
        sk = self._stream(k)
        with torch.cuda.stream(sk):
            for w in works:
                w.wait()  # frame k's stream waits for its collective (no host block with RCCL)
            if self.rank == self.root:
                self._unpack(k, sk.cuda_stream)

    def flush(self) -> None:
        """Complete every frame in flight: the current stream waits for all of them (and,
        with world > 1, for the last gather and unpack)."""
        import torch
        if self.world > 1:
            self._finish_pending()
        if self.streams:
            cur = torch.cuda.current_stream(self.device)
            for j in sorted(self._used):
                cur.wait_stream(self.streams[j])
        self._synced.clear()
        self._used.clear()

    @property
    def last_packed(self):
        return self.bufs[(self._k - 1) % self._nb] if self.world > 1 else None


def plan_group_tiles(W: int, H: int, tile: int, world: int, rank: int, tile_h: Optional[int] = None) -> List[TileT]:
    """The deal mirt_group uses (mirt_group_plan_tiles): rank 0, which also unpacks every
    frame, is weighted down (N = 8: 3 of every 31 deal slots, the others 4)."""
    th = tile if tile_h is None else tile_h
    n = L.lib().mirt_group_plan_tiles(W, H, tile, th, world, rank, None, 0)
    L.check(min(n, 0))
    arr = (L.Tile * max(n, 1))()
    L.check(min(L.lib().mirt_group_plan_tiles(W, H, tile, th, world, rank, C.cast(arr, C.c_void_p), n), 0))
    return [(t.x, t.y, t.w, t.h) for t in arr[:n]]


def plan_rank_tiles_native(W: int, H: int, tile: int, world: int, rank: int, tile_h: Optional[int] = None) -> List[TileT]:
    """The C++ tile deal of mirt_group (mirt_plan_tiles); equals assign(plan_tiles(...))."""
    th = tile if tile_h is None else tile_h
    n = L.lib().mirt_plan_tiles(W, H, tile, th, world, rank, None, 0)
    L.check(min(n, 0))
    arr = (L.Tile * max(n, 1))()
    L.check(min(L.lib().mirt_plan_tiles(W, H, tile, th, world, rank, C.cast(arr, C.c_void_p), n), 0))
    return [(t.x, t.y, t.w, t.h) for t in arr[:n]]


class NativeFrameGroup:
    """The multi-GPU frame in native code (mirt.h mirt_group_* / mirt_trace_frame): the
    same tile deal, rgbv packing, RCCL gather and unpack as FrameSharder, but one C call per
    frame — the RCCL send/recv group runs on the library's own stream, so no Python
    collective, stream switch or event is on the per-frame path.  torch.distributed is only
    the bootstrap: rank 0's RCCL unique id is broadcast over the caller's process group.

    world == 1: the whole screen as one tile straight into the framebuffer (tile=None), or
    the tiled path rehearsed on one GPU (tile > 0: packed rgbv + unpack, no RCCL).
    Frames in flight: frame k on the library's stream k % F, framebuffer frames[k % F]
    (rank 0 only), every stream on a hardware queue of its own."""

    def __init__(self, ctx, W: int, H: int, rank: int = 0, world: int = 1, tile: Optional[int] = 8,
                 inflight: int = 4, group=None, with_rgb: bool = False, tile_h: Optional[int] = 0,
                 batch: int = 1, emulate: int = 0, host_output: bool = False, timeout_ms: int = 0,
                 library_planes: bool = False):
        import torch
        self.ctx, self.W, self.H, self.rank, self.world = ctx, W, H, rank, world
        self.F = max(1, int(inflight))
        self.B = max(1, min(int(batch), self.F, 8))  # frames per k_trace launch
        self.device = torch.device("cuda", ctx.device)
        tile = (tile or 0) if world == 1 else int(tile or 8)
        th = tile if tile_h is None else int(tile_h)  # 0: full-height strips
        self.tiles_all = [(0, 0, W, H)] if tile == 0 else plan_tiles(W, H, tile, th)
        self.mine = [(0, 0, W, H)] if tile == 0 else plan_group_tiles(W, H, tile, world, rank, th)
        if self.F > 1:
            # frames in flight share the chip: at most wg_factor * CUs / F workgroups per frame
            # (2 per CU can be resident; factor 4 = twice what fits)
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            wg_factor = float(os.environ.get("MIRT_WG_FACTOR", "4"))
            launches = max(1, self.F // self.B)  # launches in flight
            fc = os.environ.get("MIRT_FUSED_COPY", "")
            if world == 1 and not tile and launches % 2 == 0 and fc != "0" and (fc == "1" or launches >= 8):
                launches //= 2  # F / B / 2 streams, fused host copies (mirt.cpp update_fused_copy)
            ctx.set_grid(int(os.environ.get("MIRT_MIN_BLOCKS", "32")), max(1, int(wg_factor * cus / launches)))
        uid = (C.c_uint8 * 128)()
        if world > 1:
            import torch.distributed as dist
            t = torch.zeros(128, dtype=torch.uint8, device=self.device if dist.get_backend(group) == "nccl" else "cpu")
            if rank == 0:
                L.check(L.lib().mirt_group_unique_id(C.cast(uid, C.c_void_p)))
                t.copy_(torch.frombuffer(bytearray(bytes(uid)), dtype=torch.uint8))
            dist.broadcast(t, src=0, group=group)
            uid = (C.c_uint8 * 128)(*t.cpu().tolist())
        # library_planes: fbs == NULL, the group owns its rgb8 + valid planes (callers that read
        # frames only through host_frame, like the C / Go workers)
        self.frames = ([alloc_planes(W * H, self.device, with_rgb) for _ in range(self.F)]
                       if rank == 0 and not library_planes else None)
        fbs = (L.Outputs * self.F)(*[p.outputs() for p in self.frames]) if self.frames else None
        self._h = C.c_void_p()
        L.check(L.lib().mirt_group_create(ctx.handle, C.cast(uid, C.c_void_p) if world > 1 else None, rank, world,
                                          W, H, tile, th if tile else 0, self.F, C.cast(fbs, C.c_void_p) if fbs else None,
                                          C.byref(self._h)))
        if self.B > 1:
            L.check(L.lib().mirt_group_set_batch(self._h, self.B))
        if emulate and emulate > 1:
            # one GPU traces every rank's share of an `emulate`-way deal and runs the whole
            # pack -> transfer -> trailer check -> unpack chain (mirt_group_emulate)
            L.check(L.lib().mirt_group_emulate(self._h, int(emulate)))
        self.emulated = int(emulate or 0)
        if host_output:
            L.check(L.lib().mirt_group_set_host_output(self._h, 1))
        if timeout_ms:
            L.check(L.lib().mirt_group_set_timeout(self._h, int(timeout_ms)))
        self._k = 0
        self._idx = C.c_uint64()

    def render(self, frame_and_keep) -> int:
        """Enqueue the next frame (no host sync, no Python collective); returns its index."""
        fr, _keep = frame_and_keep
        L.check(L.lib().mirt_trace_frame(self._h, C.byref(fr), C.byref(self._idx)))
        self._k += 1
        return int(self._idx.value)

    def wait(self) -> None:
        """Host wait for every enqueued frame (deadline-bounded with timeout_ms); raises
        MirtError MIRT_E_PEER / MIRT_E_TIMEOUT naming the failed frame and ranks."""
        L.check(L.lib().mirt_group_wait(self._h, None))

    def host_frame(self, index: int, copy: bool = True):
        """(rgb8 (W*H, 3), valid (W*H,)) numpy copies of frame `index` from the group's
        pinned host planes (host_output=True): the frame after its D2H.  copy=False: views
        of the pinned planes, valid while host output stays off or the slot is not reused."""
        out = L.Outputs()
        L.check(L.lib().mirt_group_frame_host(self._h, int(index), C.byref(out)))
        n = self.W * self.H
        rgb8 = np.ctypeslib.as_array(C.cast(out.rgb8, C.POINTER(C.c_uint8)), shape=(n * 3,)).reshape(n, 3)
        valid = np.ctypeslib.as_array(C.cast(out.valid, C.POINTER(C.c_uint8)), shape=(n,))
        return (rgb8.copy(), valid.copy()) if copy else (rgb8, valid)

    def set_host_output(self, enable: bool) -> None:
        """Copy frames enqueued from now on to pinned host memory (or stop)."""
        L.check(L.lib().mirt_group_set_host_output(self._h, 1 if enable else 0))

    def failed_ranks(self) -> List[int]:
        m = C.c_uint64()
        L.lib().mirt_group_failed_ranks(self._h, C.byref(m))
        return [r for r in range(64) if (m.value >> r) & 1]

    def drop(self, ranks: Sequence[int]) -> None:
        """Fault injection (emulated world): these ranks' transfers stop arriving."""
        L.check(L.lib().mirt_group_emulate_drop(self._h, sum(1 << r for r in ranks)))

    def exclude(self, alive: Sequence[int], new_unique_id: Optional[bytes] = None) -> None:
        """Re-deal over the ranks in `alive` (rank 0 included) after a failure."""
        uid = (C.c_uint8 * 128)(*new_unique_id) if new_unique_id else None
        L.check(L.lib().mirt_group_exclude(self._h, sum(1 << r for r in alive),
                                           C.cast(uid, C.c_void_p) if uid is not None else None))

    def flush(self) -> None:
        """torch's current stream waits for every enqueued frame (gathers and unpacks included)."""
        import torch
        L.check(L.lib().mirt_group_wait(self._h, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))

    @property
    def frame(self) -> Optional[DevicePlanes]:
        if self.frames is None:
            return None
        return self.frames[(self._k - 1) % self.F] if self._k else self.frames[0]

    def close(self) -> None:
        if self._h:
            L.lib().mirt_group_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
