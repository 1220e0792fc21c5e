"""Frame sharding over GPUs + framebuffer exchange, one process per GPU.

The reference splits a frame over host threads by interleaved rows (HW2/main.cpp:33-36,
HW2/Scene.cpp:25).  Two splits live here.  The default of bench.py (BandPlan,
BandGatherRenderer, further down): each camera's frame cut into one band of whole 8-pixel tile
rows per rank at cuts balanced by the frame's measured tile costs (rt_tile_costs), rendered in
place and sent to rank 0 straight into its frame rows — as 32-bit pixel records that rank 0
shades (rt_resolve_rows), or as RGB.  The tile deal (TileLayout, TileGatherRenderer): the deal
units of every camera's frame — 2x2 blocks of 8x8-pixel tiles
(one wavefront per tile, one traversal workgroup per block), block rows rotated by their row
index (RT_TILE_BLOCKS, include/ceng795_rt.h) — are numbered globally, camera after camera, and
dealt round-robin over ranks: rank r renders global units g = r (mod world), diagonal stripes
of blocks, which balances cost the way the row interleave does while each workgroup's rays
stay neighbours.  There is no other exchange: the scene is replicated, rays are independent.

Buffer layout.  Each rank's HBM buffer holds one fixed-size SLOT per camera
(4 ceil(blocks / world) tiles, the largest share any rank gets), and the rank's tiles of that
camera are written back to back (tile-major, 4 per block) at the slot's start.  Every rank's slot c has the
same size, so camera c's shares are gathered to rank 0 by one equal-size collective
(torch.distributed "nccl" = RCCL over xGMI).  Rank 0 then untiles camera c with ONE
index_select of 8-pixel tile rows (96 B, contiguous in both layouts) straight into the
row-major framebuffer.

TileGatherRenderer pipelines consecutive steps (frames) over `inflight` buffer sets and render
streams, the way the one-GPU bench keeps frames in flight: step k renders into set k mod F
while the gathers of earlier steps run on the communication stream.

TileLayout and the untile index are pure bookkeeping (numpy / torch CPU), and the renderers
take the tile renderer as a callable, so the N>1 logic is testable with the gloo backend on
CPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

TILE = 8
TILE_FLOATS = TILE * TILE * 3
TILE_RECORDS = TILE * TILE  # 32-bit pixel records per tile (RT_TILE_RECORDS shares)
ROW_FLOATS = TILE * 3  # one pixel row of a tile


def render_streams(n: int, device=None, streams=None) -> list:
    """`n` render streams for frames in flight: `streams` when given (reused, e.g. one set for
    every renderer of a probe), else n consecutive streams of torch's per-device stream pool —
    never the caller's default stream.  HIP hands the process's hardware queues
    (GPU_MAX_HW_QUEUES: 4, HIP's default and the GPU box's setting) to streams in turn at creation, and two
    streams on one queue serialise their kernels; streams created together sit on different
    queues as long as there are enough, whereas the default stream shares its queue with one of
    them.  (Rendering on the default stream plus three pool streams made the
    one-GPU share probe bimodal: 0.056 or 0.093 ms for the same 1/8 share)"""
    import torch
    if streams is not None:
        out = list(streams)[:n]
        assert len(out) == n, "need one stream per frame in flight"
        return out
    return [torch.cuda.Stream(device=device) for _ in range(n)]


def pick_render_streams(scene, inflight: int, world: int, sets: int = 3, steps: int = 12,
                        device=None):
    """The render streams for a rank's small per-step launches, chosen by measurement: `sets`
    fresh stream sets, each timed rendering the middle 1/world of camera 0's tile rows in place
    with `inflight` frames in flight, the fastest kept.  HIP maps streams to hardware queues
    when they are created, and which set a rank gets decides the time of its small launches: a
    1/8 band of the C3 frame took 0.071-0.085 ms per step on the first set a process created and
    0.055-0.060 on the next ones, with GPU_MAX_HW_QUEUES 4 (whole frames: within 1 %;
    profiles/r05/stream_sets/).  Returns (streams, ms per step of each set)."""
    import time
    import torch
    cam = scene.camera(0)
    tx, ty = tiles_of((cam.width, cam.height))
    rows = max(1, ty // max(1, world))
    b = CameraBand(0, (ty - rows) // 2, rows, tx, 0, 0)
    frames = [torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
              for _ in range(inflight)]
    best, best_ms, times = None, float("inf"), []
    for _ in range(max(1, sets)):
        S = render_streams(inflight, device)
        for st in S:
            st.wait_stream(torch.cuda.current_stream())

        def run(k):
            for i in range(k):
                scene.render_device(0, frames[i % inflight].data_ptr(), tile_begin=b.tile_begin,
                                    tile_step=1, tile_count=b.tile_count,
                                    stream=S[i % inflight].cuda_stream)
            for st in S:
                torch.cuda.current_stream().wait_stream(st)
            torch.cuda.synchronize()
        run(2 * inflight)
        t0 = time.perf_counter()
        run(steps)
        ms = (time.perf_counter() - t0) / steps * 1e3
        times.append(round(ms, 4))
        if ms < best_ms:
            best, best_ms = S, ms
    scene.collect_stats()
    return best, times


def tiles_of(size: Tuple[int, int]) -> Tuple[int, int]:
    w, h = size
    return (w + TILE - 1) // TILE, (h + TILE - 1) // TILE


def deal_block_tile(tiles_x: int, d, w):
    """Tile (tx, ty) of tile w of deal block d (rt_internal.h deal_block_tile: block rows
    rotated by their row index; numpy arrays welcome)."""
    nbx = (tiles_x + 1) // 2
    by = d // nbx
    bx = (d - by * nbx + by % nbx) % nbx
    return 2 * bx + (w & 1), 2 * by + (w >> 1)


def deal_block_index(tiles_x: int, tx, ty):
    """(deal block d, tile w within it) of tile (tx, ty): the inverse of deal_block_tile."""
    nbx = (tiles_x + 1) // 2
    bx, by = tx // 2, ty // 2
    return by * nbx + (bx - by) % nbx, 2 * (ty & 1) + (tx & 1)


@dataclass
class CameraShare:
    camera: int
    tile_begin: int   # first camera-local deal unit of this rank
    tile_step: int    # = world
    count: int        # deal units of this camera rendered by this rank
    offset: int       # start (in tiles) of this camera's slot in the rank buffer
    slot: int         # slot size in tiles (same on every rank)
    blocks: bool      # deal units are 2x2 tile blocks (RT_TILE_BLOCKS), else tiles


class TileLayout:
    """Global round-robin assignment of deal units to ranks for a list of camera frame sizes.
    A deal unit is a 2x2 block of tiles in deal order (blocks=True, the default: what
    rt_render_device's RT_TILE_BLOCKS renders, 4 tiles per unit in the slot) or one tile."""

    def __init__(self, sizes: Sequence[Tuple[int, int]], world: int, rank: int,
                 blocks: bool = True):
        self.sizes = [tuple(s) for s in sizes]
        self.blocks = bool(blocks)
        self.unit_tiles = 4 if self.blocks else 1
        txy = [tiles_of(s) for s in self.sizes]
        self.tiles_per_camera = [tx * ty for tx, ty in txy]
        self.units_per_camera = [((tx + 1) // 2) * ((ty + 1) // 2) if self.blocks else tx * ty
                                 for tx, ty in txy]
        self.world = world
        self.rank = rank
        self.offsets = np.concatenate([[0], np.cumsum(self.units_per_camera)]).astype(np.int64)
        self.total = int(self.offsets[-1])
        self.slots = [self.unit_tiles * ((U + world - 1) // world) for U in self.units_per_camera]
        self.slot_offsets = np.concatenate([[0], np.cumsum(self.slots)]).astype(np.int64)
        self.buffer_tiles = int(self.slot_offsets[-1])
        self.per_rank = [self._shares(r) for r in range(world)]
        self.shares = self.per_rank[rank]
        self.local_tiles = sum(s.count for s in self.shares) * self.unit_tiles

    def begin(self, r: int, c: int) -> int:
        """First unit of camera c dealt to rank r (global unit g goes to rank g mod world)."""
        return int((r - self.offsets[c]) % self.world)

    def _shares(self, r: int) -> List[CameraShare]:
        out = []
        for c, U in enumerate(self.units_per_camera):
            b = self.begin(r, c)
            count = 0 if b >= U else (U - b + self.world - 1) // self.world
            out.append(CameraShare(c, b, self.world, count, int(self.slot_offsets[c]),
                                   self.slots[c], self.blocks))
        return out

    def share_tiles(self, c: int, r: int) -> np.ndarray:
        """Row-major frame tile index of each tile rank r renders for camera c, in slot order
        (-1: a block tile outside the tile grid, rendered as zeros)."""
        sh = self.per_rank[r][c]
        tx, ty = tiles_of(self.sizes[c])
        u = sh.tile_begin + np.arange(sh.count, dtype=np.int64) * sh.tile_step
        if not self.blocks:
            return u
        d = np.repeat(u, 4)
        w = np.tile(np.arange(4, dtype=np.int64), sh.count)
        x, y = deal_block_tile(tx, d, w)
        return np.where((x < tx) & (y < ty), y * tx + x, -1)

    def row_index(self, c: int) -> np.ndarray:
        """Untile index of camera c.  The gathered slots [world, slot, 8 rows, 24 floats] are
        viewed as 96-byte tile rows; entry (y, x) of the returned [ty*8, tx] array is the tile
        row that becomes pixel row y, pixels 8x..8x+7, of the (tile-padded) frame."""
        tx, ty = tiles_of(self.sizes[c])
        t = np.arange(tx * ty, dtype=np.int64)
        if self.blocks:
            u, w = deal_block_index(tx, t % tx, t // tx)
        else:
            u, w = t, 0
        r = (u + self.offsets[c]) % self.world
        b = (r - self.offsets[c]) % self.world
        pos = self.unit_tiles * ((u - b) // self.world) + w
        tile_src = (r * self.slots[c] + pos).reshape(ty, tx)  # gathered tile of each frame tile
        y = np.arange(ty * TILE, dtype=np.int64)
        return (tile_src[y // TILE] * TILE + (y % TILE)[:, None]).astype(np.int64)


def untile_camera(gathered_c, layout: TileLayout, c: int, index=None, out=None):
    """gathered_c: tensor [world * slot_c, 192] (any device) — camera c's slots of every rank.
    Returns the [h, w, 3] row-major frame (a view of `out`, a [ty*8, tx*8, 3] buffer, when
    given)."""
    import torch
    tx, ty = tiles_of(layout.sizes[c])
    if index is None:
        index = torch.as_tensor(layout.row_index(c).reshape(-1), device=gathered_c.device)
    if out is None:
        out = torch.empty((ty * TILE, tx * TILE, 3), dtype=gathered_c.dtype,
                          device=gathered_c.device)
    torch.index_select(gathered_c.view(-1, ROW_FLOATS), 0, index, out=out.view(-1, ROW_FLOATS))
    w, h = layout.sizes[c]
    return out[:h, :w]


def scene_tile_untiler(scene, layout: TileLayout, records: bool = False) -> Callable:
    """The GPU untile: rt_untile_device of camera c's gathered shares straight into its
    row-major frame, on `stream`; skip_root: rank 0's own units are already in the frame.
    records: the shares are pixel records, shaded into the frame by rt_resolve_device."""
    def untile(c, gathered_c, frame, stream, skip_root=False):
        sh = layout.shares[c]
        fn = scene.resolve_device if records else scene.untile_device
        fn(c, layout.world, sh.slot, gathered_c.data_ptr(), frame.data_ptr(),
           tile_offset=int(layout.offsets[c] % layout.world), blocks=layout.blocks,
           skip_root=skip_root, stream=stream.cuda_stream)
    return untile


def scene_inplace_renderer(scene) -> Callable:
    """Rank 0's own share rendered in place into camera c's row-major frame (its units only)."""
    def render(sh: CameraShare, frame, stream):
        scene.render_device(sh.camera, frame.data_ptr(), tile_begin=sh.tile_begin,
                            tile_step=sh.tile_step, tile_major=False, blocks=sh.blocks,
                            stream=stream.cuda_stream)
    return render


def scene_tile_renderer(scene, records: bool = False) -> Callable:
    """The GPU tile renderer: rt_render_device of camera c's share, tile-major into `slot`
    (records: 64 pixel records per tile, RT_TILE_RECORDS, instead of RGB)."""
    def render(sh: CameraShare, slot, stream):
        scene.render_device(sh.camera, slot.data_ptr(), tile_begin=sh.tile_begin,
                            tile_step=sh.tile_step, tile_major=True, blocks=sh.blocks,
                            stream=stream.cuda_stream, records=records)
    return render


def records_ok(scene) -> bool:
    """Every camera of the scene may send its shares as pixel records (rt_scene_records_ok)."""
    return all(scene.records_ok(c) for c in range(scene.num_cameras))


class FrameRenderer:
    """One GPU, no exchange: one step = every camera of `scene` rendered in place into
    row-major frames.  Consecutive steps go to `inflight` streams in turn (each with its own
    frames and, in the library, its own scratch), so a frame's last, sparsely occupied waves
    overlap the next frame's work; finish() joins them back into `stream`."""

    def __init__(self, scene, stream, inflight: int = 1, streams=None):
        import torch
        self.scene = scene
        self.stream = stream
        self.sizes = [(scene.camera(c).width, scene.camera(c).height)
                      for c in range(scene.num_cameras)]
        dev = torch.device("cuda", torch.cuda.current_device())
        self.inflight = max(1, int(inflight))
        # render streams (render_streams: pool streams, or `streams`); `stream` only joins them
        self.streams = render_streams(self.inflight, dev, streams)
        for st in self.streams:
            st.wait_stream(stream)
        self.frame_sets = [[torch.empty((h, w, 3), dtype=torch.float32, device=dev)
                            for (w, h) in self.sizes] for _ in range(self.inflight)]
        self.frames = self.frame_sets[0]
        self.k = 0

    def step(self, events=None):
        slot = self.k % self.inflight
        self.k += 1
        st = self.streams[slot]
        if events is not None:
            events[0].record(st)
        self.frames = self.frame_sets[slot]
        for c, f in enumerate(self.frames):
            self.scene.render_device(c, f.data_ptr(), stream=st.cuda_stream)
        if events is not None:
            events[1].record(st)
        return self.frames

    def finish(self):
        for st in self.streams:
            self.stream.wait_stream(st)


class TileGatherRenderer:
    """One step = every camera of the job split over the ranks by tiles (TileLayout), gathered
    to rank 0 and untiled there: strong scaling of one frame over the N GPUs.

    render(share, slot, stream) writes the rank's tiles of camera share.camera tile-major into
    `slot` (a [slot tiles, 192] view) on `stream` (scene_tile_renderer on the GPU).  Step k uses
    buffer set s = k mod F (F = inflight): its render stream renders every share into set s,
    an event hands the set to the communication stream, which gathers each camera's slots to
    rank 0 (one equal-size dist.gather per camera: RCCL send / receive pairs over xGMI with
    backend "nccl") and, on rank 0, untiles them into set s's frames.  A set is rendered again
    only after its gather F steps earlier has finished (per-set events), so up to F frames are
    in flight per rank and a rank's render streams never wait on the exchange of the frame
    before.  host_staging=True (gloo, CPU tensors): the same exchange synchronously through the
    host, one buffer set.  frames: rank 0's frames of the last step (complete after finish())."""

    def __init__(self, layout: TileLayout, stream, render: Callable, inflight: int = 2,
                 host_staging: bool = False, device=None, untile: Optional[Callable] = None,
                 gather_stream: str = "render", render_inplace: Optional[Callable] = None,
                 cpu_fakes: bool = False, self_exchange: bool = False,
                 tile_words: int = TILE_FLOATS):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.layout = L = layout
        self.stream = stream
        self.render = render
        # untile(c, gathered_c [world, slot, 192], frame [h, w, 3], stream): rank 0's untile
        # (scene_tile_untiler: the library's kernel); None: one index_select into padded frames
        self.untile = untile
        self.host_staging = host_staging
        # "render": a step's gather and untile are enqueued on its own render stream after the
        # render (the other steps' streams keep rendering meanwhile; set s is reused on the same
        # stream, so no events); "comm": on one communication stream, handed over by events
        assert gather_stream in ("render", "comm")
        self.gather_on_render = gather_stream == "render"
        # root_inplace (GPU, library untile): rank 0 renders its own share in place into the
        # frame, receives only the other ranks' slots (point-to-point, no self-copy) and the
        # untile skips its units — at N = 1 the step is the in-place render alone
        self.render_inplace = render_inplace
        self.root_inplace = render_inplace is not None and untile is not None
        if self.root_inplace and host_staging and not cpu_fakes:
            # the library's in-place renderer and untiler write device pointers; with host
            # staging the frames are host tensors (cpu_fakes: host-memory test doubles)
            raise ValueError("render_inplace + untile need device buffers (host_staging=False)")
        # self_exchange (the one-rank rehearsal of the root-in-place exchange): with nobody else
        # to receive from, rank 0 renders its share tile-major anyway, posts it to itself as one
        # isend / irecv pair (batch_isend_irecv: RCCL send / receive) and untiles all of it —
        # the exchange an N-rank run makes, with rank 0 standing in for every peer
        self.self_loop = bool(self_exchange) and self.root_inplace and L.world == 1
        self.inflight = 1 if host_staging else max(1, int(inflight))
        F = self.inflight
        dev = device if device is not None else (
            "cpu" if host_staging else torch.device("cuda", torch.cuda.current_device()))
        self.rank = L.rank
        if host_staging:
            self.rstreams = [stream]
            self.comm = None
        else:
            self.rstreams = render_streams(F, dev)  # (pool streams, one per frame in flight)
            self.comm = torch.cuda.Stream(device=dev)
        # tile_words: 4-B words per tile in the slots (TILE_FLOATS RGB, TILE_RECORDS records)
        self.tile_words = int(tile_words)
        self.local = [torch.zeros((L.buffer_tiles, self.tile_words), dtype=torch.float32,
                                  device=dev) for _ in range(F)]
        if not host_staging:
            # the zero fill above ran on the allocating (current) stream: every stream that
            # writes or reads these buffers first waits for it
            cur = torch.cuda.current_stream(dev)
            for st in self.rstreams + [self.comm]:
                st.wait_stream(cur)
                if stream is not None:
                    st.wait_stream(stream)
        self.done = [torch.cuda.Event() if not host_staging else None for _ in range(F)]
        self.handoff = [torch.cuda.Event() if not host_staging else None for _ in range(F)]
        self.used = [False] * F
        self.k = 0
        self.frames = None
        if self.rank == 0:
            self.gathered = [[torch.empty((L.world, sh.slot, self.tile_words), dtype=torch.float32,
                                          device=dev) for sh in L.shares] for _ in range(F)]
            self.index = [torch.as_tensor(L.row_index(c).reshape(-1), device=dev)
                          for c in range(len(L.shares))]
            self.padded = []
            for _ in range(F):
                row = []
                for (w, h) in L.sizes:
                    tx, ty = tiles_of((w, h))
                    shape = (h, w, 3) if untile is not None else (ty * TILE, tx * TILE, 3)
                    row.append(torch.empty(shape, dtype=torch.float32, device=dev))
                self.padded.append(row)

    def _slot(self, s: int, sh: CameraShare):
        return self.local[s][sh.offset:sh.offset + sh.slot]

    def _gather(self, s: int, stream=None):
        torch, dist, L = self.torch, self.dist, self.layout
        root = self.rank == 0
        for c, sh in enumerate(L.shares):
            if self.root_inplace:
                if L.world > 1:
                    ops = ([dist.P2POp(dist.irecv, self.gathered[s][c][r], r)
                            for r in range(1, L.world)] if root else
                           [dist.P2POp(dist.isend, self._slot(s, sh), 0)])
                    for req in dist.batch_isend_irecv(ops):
                        req.wait()
                elif self.self_loop and self.host_staging:  # (gloo has no pair to itself)
                    self.gathered[s][c][0].copy_(self._slot(s, sh))
                elif self.self_loop:
                    ops = [dist.P2POp(dist.isend, self._slot(s, sh), 0),
                           dist.P2POp(dist.irecv, self.gathered[s][c][0], 0)]
                    for req in dist.batch_isend_irecv(ops):
                        req.wait()
            elif self.host_staging:
                glist = list(torch.empty((L.world, sh.slot, self.tile_words))) if root else None
                dist.gather(self._slot(s, sh).cpu(), glist, dst=0)
                if root:
                    self.gathered[s][c].copy_(torch.stack(glist))
            else:
                outs = list(self.gathered[s][c]) if root else None
                dist.gather(self._slot(s, sh), outs, dst=0, async_op=True).wait()
            if root and self.root_inplace:
                if L.world > 1:
                    self.untile(c, self.gathered[s][c], self.padded[s][c], stream, skip_root=True)
                elif self.self_loop:
                    self.untile(c, self.gathered[s][c], self.padded[s][c], stream, skip_root=False)
            elif root and self.untile is not None:
                self.untile(c, self.gathered[s][c], self.padded[s][c], stream)
            elif root:
                untile_camera(self.gathered[s][c].view(-1, TILE_FLOATS), L, c, self.index[c],
                              self.padded[s][c])

    def step(self, events=None):
        s = self.k % self.inflight
        self.k += 1
        st = self.rstreams[s]
        if not self.host_staging and self.used[s] and not self.gather_on_render:
            st.wait_event(self.done[s])  # its gather `inflight` steps ago
        if events is not None:
            events[0].record(st)
        for c, sh in enumerate(self.layout.shares):
            if sh.count > 0:
                if self.root_inplace and self.rank == 0 and not self.self_loop:
                    self.render_inplace(sh, self.padded[s][c], st)
                else:
                    self.render(sh, self._slot(s, sh), st)
        if events is not None:
            events[1].record(st)
        if self.host_staging:
            self._gather(s)
        elif self.gather_on_render:
            with self.torch.cuda.stream(st):
                self._gather(s, st)
        else:
            self.handoff[s].record(st)
            with self.torch.cuda.stream(self.comm):
                self.comm.wait_event(self.handoff[s])
                self._gather(s, self.comm)
                self.done[s].record(self.comm)
            self.used[s] = True
        if self.rank == 0:
            self.frames = [p[:h, :w] for p, (w, h) in zip(self.padded[s], self.layout.sizes)]
        return self.frames

    def finish(self):
        """Make `stream` wait for every render stream and every outstanding gather / untile."""
        if self.host_staging:
            return
        for st in self.rstreams:
            self.stream.wait_stream(st)
        self.stream.wait_stream(self.comm)


class FrameOwners:
    """Whole-frame assignment for jobs of at least one frame per rank (weak scaling): camera c
    belongs to rank c mod world.  Gather round j collects cameras j*world .. j*world + world-1
    (one frame from every rank; a rank with no camera in the round sends padding)."""

    def __init__(self, n_cams: int, world: int, rank: int):
        self.n_cams, self.world, self.rank = n_cams, world, rank
        self.rounds = (n_cams + world - 1) // world
        self.owned = [j * world + rank for j in range(self.rounds)]  # may exceed n_cams - 1

    def camera(self, j: int, r: int) -> int:
        return j * self.world + r


class FrameGatherRenderer:
    """One step = every rank renders its own whole frames (FrameOwners) in place and rank 0
    gathers them: per round j, one equal-size collective of full row-major frames (RCCL over
    xGMI with backend "nccl", host copies with gloo).  Unlike the tile deal of
    TileGatherRenderer, a rank's frame is one launch of a full frame, so per-launch work does
    not shrink as the world grows (weak scaling).  Consecutive steps alternate over `inflight`
    render streams, each with its own send / receive buffers; a buffer set is rendered again
    only after its gathers `inflight` steps earlier have finished (events), and rank 0's frames
    of a step are complete once finish() has joined the streams.

    render(c, out, stream) writes camera c's [h, w, 3] frame into tensor `out` on `stream`
    (None: the scene's rt_render_device), so the same bookkeeping runs in the gloo tests."""

    def __init__(self, scene, owners: FrameOwners, sizes, stream, host_staging=False,
                 inflight=2, device=None, render=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.owners, self.stream, self.host_staging = owners, stream, host_staging
        self.sizes = [tuple(x) for x in sizes]
        assert len(set(self.sizes)) == 1, "every frame of a gather round must have one size"
        w, h = self.sizes[0]
        self.render = render or (lambda c, out, st: scene.render_device(
            c, out.data_ptr(), stream=st.cuda_stream))
        self.inflight = max(1, int(inflight)) if not host_staging else 1
        dev = device
        self.streams = render_streams(self.inflight, dev) if not host_staging else []
        self.comm = torch.cuda.Stream(device=dev) if not host_staging else None
        W = owners.world
        self.send = [[torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
                      for _ in range(owners.rounds)] for _ in range(self.inflight)]
        self.recv = None
        if owners.rank == 0:
            self.recv = [[torch.empty((h, w, 3), dtype=torch.float32, device=dev)
                          for _ in range(owners.rounds * W)] for _ in range(self.inflight)]
        if not host_staging:  # the zero fill ran on the current stream (see TileGatherRenderer)
            cur = torch.cuda.current_stream(dev)
            for st in self.streams + [self.comm]:
                st.wait_stream(cur)
                if stream is not None:
                    st.wait_stream(stream)
        self.done = [torch.cuda.Event() if not host_staging else None for _ in range(self.inflight)]
        self.used = [False] * self.inflight
        self.k = 0
        self.frames = None

    def step(self, events=None):
        torch, dist, O = self.torch, self.dist, self.owners
        slot = self.k % self.inflight
        self.k += 1
        st = self.streams[slot] if not self.host_staging else None
        if events is not None and st is not None:
            events[0].record(st)
        if self.used[slot] and not self.host_staging:  # its gathers `inflight` steps ago
            st.wait_event(self.done[slot])
        for j in range(O.rounds):
            c = O.camera(j, O.rank)
            if c < O.n_cams:
                self.render(c, self.send[slot][j], st)
            outs = ([self.recv[slot][O.camera(j, r)] for r in range(O.world)]
                    if O.rank == 0 else None)
            if self.host_staging:
                if st is not None:
                    st.synchronize()
                host = self.send[slot][j].cpu()
                hl = list(torch.empty((O.world,) + tuple(host.shape))) if O.rank == 0 else None
                dist.gather(host, hl, dst=0)
                if O.rank == 0:
                    for r in range(O.world):
                        outs[r].copy_(hl[r])
                continue
            ev = torch.cuda.Event()
            ev.record(st)
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(ev)
                work = dist.gather(self.send[slot][j], outs, dst=0, async_op=True)
                work.wait()  # the comm stream waits for the collective
        if not self.host_staging:
            self.done[slot].record(self.comm)
            self.used[slot] = True
        if events is not None and st is not None:
            events[1].record(st)
        self.frames = self.recv[slot][:O.n_cams] if O.rank == 0 else None
        return self.frames

    def finish(self):
        """Make `stream` wait for every render stream and every outstanding gather."""
        if self.host_staging:
            return
        for st in self.streams:
            self.stream.wait_stream(st)
        self.stream.wait_stream(self.comm)


class ShareRenderer:
    """One GPU rendering ONE rank's share of the tile deal of `world` ranks (TileLayout), with
    no exchange: the per-rank render work of the N > 1 path, measured on one GPU to predict
    strong scaling before an N-GPU node is available (bench.py share probe).  Steps go to
    `inflight` streams / buffer sets in turn, as in TileGatherRenderer."""

    def __init__(self, scene, world: int, rank: int, stream, inflight: int = 1, streams=None,
                 records: bool = False):
        import torch
        self.layout = L = TilePlan(scene, world, rank)
        self.records = records
        self.scene, self.stream = scene, stream
        dev = torch.device("cuda", torch.cuda.current_device())
        self.inflight = max(1, int(inflight))
        # streams: the render streams to reuse (render_streams; one set for every rank probed, as
        # each rank of an N-GPU run creates its own set in a fresh process)
        self.streams = render_streams(self.inflight, dev, streams)
        for st in self.streams:
            st.wait_stream(stream)
        self.local = [torch.empty((max(1, L.buffer_tiles), TILE_FLOATS), dtype=torch.float32,
                                  device=dev) for _ in range(self.inflight)]
        self.k = 0

    def step(self, events=None):
        s = self.k % self.inflight
        self.k += 1
        st = self.streams[s]
        for sh in self.layout.shares:
            if sh.count > 0:
                slot = self.local[s][sh.offset:sh.offset + sh.slot]
                self.scene.render_device(sh.camera, slot.data_ptr(), tile_begin=sh.tile_begin,
                                         tile_step=sh.tile_step, tile_major=True,
                                         blocks=sh.blocks, stream=st.cuda_stream,
                                         records=self.records)

    def finish(self):
        for st in self.streams:
            self.stream.wait_stream(st)


# ------------------------------------------------------------------ row bands
# The band split: camera c's frame is cut into `world` bands of whole 8-pixel tile rows, band r
# to rank r, the cuts placed so the bands' measured costs (rt_tile_costs of a whole frame) are
# as equal as contiguous rows allow.  A band of tile rows is one contiguous run of the row-major
# frame, so a rank renders its band in place (a tile range of rt_render_device_range) and
# rank 0 receives every other band straight into its frame: no untile, nothing extra on rank 0.

def band_cuts(row_costs: Sequence[float], world: int,
              weights: Optional[Sequence[float]] = None) -> List[int]:
    """Cuts 0 = c_0 <= c_1 <= ... <= c_world = len(row_costs) of the rows into `world` contiguous
    bands (band r = rows [c_r, c_r+1)) minimising the heaviest band's cost / weights[r] (weights:
    each band's share of the work, default equal; rank 0's band is lighter when it also shades the
    others' pixel records): a binary search over the scale with the greedy in-order fill."""
    x = np.maximum(np.asarray(row_costs, dtype=np.float64), 0.0)
    n = len(x)
    if n == 0:
        return [0] * (world + 1)
    if x.sum() <= 0:
        x = np.ones(n)
    wt = np.ones(world) if weights is None else np.maximum(np.asarray(weights, np.float64), 0.0)
    assert len(wt) == world and wt.max() > 0
    pre = np.concatenate([[0.0], np.cumsum(x)])

    def fill(lam):  # each band in turn takes rows while its cost stays within lam * weight
        cuts, i = [0], 0
        for r in range(world):
            # the last row index j with pre[j] - pre[i] <= cap (at least i)
            j = int(np.searchsorted(pre, pre[i] + lam * wt[r] * (1 + 1e-12), side="right")) - 1
            i = max(i, min(n, j))
            cuts.append(i)
        return cuts

    lo, hi = 0.0, float(pre[-1]) / float(wt.max()) * (1 + 1e-9)
    for _ in range(80):
        mid = 0.5 * (lo + hi)
        if fill(mid)[-1] >= n:
            hi = mid
        else:
            lo = mid
    cuts = fill(hi)
    cuts[-1] = n
    return [int(c) for c in cuts]


@dataclass
class CameraBand:
    camera: int
    row0: int        # first tile row
    rows: int        # tile rows
    tiles_x: int
    y0: int          # pixel rows [y0, y1) of the frame (clipped to its height)
    y1: int

    @property
    def tile_begin(self) -> int:
        return self.row0 * self.tiles_x

    @property
    def tile_count(self) -> int:
        return self.rows * self.tiles_x


class BandPlan:
    """Row bands of every camera over `world` ranks.  cuts[c] = the world + 1 tile-row cuts of
    camera c (band_cuts of its measured row costs; equal rows when no costs are given).  Every
    rank must hold the same cuts: rank 0 measures them and broadcasts (bench.py)."""

    def __init__(self, sizes: Sequence[Tuple[int, int]], world: int, rank: int,
                 cuts: Optional[Sequence[Sequence[int]]] = None):
        self.sizes = [tuple(s) for s in sizes]
        self.world, self.rank = world, rank
        txy = [tiles_of(s) for s in self.sizes]
        if cuts is None:
            cuts = [band_cuts(np.ones(ty), world) for _, ty in txy]
        self.cuts = [[int(x) for x in c] for c in cuts]
        for c, (cc, (tx, ty)) in enumerate(zip(self.cuts, txy)):
            assert len(cc) == world + 1 and cc[0] == 0 and cc[-1] == ty and \
                all(a <= b for a, b in zip(cc, cc[1:])), f"bad cuts for camera {c}: {cc}"
        self.per_rank = [[CameraBand(c, cc[r], cc[r + 1] - cc[r], tx, min(h, TILE * cc[r]),
                                     min(h, TILE * cc[r + 1]))
                          for c, (cc, (tx, _), (_, h)) in enumerate(zip(self.cuts, txy, self.sizes))]
                         for r in range(world)]
        self.bands = self.per_rank[rank]

    @classmethod
    def from_costs(cls, sizes, world: int, rank: int, tile_costs: Sequence[np.ndarray],
                   weights: Optional[Sequence[float]] = None):
        """tile_costs[c]: camera c's row-major per-tile costs (rt_tile_costs of a whole frame);
        weights: each rank's share of the render work (band_cuts)."""
        cuts = []
        for (w, h), cost in zip(sizes, tile_costs):
            tx, ty = tiles_of((w, h))
            cuts.append(band_cuts(np.asarray(cost, np.float64).reshape(ty, tx).sum(1), world,
                                  weights))
        return cls(sizes, world, rank, cuts)

    def band_costs(self, tile_costs: Sequence[np.ndarray]) -> np.ndarray:
        """[world] summed tile costs of each rank's bands (all cameras)."""
        out = np.zeros(self.world)
        for c, ((w, h), cost) in enumerate(zip(self.sizes, tile_costs)):
            tx, ty = tiles_of((w, h))
            rows = np.asarray(cost, np.float64).reshape(ty, tx).sum(1)
            for r in range(self.world):
                out[r] += rows[self.cuts[c][r]:self.cuts[c][r + 1]].sum()
        return out


def measure_tile_costs(scene, frames: int = 5) -> List[np.ndarray]:
    """Every camera's per-tile costs: `frames` whole frames rendered one at a time on a fresh
    stream (rt_tile_costs after each), the element-wise median of the maps."""
    import torch
    st = torch.cuda.Stream()
    out = []
    for c in range(scene.num_cameras):
        cam = scene.camera(c)
        buf = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
        n = scene.num_tiles(c)
        maps = []
        for _ in range(max(1, frames)):
            scene.render_device(c, buf.data_ptr(), stream=st.cuda_stream)
            maps.append(scene.tile_costs(st.cuda_stream, n))
        out.append(np.median(np.stack(maps), axis=0))
    st.synchronize()
    scene.release_stream(st.cuda_stream)
    return out


def measure_resolve_frac(scene, frames: int = 5) -> float:
    """rt_resolve_rows of a whole frame's pixel records over the frame's in-place render, camera
    0, each timed alone on one stream (HIP events, median of `frames`): how much of a frame's
    work rank 0 adds per frame when it shades the others' records."""
    import torch
    cam = scene.camera(0)
    st = torch.cuda.Stream()
    buf = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    rec = torch.empty((cam.height, cam.width), dtype=torch.int32, device="cuda")
    scene.render_device(0, rec.data_ptr(), stream=st.cuda_stream, records=True)
    ren, res = [], []
    for _ in range(max(1, frames) + 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(st)
        scene.render_device(0, buf.data_ptr(), stream=st.cuda_stream)
        e[1].record(st)
        scene.resolve_rows(0, 0, cam.height, rec.data_ptr(), buf.data_ptr(), stream=st.cuda_stream)
        e[2].record(st)
        st.synchronize()
        ren.append(e[0].elapsed_time(e[1]))
        res.append(e[1].elapsed_time(e[2]))
    scene.release_stream(st.cuda_stream)
    return float(np.median(res[1:]) / max(1e-9, np.median(ren[1:])))


def scene_band_renderer(scene, records: bool = False) -> Callable:
    """Band b of camera b.camera rendered in place into its row-major frame (a tile range);
    records: as row-major 32-bit pixel records (RT_TILE_RECORDS) into a [h, w] word buffer."""
    def render(b: CameraBand, frame, stream):
        scene.render_device(b.camera, frame.data_ptr(), tile_begin=b.tile_begin, tile_step=1,
                            tile_count=b.tile_count, stream=stream.cuda_stream, records=records)
    return render


def scene_row_resolver(scene) -> Callable:
    """rt_resolve_rows: rows [y0, y1) of camera c's row-major records shaded into its frame."""
    def resolve(c, y0, y1, records, frame, stream):
        scene.resolve_rows(c, y0, y1, records.data_ptr(), frame.data_ptr(),
                           stream=stream.cuda_stream)
    return resolve


def root_band_weights(world: int, resolve_frac: float) -> List[float]:
    """Band weights when rank 0 also shades the other ranks' pixel records: resolve_frac = the
    resolve of a whole frame / its render.  Rank 0's band shrinks so that its render plus its
    resolve of the other (world - 1) / world of the frame takes as long as another rank's band:
    with T the per-rank time in frame renders, T = (1 + rho (N - 1) / N) / N and rank 0's band
    is T - rho (N - 1) / N (at least 0)."""
    if world <= 1:
        return [1.0]
    rho = max(0.0, float(resolve_frac)) * (world - 1) / world
    T = (1.0 + rho) / world
    return [max(0.0, T - rho) / T] + [1.0] * (world - 1)


def BandRenderPlan(scene, world: int, rank: int, cuts=None) -> BandPlan:
    sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
    return BandPlan(sizes, world, rank, cuts)


class BandGatherRenderer:
    """One step = every camera split over the ranks in row bands (BandPlan), each rank's bands
    rendered in place into its own frames, and every band of ranks > 0 sent to rank 0 straight
    into its frames (point-to-point, batch_isend_irecv: RCCL send / receive over xGMI with backend
    "nccl").  No untile: a band is a contiguous run of rows.  Steps go to `inflight` render
    streams / frame sets in turn; a step's exchange is enqueued on its own render stream after its
    render, so a set is rendered again only after its exchange `inflight` steps earlier.
    host_staging=True (gloo, CPU tensors): the same exchange through the host, one set.
    self_exchange (one-rank rehearsal): rank 0 renders its band into a separate buffer and sends
    it to itself into the frame (RCCL self send / receive; a local copy with gloo).
    frames: rank 0's frames of the last step (complete after finish())."""

    def __init__(self, plan: BandPlan, stream, render: Callable, inflight: int = 2,
                 host_staging: bool = False, device=None, self_exchange: bool = False,
                 render_records: Optional[Callable] = None, resolve: Optional[Callable] = None,
                 streams=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.plan = self.layout = plan
        self.stream, self.render = stream, render
        self.host_staging = host_staging
        self.inflight = 1 if host_staging else max(1, int(inflight))
        self.rank = plan.rank
        self.self_loop = bool(self_exchange) and plan.world == 1
        dev = device if device is not None else (
            "cpu" if host_staging else torch.device("cuda", torch.cuda.current_device()))
        self.rstreams = [stream] if host_staging else render_streams(self.inflight, dev, streams)
        self.frame_sets = [[torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
                            for (w, h) in plan.sizes] for _ in range(self.inflight)]
        self.local = ([[torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
                        for (w, h) in plan.sizes] for _ in range(self.inflight)]
                      if self.self_loop else None)
        # pixel records (render_records + resolve): ranks > 0 (and rank 0 in the rehearsal)
        # render their bands as 32-bit records into a [h, w] word buffer and send those rows;
        # rank 0 receives them into its own record buffer and shades them into the frame
        self.records = render_records is not None and resolve is not None
        self.render_records, self.resolve = render_records, resolve
        self.rec_sets = ([[torch.zeros((h, w), dtype=torch.int32, device=dev)
                           for (w, h) in plan.sizes] for _ in range(self.inflight)]
                         if self.records else None)
        self.rec_recv = {}  # (set, camera) -> the rehearsal's received record rows
        if not host_staging:
            cur = torch.cuda.current_stream(dev)
            for st in self.rstreams:
                st.wait_stream(cur)
                if stream is not None:
                    st.wait_stream(stream)
        self.k = 0
        self.frames = None

    def _payload(self, s: int, c: int, b: CameraBand, local: bool = False):
        """What travels for band b: its frame rows (RGB) or its record rows."""
        if self.records:
            return self.rec_sets[s][c][b.y0:b.y1]
        return (self.local if local else self.frame_sets)[s][c][b.y0:b.y1]

    def _exchange(self, s: int):
        dist, P = self.dist, self.plan
        ops = []
        if P.world > 1 and self.host_staging:  # gloo: host tensors, the receives copied in
            for c in range(len(P.sizes)):
                if self.rank == 0:
                    for r in range(1, P.world):
                        b = P.per_rank[r][c]
                        if b.y1 > b.y0:
                            dst = self._payload(s, c, b)
                            tmp = self.torch.empty(dst.shape, dtype=dst.dtype)
                            dist.recv(tmp, r)
                            dst.copy_(tmp)
                else:
                    b = P.bands[c]
                    if b.y1 > b.y0:
                        dist.send(self._payload(s, c, b).cpu(), 0)
        elif P.world > 1:
            for c in range(len(P.sizes)):
                if self.rank == 0:
                    for r in range(1, P.world):
                        b = P.per_rank[r][c]
                        if b.y1 > b.y0:
                            ops.append(dist.P2POp(dist.irecv, self._payload(s, c, b), r))
                else:
                    b = P.bands[c]
                    if b.y1 > b.y0:
                        ops.append(dist.P2POp(dist.isend, self._payload(s, c, b), 0))
        elif self.self_loop:
            for c, b in enumerate(P.bands):
                if b.y1 <= b.y0:
                    continue
                if self.records:  # the record rows travel; the resolve below shades them
                    src = self._payload(s, c, b)
                    dst = self.torch.empty_like(src)
                    self.rec_recv[(s, c)] = dst
                else:
                    src, dst = self._payload(s, c, b, local=True), self._payload(s, c, b)
                if self.host_staging:  # (gloo has no pair to itself)
                    dst.copy_(src)
                else:
                    ops += [dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

    def _resolve(self, s: int, stream):
        """Rank 0: shade the received record rows (every band but its own) into the frames."""
        P = self.plan
        for c, (w, h) in enumerate(P.sizes):
            if self.self_loop:
                b = P.bands[c]
                if b.y1 > b.y0:
                    rec = self.rec_sets[s][c]  # the received rows replace the sent ones
                    rec[b.y0:b.y1].copy_(self.rec_recv[(s, c)])
                    self.resolve(c, b.y0, b.y1, rec, self.frame_sets[s][c], stream)
                continue
            own = P.bands[c]
            for y0, y1 in ((0, own.y0), (own.y1, h)):
                if y1 > y0:
                    self.resolve(c, y0, y1, self.rec_sets[s][c], self.frame_sets[s][c], stream)

    def step(self, events=None):
        s = self.k % self.inflight
        self.k += 1
        st = self.rstreams[s]
        if events is not None:
            events[0].record(st)
        target = self.local[s] if self.self_loop else self.frame_sets[s]
        for c, b in enumerate(self.plan.bands):
            if b.rows > 0:
                if self.records and (self.rank > 0 or self.self_loop):
                    self.render_records(b, self.rec_sets[s][c], st)
                else:  # rank 0's own band: RGB in place
                    self.render(b, target[c], st)
        if events is not None:
            events[1].record(st)
        if self.host_staging:
            self._exchange(s)
            if self.records and self.rank == 0:
                self._resolve(s, st)
        else:
            with self.torch.cuda.stream(st):
                self._exchange(s)
                if self.records and self.rank == 0:
                    self._resolve(s, st)
        if self.rank == 0:
            self.frames = self.frame_sets[s]
        return self.frames

    def finish(self):
        if self.host_staging:
            return
        for st in self.rstreams:
            self.stream.wait_stream(st)


def TilePlan(scene, world: int, rank: int, blocks: bool = True) -> TileLayout:
    """Tile layout for every camera of `scene`, checked against the library's tile count."""
    sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
    L = TileLayout(sizes, world, rank, blocks=blocks)
    for c in range(scene.num_cameras):
        assert L.tiles_per_camera[c] == scene.num_tiles(c), "tile count disagrees with the library"
    return L
