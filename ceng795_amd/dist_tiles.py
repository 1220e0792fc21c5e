"""Image-tile sharding over GPUs + framebuffer gather.

The reference splits a frame over host threads by interleaved rows (HW2/main.cpp:33-36,
HW2/Scene.cpp:25).  Here the 8x8-pixel tiles (one wavefront each) of every camera's frame are
numbered globally, camera after camera, and dealt round-robin over ranks — rank r renders
global tiles g = r (mod world) — which balances cost the way the row interleave does.  Each
rank writes its tiles back to back (tile-major) into HBM; rank 0 gathers the per-rank buffers
over RCCL (one process per GPU, torch.distributed "nccl") and untiles them into row-major
fp32 framebuffers.  There is no other exchange: the scene is replicated, rays are independent.

TileLayout and untile() are pure bookkeeping (numpy / torch CPU) so the N>1 logic is testable
with the gloo backend on CPU; FrameRenderer drives the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

TILE = 8
TILE_FLOATS = TILE * TILE * 3


@dataclass
class CameraShare:
    camera: int
    tile_begin: int   # first camera-local tile of this rank
    tile_step: int    # = world
    count: int        # tiles of this camera rendered by this rank
    offset: int       # position (in tiles) of this camera's share in the rank buffer


class TileLayout:
    """Global round-robin assignment of tiles to ranks for a list of cameras."""

    def __init__(self, tiles_per_camera: Sequence[int], world: int, rank: int):
        self.tiles_per_camera = list(tiles_per_camera)
        self.world = world
        self.rank = rank
        self.offsets = np.concatenate([[0], np.cumsum(self.tiles_per_camera)]).astype(np.int64)
        self.total = int(self.offsets[-1])
        self.per_rank = [self._shares(r) for r in range(world)]
        self.padded_tiles = max(sum(s.count for s in shares) for shares in self.per_rank)
        self.shares = self.per_rank[rank]
        self.local_tiles = sum(s.count for s in self.shares)

    def _shares(self, r: int) -> List[CameraShare]:
        out, pos = [], 0
        for c, T in enumerate(self.tiles_per_camera):
            off = int(self.offsets[c])
            begin = (r - off) % self.world
            count = 0 if begin >= T else (T - begin + self.world - 1) // self.world
            out.append(CameraShare(c, begin, self.world, count, pos))
            pos += count
        return out

    def untile_index(self) -> np.ndarray:
        """For every global tile g (camera-major), its row in the gathered
        [world * padded_tiles] tile array."""
        idx = np.empty(self.total, np.int64)
        for r, shares in enumerate(self.per_rank):
            for s in shares:
                if s.count == 0:
                    continue
                t = s.tile_begin + s.tile_step * np.arange(s.count)
                idx[self.offsets[s.camera] + t] = r * self.padded_tiles + s.offset + np.arange(s.count)
        return idx


def untile(gathered, layout: TileLayout, sizes: Sequence[tuple], index=None):
    """gathered: torch tensor [world * padded_tiles, 192] (any device).  sizes: (w, h) per
    camera.  Returns a list of [h, w, 3] row-major framebuffers."""
    import torch
    if index is None:
        index = torch.as_tensor(layout.untile_index(), device=gathered.device)
    tiles = gathered.index_select(0, index)
    frames = []
    for c, (w, h) in enumerate(sizes):
        tx, ty = (w + TILE - 1) // TILE, (h + TILE - 1) // TILE
        t = tiles[layout.offsets[c]:layout.offsets[c + 1]].view(ty, tx, TILE, TILE, 3)
        full = t.permute(0, 2, 1, 3, 4).reshape(ty * TILE, tx * TILE, 3)
        frames.append(full[:h, :w])
    return frames


class FrameRenderer:
    """One step = render every camera of `scene`; with gather=True, gather to rank 0 and untile.

    world == 1 and gather == False renders each camera in place into a row-major frame."""

    def __init__(self, scene, layout_or_none: Optional[TileLayout], stream, gather: bool,
                 host_staging: bool = False):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.scene = scene
        self.stream = stream
        self.gather = gather
        self.host_staging = host_staging  # gloo rehearsal: collectives on host copies
        self.sizes = [(scene.camera(c).width, scene.camera(c).height)
                      for c in range(scene.num_cameras)]
        self.layout = layout_or_none
        dev = torch.device("cuda", torch.cuda.current_device())
        if not gather:
            self.frames = [torch.empty((h, w, 3), dtype=torch.float32, device=dev)
                           for (w, h) in self.sizes]
            return
        L = self.layout
        self.local = torch.zeros((L.padded_tiles, TILE_FLOATS), dtype=torch.float32, device=dev)
        self.rank = L.rank
        if L.rank == 0:
            self.gathered = torch.empty((L.world * L.padded_tiles, TILE_FLOATS),
                                        dtype=torch.float32, device=dev)
            self.gather_list = list(self.gathered.view(L.world, L.padded_tiles, TILE_FLOATS))
            self.index = torch.as_tensor(L.untile_index(), device=dev)
        self.frames = None

    def step(self, events=None):
        s = self.stream.cuda_stream
        if events is not None:
            events[0].record(self.stream)
        if not self.gather:
            for c, f in enumerate(self.frames):
                self.scene.render_device(c, f.data_ptr(), stream=s)
            if events is not None:
                events[1].record(self.stream)
            return self.frames
        for sh in self.layout.shares:
            if sh.count:
                self.scene.render_device(sh.camera, self.local[sh.offset].data_ptr(),
                                         tile_begin=sh.tile_begin, tile_step=sh.tile_step,
                                         tile_major=True, stream=s)
        if events is not None:
            events[1].record(self.stream)
        if self.host_staging:
            torch = self.torch
            self.stream.synchronize()
            host = self.local.cpu()
            glist = list(torch.empty((self.layout.world, self.layout.padded_tiles, TILE_FLOATS))) \
                if self.rank == 0 else None
            self.dist.gather(host, glist, dst=0)
            if self.rank == 0:
                self.gathered.copy_(torch.cat(glist))
        else:
            self.dist.gather(self.local, self.gather_list if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.frames = [f.contiguous() for f in
                           untile(self.gathered, self.layout, self.sizes, self.index)]
        return self.frames


def TilePlan(scene, world: int, rank: int) -> Optional[TileLayout]:
    """Tile layout for every camera of `scene` (None when a single rank renders in place)."""
    if world == 1:
        return None
    tiles = [scene.num_tiles(c) for c in range(scene.num_cameras)]
    return TileLayout(tiles, world, rank)
