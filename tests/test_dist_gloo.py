"""Multi-rank tile sharding + framebuffer gather (ceng795_amd/dist_tiles.py), exercised with
the gloo backend on CPU.  The GPU path (bench.py, FrameRenderer) uses the same TileLayout and
untile(); only the tile renderer differs (here: tiles cut out of known frames)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ceng795_amd.dist_tiles import TILE, TILE_FLOATS, TileLayout, untile

SIZES = [(37, 21), (64, 40), (5, 9), (96, 64)]  # (w, h): ragged edges, tiny frames


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames(seed=7):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal((h, w, 3)).astype(np.float32) for (w, h) in SIZES]


def _tile(frame, t):
    h, w, _ = frame.shape
    tx = (w + TILE - 1) // TILE
    y0, x0 = (t // tx) * TILE, (t % tx) * TILE
    out = np.zeros((TILE, TILE, 3), np.float32)
    blk = frame[y0:y0 + TILE, x0:x0 + TILE]
    out[:blk.shape[0], :blk.shape[1]] = blk
    return out.reshape(-1)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames()
    tiles = [((w + TILE - 1) // TILE) * ((h + TILE - 1) // TILE) for (w, h) in SIZES]
    L = TileLayout(tiles, world, rank)
    local = torch.zeros((L.padded_tiles, TILE_FLOATS))
    for sh in L.shares:  # "render": tiles tile_begin + k*world of each camera
        for k in range(sh.count):
            local[sh.offset + k] = torch.from_numpy(_tile(frames[sh.camera], sh.tile_begin + k * sh.tile_step))
    gathered = torch.empty((world * L.padded_tiles, TILE_FLOATS)) if rank == 0 else None
    dist.gather(local, list(gathered.view(world, L.padded_tiles, TILE_FLOATS)) if rank == 0 else None,
                dst=0)
    if rank == 0:
        out = untile(gathered, L, SIZES)
        ok = all(np.array_equal(o.numpy().view(np.uint32), f.view(np.uint32))
                 for o, f in zip(out, frames))
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_reassembles_frames(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_every_tile_rendered_exactly_once(world):
    tiles = [((w + TILE - 1) // TILE) * ((h + TILE - 1) // TILE) for (w, h) in SIZES]
    seen = np.zeros(sum(tiles), np.int64)
    loads = []
    for r in range(world):
        L = TileLayout(tiles, world, r)
        loads.append(L.local_tiles)
        for sh in L.shares:
            for k in range(sh.count):
                seen[L.offsets[sh.camera] + sh.tile_begin + k * sh.tile_step] += 1
    assert np.all(seen == 1)
    assert max(loads) - min(loads) <= 1  # round-robin: balanced to one tile
    idx = TileLayout(tiles, world, 0).untile_index()
    assert len(np.unique(idx)) == len(idx)
