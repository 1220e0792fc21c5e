"""Multi-rank tile sharding + framebuffer gather (ceng795_amd/dist_tiles.py), exercised with
the gloo backend on CPU.  The GPU path (bench.py, FrameRenderer) uses the same TileLayout,
per-camera slots and untile_camera(); only the tile renderer differs (here: tiles cut out of
known frames) and the collective runs on host tensors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ceng795_amd.dist_tiles import TILE, TILE_FLOATS, TileLayout, untile_camera

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


def _render_local(L, frames):
    """What rt_render_device(tile_major=True) writes: each share at its slot's start."""
    local = torch.full((L.buffer_tiles, TILE_FLOATS), float("nan"))
    for sh in L.shares:
        for k in range(sh.count):
            local[sh.offset + k] = torch.from_numpy(
                _tile(frames[sh.camera], sh.tile_begin + k * sh.tile_step))
    return local


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames()
    L = TileLayout(SIZES, world, rank)
    local = _render_local(L, frames)
    ok = True
    for c, sh in enumerate(L.shares):  # one equal-size gather per camera slot
        glist = list(torch.empty((world, sh.slot, TILE_FLOATS))) if rank == 0 else None
        dist.gather(local[sh.offset:sh.offset + sh.slot].contiguous(), glist, dst=0)
        if rank == 0:
            got = untile_camera(torch.stack(glist).view(-1, TILE_FLOATS), L, c)
            ok &= _same(got.contiguous().numpy(), frames[c])
    if rank == 0:
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_reassembles_frames(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("world", [1, 2, 5, 8, 13])
def test_untile_single_process(world):
    """All ranks simulated in one process: gathered slots -> frames, bit for bit."""
    frames = _frames(3)
    layouts = [TileLayout(SIZES, world, r) for r in range(world)]
    locals_ = [_render_local(L, frames) for L in layouts]
    for c in range(len(SIZES)):
        sh = layouts[0].shares[c]
        g = torch.stack([loc[sh.offset:sh.offset + sh.slot] for loc in locals_])
        got = untile_camera(g.view(-1, TILE_FLOATS), layouts[0], c)
        assert _same(got.contiguous().numpy(), frames[c])


@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_every_tile_rendered_exactly_once(world):
    L0 = TileLayout(SIZES, world, 0)
    seen = np.zeros(L0.total, np.int64)
    loads = []
    for r in range(world):
        L = TileLayout(SIZES, world, r)
        loads.append(L.local_tiles)
        assert L.buffer_tiles == L0.buffer_tiles
        for sh in L.shares:
            assert sh.count <= sh.slot and sh.slot == L0.shares[sh.camera].slot
            for k in range(sh.count):
                seen[L.offsets[sh.camera] + sh.tile_begin + k * sh.tile_step] += 1
    assert np.all(seen == 1)
    assert max(loads) - min(loads) <= 1  # round-robin: balanced to one tile
    for c in range(len(SIZES)):  # the untile reads every tile row of camera c exactly once
        idx = L0.row_index(c).reshape(-1)
        assert len(np.unique(idx)) == len(idx)
        assert idx.max() < world * L0.slots[c] * TILE
