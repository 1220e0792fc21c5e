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

from ceng795_amd.dist_tiles import (TILE, TILE_FLOATS, TileLayout, chunk_ranges, piece_calls,
                                    untile_camera)

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


def _render_pieces(L, frames, c, pieces):
    """What FrameRenderer's rt_render_device_range calls write into camera c's slot."""
    sh = L.shares[c]
    slot = torch.zeros((sh.slot, TILE_FLOATS))
    for lo, begin, n in piece_calls(sh, pieces):
        for k in range(n):
            slot[lo + k] = torch.from_numpy(_tile(frames[c], begin + k * sh.tile_step))
    return slot


def _split_worker(rank, world, port, outdir, size, chunks):
    """One frame split over the ranks (C4's strong-scaling mode), gathered piece by piece."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    w, h = size
    frames = [rng.standard_normal((h, w, 3)).astype(np.float32)]
    L = TileLayout([size], world, rank)
    sh = L.shares[0]
    pieces = chunk_ranges(sh.slot, chunks)
    slot = _render_pieces(L, frames, 0, pieces)
    gathered = torch.full((world, sh.slot, TILE_FLOATS), float("nan"))
    for lo, hi in pieces:
        outs = [gathered[r, lo:hi] for r in range(world)] if rank == 0 else None
        if rank == 0:
            tmp = [torch.empty(hi - lo, TILE_FLOATS) for _ in range(world)]
            dist.gather(slot[lo:hi].contiguous(), tmp, dst=0)
            for o, t in zip(outs, tmp):
                o.copy_(t)
        else:
            dist.gather(slot[lo:hi].contiguous(), None, dst=0)
    if rank == 0:
        got = untile_camera(gathered.view(-1, TILE_FLOATS), L, 0)
        ok = _same(got.contiguous().numpy(), frames[0])
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,size,chunks", [(2, (3840 // 8, 2160 // 8), 4), (2, (37, 21), 3),
                                               (3, (64, 40), 1), (3, (21, 13), 5)])
def test_single_frame_split_in_pieces(tmp_path, world, size, chunks):
    mp.spawn(_split_worker, args=(world, _free_port(), str(tmp_path), size, chunks),
             nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("slot,chunks", [(0, 4), (1, 4), (7, 3), (8, 4), (130, 4), (5, 1)])
def test_chunk_ranges_cover_slot(slot, chunks):
    pieces = chunk_ranges(slot, chunks)
    covered = [t for lo, hi in pieces for t in range(lo, hi)]
    assert covered == list(range(slot))
    assert len(pieces) <= max(1, chunks)


def test_piece_calls_cover_share():
    for world in (1, 2, 3, 8):
        for size in [(37, 21), (3840 // 8, 2160 // 8)]:
            for r in range(world):
                L = TileLayout([size], world, r)
                sh = L.shares[0]
                tiles = []
                for lo, begin, n in piece_calls(sh, chunk_ranges(sh.slot, 4)):
                    tiles += [begin + k * sh.tile_step for k in range(n)]
                assert tiles == [sh.tile_begin + k * world for k in range(sh.count)]


# --------------------------------------------------------------------------- whole frames per rank
def _frame_worker(rank, world, port, outdir, n_cams):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ceng795_amd.dist_tiles import FrameGatherRenderer, FrameOwners
    w, h = 24, 16
    rng = np.random.default_rng(11)
    truth = [rng.standard_normal((h, w, 3)).astype(np.float32) for _ in range(n_cams)]
    rendered = []

    def render(c, out, stream):  # what rt_render_device writes for camera c
        rendered.append(c)
        out.copy_(torch.from_numpy(truth[c]))

    owners = FrameOwners(n_cams, world, rank)
    R = FrameGatherRenderer(None, owners, [(w, h)] * n_cams, None, host_staging=True,
                            device="cpu", render=render)
    for _ in range(2):  # two steps: buffers reused
        frames = R.step()
    R.finish()
    assert sorted(set(rendered)) == [c for c in range(n_cams) if c % world == rank]
    if rank == 0:
        assert len(frames) == n_cams
        ok = all(_same(frames[c].numpy(), truth[c]) for c in range(n_cams))
        with open(os.path.join(outdir, "frames_ok"), "w") as f:
            f.write("1" if ok else "0")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_cams", [(2, 2), (2, 4), (3, 4)])
def test_whole_frames_per_rank_gather(tmp_path, world, n_cams):
    """Weak-scaling layout: camera c rendered whole by rank c mod world, gathered per round
    (a rank with no camera in the last round sends padding, which rank 0 drops)."""
    mp.spawn(_frame_worker, args=(world, _free_port(), str(tmp_path), n_cams), nprocs=world,
             join=True)
    assert open(os.path.join(tmp_path, "frames_ok")).read() == "1"
