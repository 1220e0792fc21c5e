"""Multi-rank tile sharding + framebuffer gather (ceng795_amd/dist_tiles.py), exercised with
the gloo backend on CPU.  The GPU path (bench.py, TileGatherRenderer) uses the same
TileLayout, per-camera slots and untile_camera(); only the tile renderer differs (here: tiles
cut out of known frames) and the collective runs on host tensors.  The last tests run bench.py
itself: `--gpus N` without a launcher starts N ranks, and `--cpu-rehearsal` drives the default
N>1 path (tile deal, pipelined gather, untile, check) with synthetic tiles."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ceng795_amd import dist_tiles
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


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_library_untile_index_math(world):
    """rt_untile_device (untile_kernel in rt_kernels.hip) finds frame tile t of camera c at
    rank r = (t + off) mod world, slot position (t - b) / world with b = (r - off) mod world
    (off = the camera's first global tile): the same tile TileLayout.row_index maps, for every
    camera of a multi-camera layout (restated here in numpy; the GPU runs are the bench's
    gather_verified and test_c4_eight_way_tile_split_matches_oracle)."""
    sizes = [(64, 40), (24, 24), (1920, 1080)]
    L = dist_tiles.TileLayout(sizes, world, 0)
    for c, (w, h) in enumerate(sizes):
        tx, ty = dist_tiles.tiles_of((w, h))
        t = np.arange(tx * ty)
        off = int(L.offsets[c] % world)
        r = (t + off) % world
        b = ((r - off) % world + world) % world
        src = r * L.slots[c] + (t - b) // world
        idx = L.row_index(c)  # [ty*8, tx] tile rows
        want = idx[::dist_tiles.TILE, :].reshape(-1) // dist_tiles.TILE
        assert np.array_equal(src, want), (world, c)


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


def _pipeline_worker(rank, world, port, outdir, sizes, steps):
    """TileGatherRenderer over gloo: several cameras per step, several steps (buffers reused);
    every rank renders exactly its tiles, and rank 0's frames equal the truth each step."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ceng795_amd.dist_tiles import TileGatherRenderer
    L = TileLayout(sizes, world, rank)
    done = []

    def truth(step):
        return _frames(100 + step)[:len(sizes)] if sizes == SIZES else \
            [np.random.default_rng(100 + step).standard_normal((h, w, 3)).astype(np.float32)
             for (w, h) in sizes]

    state = {"step": 0}

    def render(sh, slot, stream):  # what rt_render_device(tile_major=True) writes
        frame = truth(state["step"])[sh.camera]
        for k in range(sh.count):
            slot[k] = torch.from_numpy(_tile(frame, sh.tile_begin + k * sh.tile_step))
        done.append((sh.camera, sh.count))

    R = TileGatherRenderer(L, None, render, host_staging=True, device="cpu")
    ok = True
    for step in range(steps):
        state["step"] = step
        frames = R.step()
        if rank == 0:
            ok &= all(_same(frames[c].contiguous().numpy(), truth(step)[c])
                      for c in range(len(sizes)))
    R.finish()
    assert sorted(done) == sorted([(sh.camera, sh.count) for sh in L.shares if sh.count] * steps)
    if rank == 0:
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes,steps", [(2, [(1920 // 8, 1080 // 8)], 3),
                                               (3, SIZES, 2), (2, [(5, 9)], 2)])
def test_tile_gather_renderer_pipeline(tmp_path, world, sizes, steps):
    mp.spawn(_pipeline_worker, args=(world, _free_port(), str(tmp_path), sizes, steps),
             nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("world", [2, 3])
def test_bench_self_launches_ranks(tmp_path, world):
    """`python bench.py --gpus N` with no launcher: bench.py starts N ranks itself (before
    any GPU call) and rank 0 prints one JSON line with n_gpus == N; the default N>1 path (tile
    deal, TileGatherRenderer exchange, untile) reassembles the frame bit for bit."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world),
                        "--cpu-rehearsal", "--workload", "c2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert line["config"]["parallelism"] == f"tiles{world}+gloo_gather"
    assert line["config"]["gather_verified"] is True


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


def _ppm_merge_worker(rank, world, port, out_dir):
    """gather_merged_state over gloo: rank r's state holds r+1 in the rows it owns and garbage
    elsewhere; rank 0 must get every row from its owner."""
    import numpy as np
    import torch.distributed as dist
    from ceng795_amd.dist_ppm import gather_merged_state
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1001
    owners = (np.arange(n) * 7 % world).astype(np.int32)
    state = np.full((n, 5), -1.0, np.float32)
    state[owners == rank] = rank + 1
    got = gather_merged_state(state, owners)
    if rank == 0:
        assert got.shape == (n, 5)
        assert np.array_equal(got[:, 0], owners + 1.0)
        np.save(os.path.join(out_dir, "merged.npy"), got)
    else:
        assert got is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ppm_shard_state_gather(tmp_path, world):
    mp.spawn(_ppm_merge_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / "merged.npy").exists()


def test_ppm_photon_budget_matches_reference_rule():
    from ceng795_amd.dist_ppm import photons_and_normaliser
    assert photons_and_normaliser(10000, 1000, 256, 8) == (10_000_000, 10000 * 1250 * 8)
    assert photons_and_normaliser(10000, 1000, 256, 3) == (3333 * 1000 * 3, 10000 * 3333 * 3)
    assert photons_and_normaliser(100, 10, 2, 8) == (1000, 100 * 12 * 8)  # height < T
