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
    """What rt_render_device(tile_major=True[, blocks]) writes: each share at its slot's start,
    zeros for a block's tiles outside the tile grid."""
    local = torch.full((L.buffer_tiles, TILE_FLOATS), float("nan"))
    for sh in L.shares:
        for k, t in enumerate(L.share_tiles(sh.camera, L.rank)):
            local[sh.offset + k] = (torch.from_numpy(_tile(frames[sh.camera], int(t))) if t >= 0
                                    else torch.zeros(TILE_FLOATS))
    return local


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def _worker(rank, world, port, outdir, blocks=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames()
    L = TileLayout(SIZES, world, rank, blocks=blocks)
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


@pytest.mark.parametrize("world,blocks", [(2, True), (3, True), (2, False)])
def test_gather_reassembles_frames(tmp_path, world, blocks):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), blocks), nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("blocks", [True, False])
@pytest.mark.parametrize("world", [1, 2, 5, 8, 13])
def test_untile_single_process(world, blocks):
    """All ranks simulated in one process: gathered slots -> frames, bit for bit."""
    frames = _frames(3)
    layouts = [TileLayout(SIZES, world, r, blocks=blocks) for r in range(world)]
    locals_ = [_render_local(L, frames) for L in layouts]
    for c in range(len(SIZES)):
        sh = layouts[0].shares[c]
        g = torch.stack([loc[sh.offset:sh.offset + sh.slot] for loc in locals_])
        got = untile_camera(g.view(-1, TILE_FLOATS), layouts[0], c)
        assert _same(got.contiguous().numpy(), frames[c])


@pytest.mark.parametrize("blocks", [True, False])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_library_untile_index_math(world, blocks):
    """rt_untile_device (untile_kernel in rt_kernels.hip, deal_block_index in rt_internal.h)
    finds frame tile (tx, ty) of camera c in deal unit u — the tile itself, or block
    d = by*nbx + (bx - by) mod nbx with w = 2*(ty&1) + (tx&1) — at rank
    r = (u + off) mod world, slot tile k = (u - b) / world (times 4, plus w, for blocks),
    b = (r - off) mod world, off = the camera's first global unit: the same tile
    TileLayout.row_index maps, for every camera of a multi-camera layout (restated here in
    numpy; the GPU runs are the bench's gather_verified and the multi-device / 8-way split
    tests)."""
    sizes = [(64, 40), (24, 24), (1920, 1080), (40, 8)]
    L = dist_tiles.TileLayout(sizes, world, 0, blocks=blocks)
    for c, (w, h) in enumerate(sizes):
        tx, ty = dist_tiles.tiles_of((w, h))
        t = np.arange(tx * ty)
        x, y = t % tx, t // tx
        nbx = (tx + 1) >> 1
        if blocks:
            cc = (x >> 1) - (y >> 1) % nbx
            u = (y >> 1) * nbx + np.where(cc < 0, cc + nbx, cc)
            wi = ((y & 1) << 1) | (x & 1)
        else:
            u, wi = t, 0
        off = int(L.offsets[c] % world)
        r = (u + off) % world
        b = ((r - off) % world + world) % world
        k = 4 * ((u - b) // world) + wi if blocks else (u - b) // world
        src = r * L.slots[c] + k
        idx = L.row_index(c)  # [ty*8, tx] tile rows
        want = idx[::dist_tiles.TILE, :].reshape(-1) // dist_tiles.TILE
        assert np.array_equal(src, want), (world, c)


def test_block_deal_order():
    """deal_block_tile / deal_block_index (the kernel's packet_pixel and untile) are inverse
    bijections, and a deal d = r (mod N) takes every block column in turn (diagonal stripes)
    even when the block row length is a multiple of N (C3: 120 blocks, N = 8)."""
    for tx, ty in [(240, 135), (5, 3), (1, 1), (7, 8)]:
        nbx, nby = (tx + 1) // 2, (ty + 1) // 2
        d = np.arange(nbx * nby)
        for w in range(4):
            x, y = dist_tiles.deal_block_tile(tx, d, w)
            d2, w2 = dist_tiles.deal_block_index(tx, x, y)
            assert np.array_equal(d2, d) and np.all(w2 == w)
        x, y = dist_tiles.deal_block_tile(tx, d, 0)
        assert len(set(zip(x.tolist(), y.tolist()))) == len(d)
    x, y = dist_tiles.deal_block_tile(240, np.arange(120 * 68), 0)
    for r in range(8):
        cols = (x[r::8] // 2) % 8
        assert len(set(cols.tolist())) == 8  # not one column class per rank


@pytest.mark.parametrize("blocks", [True, False])
@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_every_tile_rendered_exactly_once(world, blocks):
    L0 = TileLayout(SIZES, world, 0, blocks=blocks)
    seen = [np.zeros(T, np.int64) for T in L0.tiles_per_camera]
    loads = []
    for r in range(world):
        L = TileLayout(SIZES, world, r, blocks=blocks)
        loads.append(sum(sh.count for sh in L.shares))
        assert L.buffer_tiles == L0.buffer_tiles
        for sh in L.shares:
            assert sh.count * L.unit_tiles <= sh.slot and sh.slot == L0.shares[sh.camera].slot
            t = L.share_tiles(sh.camera, r)
            assert len(t) == sh.count * L.unit_tiles
            np.add.at(seen[sh.camera], t[t >= 0], 1)
    assert all(np.all(x == 1) for x in seen)
    assert max(loads) - min(loads) <= 1  # round-robin: balanced to one unit
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

    def render(sh, slot, stream):  # what rt_render_device(tile_major=True, blocks) writes
        frame = truth(state["step"])[sh.camera]
        for k, t in enumerate(L.share_tiles(sh.camera, rank)):
            slot[k] = torch.from_numpy(_tile(frame, int(t))) if t >= 0 else 0.0
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


def _root_inplace_worker(rank, world, port, outdir, sizes, steps, self_exchange=False):
    """The N>1 GPU exchange (TileGatherRenderer with render_inplace): rank 0 renders its own
    units in place into its frames, the other ranks send their slots point-to-point
    (batch_isend_irecv), and rank 0's untile fills everything but its own units."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ceng795_amd.dist_tiles import TileGatherRenderer
    L = TileLayout(sizes, world, rank)
    state = {"step": 0}

    def truth(step):
        return [np.random.default_rng(300 + step).standard_normal((h, w, 3)).astype(np.float32)
                for (w, h) in sizes]

    def render(sh, slot, stream):  # tile-major share (ranks > 0)
        frame = truth(state["step"])[sh.camera]
        for k, t in enumerate(L.share_tiles(sh.camera, rank)):
            slot[k] = torch.from_numpy(_tile(frame, int(t))) if t >= 0 else 0.0

    def render_inplace(sh, out, stream):  # rank 0: its own tiles straight into the frame
        frame = truth(state["step"])[sh.camera]
        h, w, _ = frame.shape
        tx = (w + TILE - 1) // TILE
        for t in L.share_tiles(sh.camera, 0):
            if t < 0:
                continue
            y0, x0 = (t // tx) * TILE, (t % tx) * TILE
            out[y0:y0 + TILE, x0:x0 + TILE] = torch.from_numpy(frame[y0:y0 + TILE, x0:x0 + TILE])

    def untile(c, gathered_c, out, stream, skip_root=False):  # rt_untile_device's contract
        full = untile_camera(gathered_c.view(-1, TILE_FLOATS), L, c)
        h, w, _ = out.shape
        tx = (w + TILE - 1) // TILE
        mine = set(int(t) for t in L.share_tiles(c, 0) if t >= 0) if skip_root else set()
        for t in range(tx * ((h + TILE - 1) // TILE)):
            if t in mine:
                continue
            y0, x0 = (t // tx) * TILE, (t % tx) * TILE
            out[y0:y0 + TILE, x0:x0 + TILE] = full[y0:y0 + TILE, x0:x0 + TILE]

    R = TileGatherRenderer(L, None, render, host_staging=True, device="cpu", untile=untile,
                           render_inplace=render_inplace, cpu_fakes=True,
                           self_exchange=self_exchange)
    assert R.root_inplace and R.self_loop == (self_exchange and world == 1)
    ok = True
    for step in range(steps):
        state["step"] = step
        frames = R.step()
        if rank == 0:
            ok &= all(_same(frames[c].contiguous().numpy(), truth(step)[c])
                      for c in range(len(sizes)))
    R.finish()
    if rank == 0:
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes,self_exchange", [(2, [(64, 40), (37, 21)], False),
                                                       (3, [(96, 64)], False),
                                                       (1, [(40, 24)], False),
                                                       (1, [(40, 24), (17, 9)], True)])
def test_root_inplace_exchange(tmp_path, world, sizes, self_exchange):
    """world 1 with self_exchange: the one-rank rehearsal's self send / receive pair + the
    whole-frame untile (what bench.py --gather-rehearsal runs over RCCL)."""
    mp.spawn(_root_inplace_worker, args=(world, _free_port(), str(tmp_path), sizes, 2,
                                         self_exchange), nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


@pytest.mark.parametrize("world,split", [(2, "bands"), (3, "bands"), (2, "tiles"), (3, "tiles")])
def test_bench_self_launches_ranks(tmp_path, world, split):
    """`python bench.py --gpus N` with no launcher: bench.py starts N ranks itself (before
    any GPU call) and rank 0 prints one JSON line with n_gpus == N; the default N>1 path (row
    bands received into rank 0's frame) and the tile deal (TileGatherRenderer exchange, untile)
    reassemble the frame bit for bit."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world),
                        "--cpu-rehearsal", "--workload", "c2", "--steps", "2", "--warmup", "1",
                        "--split", split],
                       capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert line["config"]["parallelism"] == (f"tiles{world}+gloo_gather" if split == "tiles"
                                             else f"bands{world}+gloo_p2p")
    assert line["config"]["gather_verified"] is True
    if split == "bands":  # cost-balanced cuts of the synthetic cost map: uneven bands
        cuts = line["config"]["band_cuts"]
        assert len(cuts) == world + 1 and cuts[0] == 0 and all(a < b for a, b in zip(cuts, cuts[1:]))


# --------------------------------------------------------------------------- row bands
def _brute_min_max(w, world, wt):
    """The lightest possible heaviest band (cost / weight) over every way to cut w into `world`
    contiguous bands."""
    import itertools
    n = len(w)
    best = float("inf")
    for cuts in itertools.combinations_with_replacement(range(n + 1), world - 1):
        edges = (0,) + cuts + (n,)
        best = min(best, max(_load(sum(w[a:b]), x) for a, b, x in zip(edges, edges[1:], wt)))
    return best


def _load(cost, weight):
    return cost / weight if weight > 0 else (float("inf") if cost > 0 else 0.0)


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_band_cuts_minimise_the_heaviest_band(seed, world, weighted):
    rng = np.random.default_rng(seed)
    w = rng.integers(1, 50, size=int(rng.integers(1, 9))).astype(float)
    wt = ([float(rng.choice([0.0, 0.3, 0.6]))] + [1.0] * (world - 1)) if weighted else [1.0] * world
    if world == 1:
        wt = [1.0]
    cuts = dist_tiles.band_cuts(w, world, wt if weighted else None)
    assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == len(w)
    assert all(a <= b for a, b in zip(cuts, cuts[1:]))
    heaviest = max(_load(w[a:b].sum(), x) for a, b, x in zip(cuts, cuts[1:], wt))
    assert heaviest <= _brute_min_max(list(w), world, wt) * (1 + 1e-9)


def test_root_band_weights():
    """Rank 0's band shrinks by its resolve of the others' records: with rho the resolve of a
    whole frame over its render, every rank's time (in frames) is (1 + rho (N-1)/N) / N."""
    assert dist_tiles.root_band_weights(1, 0.3) == [1.0]
    for n, rho in [(2, 0.0), (8, 0.08), (4, 0.5), (8, 5.0)]:
        wt = dist_tiles.root_band_weights(n, rho)
        T = (1 + rho * (n - 1) / n) / n
        assert len(wt) == n and wt[1:] == [1.0] * (n - 1)
        assert wt[0] == pytest.approx(max(0.0, T - rho * (n - 1) / n) / T)


def test_band_plan_covers_every_row_once():
    costs = [np.random.default_rng(c).random(dist_tiles.tiles_of(s)[0] * dist_tiles.tiles_of(s)[1])
             for c, s in enumerate(SIZES)]
    for world in (1, 2, 3, 8):
        P = dist_tiles.BandPlan.from_costs(SIZES, world, 0, costs)
        for c, (w, h) in enumerate(SIZES):
            rows = np.zeros(h, int)
            for r in range(world):
                b = P.per_rank[r][c]
                assert b.tile_begin == b.row0 * b.tiles_x and b.tile_count == b.rows * b.tiles_x
                rows[b.y0:b.y1] += 1
            assert (rows == 1).all()
        assert np.isclose(P.band_costs(costs).sum(), sum(x.sum() for x in costs))


def _band_worker(rank, world, port, outdir, sizes, steps, self_exchange=False, records=False):
    """The band split's exchange (BandGatherRenderer): each rank writes its bands into its own
    frames (in place, as rt_render_device_range does), the other ranks' bands land in rank 0's
    frames; uneven bands from a random cost map."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ceng795_amd.dist_tiles import BandGatherRenderer, BandPlan, tiles_of
    costs = [np.random.default_rng(40 + c).random(tiles_of(s)[0] * tiles_of(s)[1]) ** 4
             for c, s in enumerate(sizes)]
    P = BandPlan.from_costs(sizes, world, rank, costs)
    state = {"step": 0, "rows": 0}

    def truth(step):
        return [np.random.default_rng(500 + step).standard_normal((h, w, 3)).astype(np.float32)
                for (w, h) in sizes]

    def render(b, frame, stream):
        state["rows"] += b.y1 - b.y0
        frame[b.y0:b.y1] = torch.from_numpy(truth(state["step"])[b.camera][b.y0:b.y1])

    def render_records(b, rec, stream):  # a "record" = the pixel's index in the frame
        state["rows"] += b.y1 - b.y0
        h, w = rec.shape
        rec[b.y0:b.y1] = torch.arange(b.y0 * w, b.y1 * w, dtype=torch.int32).view(-1, w)

    def resolve(c, y0, y1, rec, frame, stream):  # ... shaded = looked up in this step's truth
        flat = torch.from_numpy(truth(state["step"])[c]).view(-1, 3)
        frame[y0:y1] = flat[rec[y0:y1].reshape(-1).long()].view(y1 - y0, -1, 3)

    R = BandGatherRenderer(P, None, render, host_staging=True, device="cpu",
                           self_exchange=self_exchange,
                           render_records=render_records if records else None,
                           resolve=resolve if records else None)
    assert R.records == records
    ok = True
    for step in range(steps):
        state["step"] = step
        frames = R.step()
        if rank == 0:
            ok &= all(_same(frames[c].numpy(), truth(step)[c]) for c in range(len(sizes)))
    R.finish()
    ok &= state["rows"] == steps * sum(b.y1 - b.y0 for b in P.bands)
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        with open(os.path.join(outdir, "result"), "w") as fh:
            fh.write("ok" if flag.item() else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("records", [False, True])
@pytest.mark.parametrize("world,sizes,self_exchange", [(2, [(64, 40), (37, 21)], False),
                                                       (3, [(96, 64)], False),
                                                       (3, [(5, 9)], False),
                                                       (1, [(40, 24), (17, 9)], True)])
def test_band_exchange(tmp_path, world, sizes, self_exchange, records):
    """world 3 on a one-tile-row frame: two ranks get empty bands and send nothing.  records:
    the bands travel as pixel records that rank 0 resolves (every band but its own)."""
    mp.spawn(_band_worker, args=(world, _free_port(), str(tmp_path), sizes, 2, self_exchange,
                                 records), nprocs=world, join=True)
    assert (tmp_path / "result").read_text() == "ok"


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
