"""The band split of the N>1 bench (dist_tiles.BandPlan / BandGatherRenderer) on the GPU.

rt_tile_costs returns the measured per-tile cost map of the last frame on a stream; the bands
are cut from it; every rank's band is a tile range of rt_render_device_range rendered in place
into the row-major frame (HW2/main.cpp:33-36 splits the frame over threads by rows too).  The
frame assembled from the bands must be bit-identical to the oracle's for any cut."""
import numpy as np
import pytest

import scenes
from conftest import assert_parity
from oracle.cpu_ref import OracleScene

pytestmark = pytest.mark.gpu


def test_tile_costs_of_a_whole_frame(scene_dir):
    import torch
    import ceng795_amd
    xml = scenes.write("hf_side", scene_dir)
    with ceng795_amd.Scene(xml) as s:
        st = torch.cuda.Stream()
        cam = s.camera(0)
        n = s.num_tiles(0)
        with pytest.raises(Exception):  # nothing rendered on this stream yet
            s.tile_costs(st.cuda_stream, n)
        buf = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
        for _ in range(3):  # cold, then warm-ordered frames (split tiles: quadrant sums)
            s.render_device(0, buf.data_ptr(), stream=st.cuda_stream)
            c = s.tile_costs(st.cuda_stream, n)
            assert c.shape == (n,) and (c > 0).all()
        with pytest.raises(Exception):  # capacity below the frame's tiles
            s.tile_costs(st.cuda_stream, n - 1)
        s.release_stream(st.cuda_stream)


@pytest.mark.parametrize("name", ["c1", "hf_side", "soup2", "single_sphere", "c2", "ragged"])
def test_bands_assemble_the_oracle_frame(scene_dir, name):
    import torch
    import ceng795_amd
    from ceng795_amd import dist_tiles
    xml = scenes.write(name, scene_dir)
    o = OracleScene(xml)
    with ceng795_amd.Scene(xml) as s:
        refs = [o.render(c, threads=8)[0] for c in range(s.num_cameras)]
        costs = dist_tiles.measure_tile_costs(s, frames=2)
        render = dist_tiles.scene_band_renderer(s)
        st = torch.cuda.current_stream()
        for world in (1, 2, 3, 8):
            plan = dist_tiles.BandRenderPlan(s, world, 0, dist_tiles.BandPlan.from_costs(
                plan_sizes(s), world, 0, costs).cuts)
            for c, ref in enumerate(refs):
                frame = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
                for r in range(world):
                    b = plan.per_rank[r][c]
                    if b.rows:
                        render(b, frame, st)
                torch.cuda.synchronize()
                what = f"{name}/cam{c}/world{world}"
                assert assert_parity(frame.cpu().numpy(), ref, what) == 0, what


def plan_sizes(s):
    return [(s.camera(c).width, s.camera(c).height) for c in range(s.num_cameras)]


def test_c3_band_costs_balance(scene_dir):
    """On C3 the cost-balanced cuts give eight bands within a tile row's cost of each other —
    the balance the bench's N=8 split is built on."""
    import ceng795_amd
    from ceng795_amd import dist_tiles
    xml = scenes.write_c3(scene_dir)
    with ceng795_amd.Scene(xml) as s:
        costs = dist_tiles.measure_tile_costs(s, frames=3)
    sizes = [(1920, 1080)]
    plan = dist_tiles.BandPlan.from_costs(sizes, 8, 0, costs)
    bc = plan.band_costs(costs)
    rows = costs[0].reshape(135, 240).sum(1)
    assert bc.max() - bc.min() <= 2 * rows.max()
    assert bc.max() / bc.mean() < 1.05


@pytest.mark.parametrize("name", ["c1", "soup2", "single_sphere", "graze_plane", "c2", "ragged"])
def test_record_bands_assemble_the_oracle_frame(scene_dir, name):
    """Bands as row-major pixel records (RT_TILE_RECORDS without RT_TILE_MAJOR) from ranks > 0,
    rank 0's (smaller) band in place as RGB, then rt_resolve_rows over every other row: the
    oracle's frame bit for bit."""
    import torch
    import ceng795_amd
    from ceng795_amd import dist_tiles
    xml = scenes.write(name, scene_dir)
    o = OracleScene(xml)
    with ceng795_amd.Scene(xml) as s:
        assert dist_tiles.records_ok(s)
        refs = [o.render(c, threads=8)[0] for c in range(s.num_cameras)]
        costs = dist_tiles.measure_tile_costs(s, frames=2)
        rho = dist_tiles.measure_resolve_frac(s, frames=2)
        assert 0.0 < rho < 5.0
        rgb = dist_tiles.scene_band_renderer(s)
        rec_render = dist_tiles.scene_band_renderer(s, records=True)
        resolve = dist_tiles.scene_row_resolver(s)
        st = torch.cuda.current_stream()
        for world in (1, 2, 3, 8):
            plan = dist_tiles.BandPlan.from_costs(plan_sizes(s), world, 0, costs,
                                                  dist_tiles.root_band_weights(world, rho))
            for c, ref in enumerate(refs):
                h, w, _ = ref.shape
                frame = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
                recs = torch.full((h, w), -1, dtype=torch.int32, device="cuda")
                own = plan.per_rank[0][c]
                if own.rows:
                    rgb(own, frame, st)
                for r in range(1, world):
                    b = plan.per_rank[r][c]
                    if b.rows:
                        rec_render(b, recs, st)
                for y0, y1 in ((0, own.y0), (own.y1, h)):
                    if y1 > y0:
                        resolve(c, y0, y1, recs, frame, st)
                torch.cuda.synchronize()
                what = f"{name}/cam{c}/world{world}"
                assert assert_parity(frame.cpu().numpy(), ref, what) == 0, what
                if world == 1:  # and a whole frame of records alone
                    full = dist_tiles.BandPlan(plan_sizes(s), 1, 0).bands[c]
                    rec_render(full, recs, st)
                    resolve(c, 0, h, recs, frame, st)
                    torch.cuda.synchronize()
                    assert assert_parity(frame.cpu().numpy(), ref, what + "/all") == 0
