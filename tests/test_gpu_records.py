"""The pixel-record exchange of the N>1 tile split (RT_TILE_RECORDS + rt_resolve_device).

Ranks > 0 send, per pixel, one 32-bit record — the DFS leaf of the primary hit and the
shadow-test bits of up to four lights (rt_internal.h kRec*) — instead of 12 bytes of RGB, and
rank 0 shades them (shade_hit, the shading the frame kernel runs, HW2/Scene.cpp:97-139).  The
frame rank 0 assembles this way must be bit-identical to the oracle's, for every deal of the
scene's cameras over `world` ranks: misses, pixels outside a ragged frame, spheres, grazing
hits and multi-camera deals (tile_offset != 0) included."""
import numpy as np
import pytest

import scenes
from conftest import assert_parity
from oracle.cpu_ref import OracleScene

pytestmark = pytest.mark.gpu

NAMES = ["c1", "hf_side", "soup2", "single_sphere", "single_triangle", "graze_plane", "c2",
         "ragged"]


def assembled(s, world, *, root_inplace):
    """Every camera of `s` dealt over `world` ranks, each rank's share rendered as records into
    its slot, then rank 0's frame: its own units in place (root_inplace) or resolved too."""
    import torch
    from ceng795_amd import dist_tiles
    stream = torch.cuda.current_stream().cuda_stream
    L = dist_tiles.TilePlan(s, world, 0)
    frames = []
    for c, sh in enumerate(L.shares):
        gathered = torch.full((world, sh.slot, dist_tiles.TILE_RECORDS), -1.0,
                              dtype=torch.float32, device="cuda")
        for r in range(world):
            sr = L.per_rank[r][c]
            if sr.count:
                s.render_device(c, gathered[r].data_ptr(), tile_begin=sr.tile_begin,
                                tile_step=sr.tile_step, tile_major=True, blocks=True,
                                records=True, stream=stream)
        cam = s.camera(c)
        frame = torch.full((cam.height, cam.width, 3), -1.0, dtype=torch.float32, device="cuda")
        if root_inplace and sh.count:
            s.render_device(c, frame.data_ptr(), tile_begin=sh.tile_begin, tile_step=sh.tile_step,
                            blocks=True, stream=stream)
        s.resolve_device(c, world, sh.slot, gathered.data_ptr(), frame.data_ptr(),
                         tile_offset=int(L.offsets[c] % world), blocks=True,
                         skip_root=root_inplace, stream=stream)
        frames.append(frame)
    torch.cuda.synchronize()
    return [f.cpu().numpy() for f in frames]


@pytest.mark.parametrize("name", NAMES)
def test_record_exchange_matches_oracle(scene_dir, name):
    import ceng795_amd
    xml = scenes.write(name, scene_dir)
    o = OracleScene(xml)
    with ceng795_amd.Scene(xml) as s:
        assert all(s.records_ok(c) for c in range(s.num_cameras))
        refs = [o.render(c, threads=8)[0] for c in range(s.num_cameras)]
        for world in (1, 3, 8):
            for inplace in (False, True):
                got = assembled(s, world, root_inplace=inplace)
                for c, (g, ref) in enumerate(zip(got, refs)):
                    what = f"{name}/cam{c}/world{world}/inplace{inplace}"
                    assert assert_parity(g, ref, what) == 0, what


def test_records_need_direct_shading_and_four_lights(scene_dir):
    """Recursive and multi-sample scenes (their colour is not a function of one hit and its
    shadow bits) refuse records loudly; the bench then exchanges RGB."""
    import torch
    import ceng795_amd
    from ceng795_amd import dist_tiles
    for name in ("soup_depth1", "msaa4"):
        xml = scenes.write(name, scene_dir)
        with ceng795_amd.Scene(xml) as s:
            assert not s.records_ok(0)
            assert not dist_tiles.records_ok(s)
            out = torch.zeros((s.num_tiles(0), 64), dtype=torch.float32, device="cuda")
            with pytest.raises(Exception):
                s.render_device(0, out.data_ptr(), tile_major=True, records=True,
                                stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()


def test_records_are_a_third_of_the_rgb_bytes(scene_dir):
    """What travels: 4 B per pixel (RGB: 12), flagged hit / miss / outside the frame."""
    import torch
    import ceng795_amd
    xml = scenes.write("soup2", scene_dir)
    with ceng795_amd.Scene(xml) as s:
        n = s.num_tiles(0)
        out = torch.zeros((n, 64), dtype=torch.int32, device="cuda")
        s.render_device(0, out.data_ptr(), tile_major=True, records=True,
                        stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        rec = out.cpu().numpy().view(np.uint32)
    flags = rec >> 30
    assert set(np.unique(flags)) <= {0, 1, 2}
    hit = flags == 0
    assert hit.any()
    assert rec.nbytes * 3 == n * 64 * 3 * 4
