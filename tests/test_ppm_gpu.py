"""GPU parity of the photon-mapping path (libceng795_ppm.so) against the CPU oracle
(oracle/ppm_ref, pinned to the reference by tests/test_ppm_oracle.py).

The GPU reorganises the photon pass (per-photon deposits, a stable bucket sort, one lane per
hit point applying its deposits in photon order) but must reproduce the oracle's sequential
single-threaded run bit for bit: hit points, hash grid, every hit point's (flux, r^2, n) and
the final frame."""
import numpy as np
import pytest

import scenes
from oracle.ppm_ref import OraclePPM

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ppm():
    from ceng795_amd import ppm as P
    return P


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("name", list(scenes.PPM) + list(scenes.PPM_DEEP))
def test_eye_pass_and_grid_match_oracle(ppm, scene_dir, name):
    xml = scenes.write_ppm(name, scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=9) as g:
        c = g.camera(0)
        n = g.eye_trace_lines(0)
        o.eye_pass(0, seed=9)
        info = g.build_hash_grid(c.width, c.height)
        oinfo = o.build_hash_grid(c.width, c.height)
        assert n == o.hit_points().shape[0]
        assert np.array_equal(bits(g.hit_points()), bits(o.hit_points()))
        assert np.array_equal(np.float32(info), np.float32(oinfo))


@pytest.mark.parametrize("name", list(scenes.PPM) + list(scenes.PPM_DEEP))
def test_photon_updates_match_oracle(ppm, scene_dir, name):
    xml = scenes.write_ppm(name, scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=4) as g:
        c = g.camera(0)
        g.eye_trace_lines(0)
        g.build_hash_grid(c.width, c.height)
        o.eye_pass(0, seed=4)
        o.build_hash_grid(c.width, c.height)
        g.trace_photons(0, 7000)
        g.trace_photons(7000, 13000)  # ranges compose
        ost = o.trace_photons(4, 0, 20000)
        got, want = g.hit_state(), o.hit_state()
        assert np.array_equal(bits(got), bits(want)), \
            f"{(bits(got) != bits(want)).any(1).sum()} of {len(want)} hit points differ"
        st = g.collect_stats()
        assert st.photons == 20000
        assert st.photon_rays == ost.photon_rays
        assert st.deposits == ost.deposits
        assert st.updates == ost.updates


@pytest.mark.parametrize("threads", [1, 8])
def test_render_matches_oracle(ppm, scene_dir, threads):
    xml = scenes.write_ppm("ppm_box", scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=21) as g:
        img, st = g.render(0, reference_threads=threads)
        want, ost = o.render(0, seed=21, threads=threads)
        assert np.array_equal(bits(img), bits(want))
        assert st.photons == ost.photons
        assert st.hit_points == ost.hit_points
        assert st.eye_rays == ost.eye_rays


def test_errors_are_loud(ppm, scene_dir, tmp_path):
    xml = scenes.write_ppm("ppm_shallow", scene_dir)
    with ppm.PhotonScene(xml) as g:
        with pytest.raises(ppm.RTError):
            g.trace_photons(0, 10)  # before the eye pass / hash grid
        with pytest.raises(ppm.RTError):
            g.eye_trace_lines(5)
    bad = tmp_path / "bad.xml"
    bad.write_text("<Scene><Objects><Sphere><Material>1</Material></Sphere></Objects></Scene>")
    with pytest.raises(ppm.RTError):
        ppm.PhotonScene(str(bad))


@pytest.mark.parametrize("slot_bytes,max_updates", [(1 << 20, 0), (0, 5000), (256 << 10, 3000)])
def test_batched_photon_pass_matches_oracle(ppm, scene_dir, slot_bytes, max_updates):
    """Many batches per ppm_trace_photons call (1 MB / 256 KB of deposit slots: 20k photons
    in ~20-80 batches), and batches split in halves when their (group, deposit) expansion
    exceeds max_updates: the same bits as one batch, since each batch applies its deposits
    in photon order after the previous batch's."""
    xml = scenes.write_ppm("ppm_box", scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=4) as g:
        g.set_batching(slot_bytes, max_updates)
        c = g.camera(0)
        g.eye_trace_lines(0)
        g.build_hash_grid(c.width, c.height)
        o.eye_pass(0, seed=4)
        o.build_hash_grid(c.width, c.height)
        g.trace_photons(0, 20000)
        ost = o.trace_photons(4, 0, 20000)
        assert np.array_equal(bits(g.hit_state()), bits(o.hit_state()))
        st = g.collect_stats()
        assert (st.photons, st.photon_rays, st.deposits, st.updates) == \
            (20000, ost.photon_rays, ost.deposits, ost.updates)


def test_batching_arguments_are_checked(ppm, scene_dir):
    xml = scenes.write_ppm("ppm_shallow", scene_dir)
    with ppm.PhotonScene(xml) as g:
        with pytest.raises(ppm.RTError):
            g.set_batching(-1, 0)
        with pytest.raises(ppm.RTError):
            g.set_batching(0, -5)
        g.set_batching(0, 0)


@pytest.mark.parametrize("name", list(scenes.PPM))
@pytest.mark.parametrize("min_list,seg", [(1, 0), (256, 0), (0, 0), (1, 64), (1, 300)])
def test_update_compaction_matches_oracle(ppm, scene_dir, name, min_list, seg):
    """Tile-list compaction (update-pass phase (0)): tiles whose group list holds >= min_list
    deposits stream a photon-order copy of the deposits their hit points can reach, segment by
    segment (seg deposits each; 64 and 300 split these scenes' lists into many segments, each
    copied with the radii its hit points have at its start); a copy that overflows its scratch
    range (a quarter of the segment) falls back to the segment itself.  Either way the bits are
    the oracle's.  min_list 0 is the uncompacted pass."""
    xml = scenes.write_ppm(name, scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=4) as g:
        g.set_update_compaction(min_list)
        g.set_update_segment(seg)
        g.set_batching(256 << 10, 0)  # several batches: later ones start from shrunken radii
        c = g.camera(0)
        g.eye_trace_lines(0)
        g.build_hash_grid(c.width, c.height)
        o.eye_pass(0, seed=4)
        o.build_hash_grid(c.width, c.height)
        g.trace_photons(0, 20000)
        ost = o.trace_photons(4, 0, 20000)
        got, want = g.hit_state(), o.hit_state()
        assert np.array_equal(bits(got), bits(want)), \
            f"{(bits(got) != bits(want)).any(1).sum()} of {len(want)} hit points differ"
        st = g.collect_stats()
        assert st.updates == ost.updates
        if min_list == 0:
            assert st.update_compacted_segments == st.update_compaction_fallbacks == 0
        if min_list == 1:
            assert st.update_compacted_segments > 0, "no tile took the compacted path"
        with pytest.raises(ppm.RTError):
            g.set_update_compaction(-2)
        with pytest.raises(ppm.RTError):
            g.set_update_segment(8)


# ---------------------------------------------------------------- several GPUs
# The reference shares every hit point between its T threads under a mutex
# (PPM/src/Scene.cpp:131-168); the GPU path shards the update pass by hit point instead.  On
# the one-GPU test box the multi-device scene lists device 0 several times: each replica is a
# complete scene on its own stream, so the shard, gather and merge code is the multi-GPU one.
@pytest.mark.parametrize("name", list(scenes.PPM))
@pytest.mark.parametrize("replicas", [2, 3])
def test_multi_device_scene_matches_oracle(ppm, scene_dir, name, replicas):
    xml = scenes.write_ppm(name, scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=4, devices=[0] * replicas) as g:
        assert g.device_count == replicas
        g.set_batching(256 << 10, 0)  # several batches: each shard keeps its hit points' state
        c = g.camera(0)
        g.eye_trace_lines(0)
        g.build_hash_grid(c.width, c.height)
        o.eye_pass(0, seed=4)
        o.build_hash_grid(c.width, c.height)
        g.trace_photons(0, 7000)
        g.trace_photons(7000, 13000)
        ost = o.trace_photons(4, 0, 20000)
        got, want = g.hit_state(), o.hit_state()
        assert np.array_equal(bits(got), bits(want)), \
            f"{(bits(got) != bits(want)).any(1).sum()} of {len(want)} hit points differ"
        owners = g.hit_point_shards()
        assert owners.min() >= 0 and owners.max() < replicas
        assert len(set(owners.tolist())) == min(replicas, len(owners))  # every shard has work
        st = g.collect_stats()
        assert (st.photons, st.photon_rays, st.deposits, st.updates) == \
            (20000, ost.photon_rays, ost.deposits, ost.updates)


@pytest.mark.parametrize("replicas", [2, 3])
def test_multi_device_render_matches_oracle(ppm, scene_dir, replicas):
    xml = scenes.write_ppm("ppm_box", scene_dir)
    o = OraclePPM(xml)
    with ppm.PhotonScene(xml, seed=21, devices=[0] * replicas) as g:
        img, st = g.render(0, reference_threads=8)
        want, ost = o.render(0, seed=21, threads=8)
        assert np.array_equal(bits(img), bits(want))
        assert (st.photons, st.hit_points, st.eye_rays) == (ost.photons, ost.hit_points, ost.eye_rays)
        assert st.updates == ost.updates
        img2, _ = g.render(0, reference_threads=8)  # again on the same scene: same bits
        assert np.array_equal(bits(img2), bits(want))


@pytest.mark.parametrize("shards", [2, 4])
def test_update_shards_merge_to_oracle(ppm, scene_dir, shards):
    """One process per GPU: S scenes, each applying update shard s of S, merged by hit-point
    owner (ppm.merge_shard_states) and written back for the density estimation."""
    xml = scenes.write_ppm("ppm_box", scene_dir)
    o = OraclePPM(xml)
    states, owners, gs = [], None, []
    try:
        for s in range(shards):
            g = ppm.PhotonScene(xml, seed=21)
            gs.append(g)
            g.set_update_shard(s, shards)
            c = g.camera(0)
            g.eye_trace_lines(0)
            g.build_hash_grid(c.width, c.height)
            g.trace_photons(0, 20000)
            states.append(g.hit_state())
            own = g.hit_point_shards()
            assert owners is None or np.array_equal(own, owners)
            owners = own
        o.eye_pass(0, seed=21)
        o.build_hash_grid(c.width, c.height)
        o.trace_photons(21, 0, 20000)
        merged = ppm.merge_shard_states(states, owners)
        assert np.array_equal(bits(merged), bits(o.hit_state()))
        gs[0].write_hit_state(merged)
        assert np.array_equal(bits(gs[0].hit_state()), bits(merged))
        img = gs[0].density_estimation(20000)
        assert np.array_equal(bits(img), bits(o.density(20000)))
        with pytest.raises(ppm.RTError):
            gs[0].set_update_shard(shards, shards)
    finally:
        for g in gs:
            g.close()


def test_ppm_cli_single_and_multi_device_write_the_same_png(scene_dir, tmp_path):
    """ceng795_amd/bin/ppm_render (the PPM/src/main.cpp driver on the C ABI): the PNG of a
    one-device run and of `--gpus 1` (the multi-device scene with one device) are byte-identical."""
    import os
    import shutil
    import subprocess
    import xml.etree.ElementTree as ET
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "ceng795_amd", "bin", "ppm_render")
    assert os.path.exists(cli), "build the product first (make -C ceng795_amd/csrc)"
    xml = scenes.write_ppm("ppm_box", scene_dir)
    name = ET.parse(xml).getroot().find(".//Camera/ImageName").text.strip()
    png = os.path.splitext(name)[0] + ".png"
    outs = []
    for k, extra in enumerate([[], ["--gpus", "1"]]):
        d = tmp_path / f"run{k}"
        d.mkdir()
        r = subprocess.run([cli, *extra, xml, "8"], cwd=d, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert "Tracing photon rays is completed" in r.stdout
        outs.append((d / png).read_bytes())
    assert outs[0] == outs[1]
    shutil.rmtree(tmp_path, ignore_errors=True)
