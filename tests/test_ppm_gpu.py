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


@pytest.mark.parametrize("name", list(scenes.PPM))
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


@pytest.mark.parametrize("name", list(scenes.PPM))
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
