"""Pin the CPU oracle (oracle/cpu_ref) to the reference: every golden frame in tests/golden/
was produced by the reference itself (tests/golden/make_golden.py); the oracle must reproduce
each one bit for bit.  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

import scenes
from oracle.cpu_ref import OracleScene

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
ARRAYS = np.load(os.path.join(HERE, "golden", "golden.npz"))  # allow_pickle=False default
THREADS = min(8, os.cpu_count() or 1)

NAMES = [n for n in GOLDEN if not n.startswith("_")]


def scene_xml(name, directory):
    return scenes.write_c3(directory) if name == "c3" else scenes.write(name, directory)


@pytest.mark.parametrize("name", NAMES)
def test_scene_text_matches_golden(scene_dir, name):
    """The generator still produces the exact XML the fixture was made from."""
    xml = scene_xml(name, scene_dir)
    assert hashlib.sha256(open(xml, "rb").read()).hexdigest() == GOLDEN[name]["xml_sha256"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_reference_frames(scene_dir, name):
    xml = scene_xml(name, scene_dir)
    o = OracleScene(xml)
    g = GOLDEN[name]
    assert o.num_cameras == len(g["cameras"])
    for cam, gc in enumerate(g["cameras"]):
        img, st = o.render(cam, threads=THREADS)
        assert img.shape == (gc["height"], gc["width"], 3)
        key = f"{name}__{cam}"
        ys, xs = ARRAYS[key + "__ys"], ARRAYS[key + "__xs"]
        assert np.array_equal(img[ys, xs].view(np.uint32), ARRAYS[key + "__samples"].view(np.uint32))
        y0, x0 = gc["crop_origin"]
        crop = ARRAYS[key + "__crop"]
        assert np.array_equal(img[y0:y0 + crop.shape[0], x0:x0 + crop.shape[1]].view(np.uint32),
                              crop.view(np.uint32))
        assert hashlib.sha256(img.tobytes()).hexdigest() == gc["frame_sha256"], f"{name}/cam{cam}"
        if name not in scenes.RECURSIVE:  # the harness counts depth-0 rays only
            assert st.primary_rays + st.shadow_rays == gc["rays"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_bvh_topology_matches_reference(scene_dir, tmp_path, name):
    xml = scene_xml(name, scene_dir)
    o = OracleScene(xml)
    out = tmp_path / "bvh.txt"
    o.dump_bvh(str(out))
    lines = [l for l in out.read_text().splitlines() if l != "M"]
    text = "\n".join(lines) + "\n"
    assert hashlib.sha256(text.encode()).hexdigest() == GOLDEN[name]["bvh_sha256"]


def test_reference_order_visit_counts_c3(scene_dir):
    """SURVEY §3.2's per-ray visit counts on C3 (they price roofline.achieved)."""
    o = OracleScene(scenes.write_c3(scene_dir))
    _, st = o.render(0, threads=THREADS)
    s = st.as_dict()
    assert abs(s["box_tests"][0] / s["primary_rays"] - 146.0) < 0.2
    assert abs(s["prim_tests"][0] / s["primary_rays"] - 9.6) < 0.1
    assert abs(s["box_tests"][1] / s["shadow_rays"] - 99.5) < 0.2
    assert abs(s["prim_tests"][1] / s["shadow_rays"] - 5.9) < 0.1
