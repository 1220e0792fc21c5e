"""Host-side logic of the product library, CPU only (no HIP call is made):
the C-ABI exports, the XML ingest + reference-identical BVH build + flattening (checked
against the reference's own topology hashes in tests/golden/), the camera precompute, the PNG
writer and the loader's error behaviour."""
import ctypes as C
import hashlib
import json
import os
import re
import struct
import sys
import zlib

import numpy as np
import pytest

import scenes
from ceng795_amd import _lib
from ceng795_amd.scene import host_dump_bvh, write_png
from oracle.cpu_ref import OracleScene

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
HEADER = os.path.join(ROOT, "include", "ceng795_rt.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\s*\*)\s*(rt_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_function():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes table"
    assert L.rt_abi_version() == _lib.ABI_VERSION == 7


def test_oracle_is_not_linked_into_the_product():
    """The product must not route through the CPU oracle: no cpuref_* symbol, no libcpu_ref."""
    path = _lib.LIB_PATH
    data = open(path, "rb").read()
    assert b"cpuref_" not in data and b"libcpu_ref" not in data


@pytest.mark.parametrize("name", [n for n in GOLDEN if not n.startswith("_")])
def test_bvh_topology_matches_reference(scene_dir, tmp_path, name):
    """XML ingest + BVH build + DFS flattening reproduce the reference's tree exactly
    (boxes as fp32 bits, leaf order, vertex ids, materials)."""
    xml = scenes.write_c3(scene_dir) if name == "c3" else scenes.write(name, scene_dir)
    out = tmp_path / "bvh.txt"
    host_dump_bvh(xml, str(out))
    assert hashlib.sha256(out.read_bytes()).hexdigest() == GOLDEN[name]["bvh_sha256"]


def primary_dirs(cam: _lib.rt_camera, w: int, h: int) -> np.ndarray:
    """Camera::calculate_ray_at (HW2/Camera.h:30-35) replayed in numpy fp32 (one rounding
    per operation, like the reference's SSE code)."""
    f32 = np.float32
    tl, su, sv, e = (np.array(list(v), f32) for v in (cam.top_left, cam.s_u, cam.s_v, cam.e))
    xs = np.arange(w, dtype=f32) + f32(0.5)
    ys = np.arange(h, dtype=f32) + f32(0.5)
    s = (tl[None, None, :] + su[None, None, :] * xs[None, :, None]) - sv[None, None, :] * ys[:, None, None]
    v = s - e
    ln = np.sqrt((v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1]) + v[..., 2] * v[..., 2])
    return v / ln[..., None]


@pytest.mark.parametrize("name", ["c1", "hf_small", "hf_side", "soup1", "single_sphere"])
def test_camera_precompute_matches_reference(scene_dir, name):
    spec = scenes.CATALOGUE[name][0]()
    xml = scenes.write(name, scene_dir)
    o = OracleScene(xml)
    for k, c in enumerate(spec.cameras):
        cam = _lib.rt_camera()
        f3 = lambda v: (C.c_float * 3)(*[np.float32(x) for x in v])
        np4 = (C.c_float * 4)(*[np.float32(x) for x in c.near_plane])
        _lib.check(_lib.lib().rt_camera_from_view(f3(c.position), f3(c.gaze), f3(c.up), np4,
                                                  np.float32(c.near_distance), c.width,
                                                  c.height, 1, C.byref(cam)))
        d = primary_dirs(cam, c.width, c.height)
        ref = o.primary_records(k)[..., :3]
        assert np.array_equal(d.view(np.uint32), ref.view(np.uint32)), (name, k)


def png_parts(path):
    """(IHDR fields, PLTE bytes, inflated IDAT bytes, other chunk types), CRCs checked."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, plte, hdr, other = 8, b"", b"", None, []
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        assert struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0] == zlib.crc32(typ + body)
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"PLTE":
            plte += body
        elif typ == b"IDAT":
            idat += body
        elif typ != b"IEND":
            other.append(typ)
        pos += 12 + n
    return hdr, plte, zlib.decompress(idat), other


def decode_png_rgb(path):
    """A minimal PNG decoder (colour types 0, 2, 3; bit depths 1-8; filters 0-4) -> RGB8."""
    (w, h, depth, ctype, _, _, interlace), plte, raw, _ = png_parts(path)
    assert interlace == 0 and ctype in (0, 2, 3)
    bpp = depth * (3 if ctype == 2 else 1)
    line, bw = (w * bpp + 7) // 8, max(1, bpp // 8)
    prev = bytearray(line)
    out = []
    for r in range(h):
        f = raw[r * (line + 1)]
        cur = bytearray(raw[r * (line + 1) + 1:(r + 1) * (line + 1)])
        for i in range(line):
            a = cur[i - bw] if i >= bw else 0
            b, c = prev[i], (prev[i - bw] if i >= bw else 0)
            if f == 1:
                cur[i] = (cur[i] + a) & 255
            elif f == 2:
                cur[i] = (cur[i] + b) & 255
            elif f == 3:
                cur[i] = (cur[i] + ((a + b) >> 1)) & 255
            elif f == 4:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                cur[i] = (cur[i] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))) & 255
        out.append(bytes(cur))
        prev = cur
    px = np.zeros((h, w, 3), np.uint8)
    for r, row in enumerate(out):
        if ctype == 2:
            px[r] = np.frombuffer(row, np.uint8)[:3 * w].reshape(w, 3)
            continue
        bits = np.unpackbits(np.frombuffer(row, np.uint8))[:w * depth].reshape(w, depth)
        v = bits.dot(1 << np.arange(depth - 1, -1, -1))
        if ctype == 0:
            px[r] = (v * (255 // ((1 << depth) - 1)))[:, None]
        else:
            pal = np.frombuffer(plte, np.uint8).reshape(-1, 3)
            px[r] = pal[v]
    return px


def test_png_quantisation_like_pixel_get_color(tmp_path):
    """HW2/Pixel.h:17-28 + main.cpp:43-54: clamp(int(c), 0, 255), truncation, NaN -> 0."""
    vals = np.array([0.0, 0.99, 1.0, 254.99, 255.0, 300.0, -0.5, -3.0, np.nan, np.inf, -np.inf,
                     127.5], np.float32)
    img = np.tile(vals, (2, 1)).reshape(2, 4, 3)
    path = tmp_path / "q.png"
    write_png(str(path), img)
    got = decode_png_rgb(str(path))
    exp = np.array([0, 0, 1, 254, 255, 255, 0, 0, 0, 0, 0, 127], np.uint8)
    assert np.array_equal(got.reshape(2, -1)[0], exp)


@pytest.mark.parametrize("name", ["c1", "soup1", "hf_small", "hf_side", "single_sphere"])
def test_png_matches_the_reference_file(scene_dir, tmp_path, name):
    """rt_write_png against the PNG the reference itself wrote (HW2/main.cpp:43-57 through its
    lodepng 20180114, tests/golden/png, make_golden_png.py) for the same frame: the colour type
    and bit depth lodepng chose (RGB, grey and palette cases), the palette in its order, and the
    filtered image data are byte-identical; the files differ only in the deflate stream
    carrying that data (zlib here), so both decode to the same pixels."""
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "png", "golden_png.json")))[name]
    xml = scenes.write(name, scene_dir)
    assert hashlib.sha256(open(xml, "rb").read()).hexdigest() == meta["xml_sha256"]
    ref_png = os.path.join(ROOT, "tests", "golden", "png", f"{name}_cam0.png")
    assert hashlib.sha256(open(ref_png, "rb").read()).hexdigest() == meta["png_sha256"]
    from oracle.cpu_ref import OracleScene
    img, _ = OracleScene(xml).render(0, threads=4)  # = the reference's Pixel::color, bit for bit
    ours = tmp_path / "ours.png"
    write_png(str(ours), img)
    a, b = png_parts(ref_png), png_parts(str(ours))
    assert a[0] == b[0], (a[0], b[0])  # width, height, bit depth, colour type, ...
    assert a[1] == b[1]                # palette
    assert a[2] == b[2]                # filter bytes + filtered scanlines
    assert a[3] == b[3] == []
    assert np.array_equal(decode_png_rgb(ref_png), decode_png_rgb(str(ours)))


# ---------------------------------------------------------------- loader error behaviour
def _variant(scene_dir, tmp_path, transform, base="soup1"):
    text = open(scenes.write(base, scene_dir)).read()
    p = tmp_path / "v.xml"
    p.write_text(transform(text))
    return str(p)


def _dump_rc(xml, tmp_path):
    return _lib.lib().rt_host_dump_bvh_xml(xml.encode(), str(tmp_path / "o.txt").encode())


@pytest.mark.parametrize("prolog", ['<?xml version="1.0"?>\n', "<!-- scene -->\n",
                                    "  \n<!DOCTYPE Scene>\n"])
def test_xml_prolog_is_refused_like_the_reference(scene_dir, tmp_path, prolog):
    """The reference takes file.FirstChild() as root (HW2/Scene.cpp:206): a prolog node becomes
    the root and the load fails (a crash there, RT_E_PARSE here); comments
    INSIDE the scene element are fine, and leading whitespace is no node."""
    v = _variant(scene_dir, tmp_path, lambda t: prolog + t)
    assert _dump_rc(v, tmp_path) == _lib.RT_E_PARSE
    assert "FirstChild" in _lib.lib().rt_last_error().decode()
    plain = scenes.write("soup1", scene_dir)
    host_dump_bvh(plain, str(tmp_path / "a.txt"))
    inner = _variant(scene_dir, tmp_path,
                     lambda t: "\n  " + t.replace("<Objects>", "<Objects><!-- objects -->"))
    host_dump_bvh(inner, str(tmp_path / "b.txt"))
    assert (tmp_path / "a.txt").read_text() == (tmp_path / "b.txt").read_text()


@pytest.mark.parametrize("mutate,code", [
    (lambda t: t.replace("<Cameras>", "<CamerasX>").replace("</Cameras>", "</CamerasX>"),
     _lib.RT_E_PARSE),
    (lambda t: t.replace("</Scene>", ""), _lib.RT_E_PARSE),
    (lambda t: re.sub(r"<Faces>.*?</Faces>", "<Faces> </Faces>", t, count=1, flags=re.S),
     _lib.RT_E_INVALID),
    (lambda t: re.sub(r"<Material>1</Material>", "<Material>99</Material>", t, count=1),
     _lib.RT_E_INVALID),
    (lambda t: re.sub(r"<Indices>\d+", "<Indices>999999", t, count=1), _lib.RT_E_INVALID),
    (lambda t: re.sub(r"<Objects>.*</Objects>", "<Objects></Objects>", t, flags=re.S),
     _lib.RT_E_INVALID),
])
def test_loader_errors(scene_dir, tmp_path, mutate, code):
    rc = _dump_rc(_variant(scene_dir, tmp_path, mutate), tmp_path)
    assert rc == code, (rc, _lib.lib().rt_last_error())
    assert _lib.lib().rt_last_error()


def test_missing_file_is_io_error(tmp_path):
    assert _dump_rc(str(tmp_path / "nope.xml"), tmp_path) == _lib.RT_E_IO


def test_defaults_match_reference(scene_dir, tmp_path):
    """Optional tags fall back to the reference's defaults (HW2/Scene.cpp:211-236, 312-353):
    stripping BackgroundColor / ShadowRayEpsilon / MaxRecursionDepth and the optional
    material fields must not change the tree."""
    v = _variant(scene_dir, tmp_path,
                 lambda t: re.sub(r"\s*<(BackgroundColor|ShadowRayEpsilon|MaxRecursionDepth)>.*?</\1>",
                                  "", t))
    assert _dump_rc(v, tmp_path) == 0


def test_ppm_library_exports_every_declared_function():
    from ceng795_amd import ppm
    text = open(os.path.join(ROOT, "include", "ceng795_ppm.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|void|const char\s*\*)\s*(ppm_\w+)\s*\(", text, re.M)))
    assert len(names) >= 18
    L = ppm.lib()
    for n in names:
        assert hasattr(L, n), n
        assert n in ppm.SIGNATURES, f"{n} missing from the ctypes table"
    assert L.ppm_abi_version() == ppm.ABI_VERSION
    data = open(ppm.LIB_PATH, "rb").read()
    assert b"ppmref_" not in data and b"libppm_ref" not in data and b"cpuref_" not in data


@pytest.mark.parametrize("name", ["hf_small", "soup1", "soup3"])
@pytest.mark.parametrize("zero_based", [False, True])
def test_binary_mesh_lists_load_to_the_same_scene(scene_dir, tmp_path, name, zero_based):
    """f4: HW7's binary VertexData / Faces (int32 N + triples) load to exactly the scene the
    text lists give — same BVH dump, bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import xml_to_binary
    xml = scenes.write(name, scene_dir)
    binxml = str(tmp_path / f"{name}_bin.xml")
    xml_to_binary.convert(xml, binxml, zero_based=zero_based)
    assert "binaryFile" in open(binxml).read()
    a, b = tmp_path / "text.txt", tmp_path / "bin.txt"
    host_dump_bvh(xml, str(a))
    host_dump_bvh(binxml, str(b))
    assert a.read_bytes() == b.read_bytes()


@pytest.mark.parametrize("name", ["c1", "hf_small", "hf_side", "soup1", "single_sphere", "c2"])
@pytest.mark.parametrize("k", [1, 2])
def test_culling_tree_invariants(scene_dir, name, k):
    """The 8-wide culling tree over reference treelets keeps the invariants
    the kernels' exactness rests on: every leaf in exactly one treelet (a lone leaf, or with
    K = 2 the two leaf children of one reference node), each leaf record's guard box bit-equal
    to its holder's reference box, every fp16 slot box holding every guard box below it with
    the culling margin, children laid out where the kernels look for them, ancestry links
    matching the reference tree."""
    xml = scenes.write(name, scene_dir)
    st = (C.c_longlong * 4)()
    rc = _lib.lib().rt_host_check_accel_xml(xml.encode(), k, st)
    assert rc == 0, _lib.lib().rt_last_error().decode()
    treelets, culling_nodes, depth, lone = list(st)
    if treelets:  # a scene whose whole tree is one treelet gets no culling tree
        # 2 to 8 slots per node
        assert (treelets - 1 + 6) // 7 <= culling_nodes <= treelets - 1
        assert 1 <= depth <= treelets
        assert 0 <= lone <= treelets
        if k == 1:
            assert lone == treelets


def test_culling_tree_on_c3(scene_dir):
    xml = scenes.write_c3(scene_dir)
    st = (C.c_longlong * 4)()
    rc = _lib.lib().rt_host_check_accel_xml(xml.encode(), 2, st)
    assert rc == 0, _lib.lib().rt_last_error().decode()
    treelets, culling_nodes, depth, lone = list(st)
    assert treelets > 300000 and (treelets + 6) // 7 <= culling_nodes < treelets // 3 and depth < 32


# ---- the caller's own BVH in rt_scene_desc (ABI 7) ----------------------
def _dump_desc(desc, path) -> str:
    rc = _lib.lib().rt_host_dump_bvh_desc(C.byref(desc.d), str(path).encode())
    assert rc == 0, _lib.lib().rt_last_error()
    return open(path).read()


@pytest.mark.parametrize("name", ["c1", "hf_small", "soup1", "soup3", "single_sphere",
                                  "single_triangle", "graze_plane"])
def test_prebuilt_tree_is_adopted_exactly(scene_dir, tmp_path, name):
    """A desc carrying its own tree (children, boxes, leaf objects in DFS order, as the binding
    walks the reference's Scene::bvh) flattens to the same preorder dump as the library's own
    build — which is the reference's tree (its golden topology hash) — and a desc without one
    still builds that tree from the object lists."""
    import desc_xml
    xml = scenes.write(name, scene_dir)
    host_dump_bvh(xml, str(tmp_path / "xml.txt"))
    ref = (tmp_path / "xml.txt").read_text()
    assert hashlib.sha256(ref.encode()).hexdigest() == GOLDEN[name]["bvh_sha256"]
    d = desc_xml.Desc(xml)
    assert _dump_desc(d, tmp_path / "built.txt") == ref
    children, boxes, objs = desc_xml.tree_from_dump(ref, d)
    d.set_tree(children, boxes, objs)
    assert _dump_desc(d, tmp_path / "adopted.txt") == ref


def test_prebuilt_tree_normals_are_the_callers(scene_dir, tmp_path):
    """bvh_leaf_normals: the caller's flat normals are taken as given (the binding passes the
    reference's Triangle::normal); a desc with them builds the same tree (the dump carries no
    normals; the GPU binding test checks the shading with the reference's own)."""
    import desc_xml
    xml = scenes.write("soup1", scene_dir)
    host_dump_bvh(xml, str(tmp_path / "xml.txt"))
    ref = (tmp_path / "xml.txt").read_text()
    d = desc_xml.Desc(xml)
    children, boxes, objs = desc_xml.tree_from_dump(ref, d)
    d.set_tree(children, boxes, objs, normals=np.ones(3 * len(objs), np.float32))
    assert _dump_desc(d, tmp_path / "n.txt") == ref


def test_prebuilt_tree_is_validated(scene_dir, tmp_path):
    """Malformed trees are refused with RT_E_INVALID: a leaf out of DFS order, a primitive used
    twice, nodes not in preorder, a wrong node count."""
    import desc_xml
    xml = scenes.write("hf_small", scene_dir)
    host_dump_bvh(xml, str(tmp_path / "xml.txt"))
    d = desc_xml.Desc(xml)
    children, boxes, objs = desc_xml.tree_from_dump((tmp_path / "xml.txt").read_text(), d)
    L = _lib.lib()

    def refused(ch, bx, ob, what):
        d.set_tree(ch, bx, ob)
        rc = L.rt_host_dump_bvh_desc(C.byref(d.d), str(tmp_path / "bad.txt").encode())
        assert rc == _lib.RT_E_INVALID, what
        assert what in L.rt_last_error().decode(), L.rt_last_error()

    swapped = list(children)
    i = swapped.index(-1)  # leaf 0's slot
    j = swapped.index(-2)
    swapped[i], swapped[j] = swapped[j], swapped[i]
    refused(swapped, boxes, objs, "DFS order")
    dup = list(objs)
    dup[1] = dup[0]
    refused(children, boxes, dup, "two leaves")
    k = next(k for k, c in enumerate(children) if c > 1)
    bad = list(children)
    bad[k] += 1
    refused(bad, boxes, objs, "preorder")
    refused(children[:-2], boxes[:-6], objs, "internal nodes")


def test_bench_efficiency_check_names_every_prediction_above_one():
    """bench.py's efficiency_check: any predicted efficiency above 1.0 —
    the line's own split or the RGB bands, record bands and tile deal beside it — is either
    tied to its measured cause (C4's band locality, profiles/r06/band_locality.json) or
    flagged SUSPECT; none above 1.0 reads ok."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    ok = {"8": {"predicted_efficiency": 0.85, "bands": {"predicted_efficiency": 0.9},
                "tiles": {"predicted_efficiency": 0.6}}}
    assert bench.efficiency_check("1920x1080", ok).startswith("ok")
    c3 = {"2": {"predicted_efficiency": 0.97, "bands": {"predicted_efficiency": 1.003}}}
    msg = bench.efficiency_check("1920x1080", c3)
    assert msg.startswith("SUSPECT") and "N = 2 rgb bands 1.003" in msg
    c4 = {"2": {"predicted_efficiency": 1.01, "bands_records": {"predicted_efficiency": 1.01}}}
    msg = bench.efficiency_check("3840x2160", c4)
    assert msg.startswith("above 1.0") and "band_locality.json" in msg
    assert os.path.exists(os.path.join(os.path.dirname(bench.__file__), "profiles", "r06",
                                       "band_locality.json"))
