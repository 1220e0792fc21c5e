"""The C ABI's multi-device scenes and its concurrency contract, on the GPU box.

* rt_scene_load_xml_multi: one scene over several GPUs of this process; every frame's 8x8 tiles
  are dealt round-robin over the devices, rendered tile-major per device, gathered onto the
  first one (RCCL: single-process communicators, one send / receive group) and untiled there
  (include/ceng795_rt.h).  On the one-GPU box it runs with device_count 1 — the RCCL path with
  a self send / receive — and with device 0 listed 2, 3 and 8 times, which deals the tiles over
  that many replicas of the scene on the one GPU and gathers them by peer copies: the deal and
  untile of the 8-GPU node, rehearsed.  Every frame must equal the CPU oracle's bit for bit.
* Reentrancy: the reference renders one frame from T host threads on disjoint rows
  (HW2/main.cpp:33-36, Scene.cpp:25); rt_render must give the same pixels when called that way,
  and rt_render_device from several host threads, each on a stream of its own.
"""
import os
import threading

import numpy as np
import pytest

import scenes
from oracle.cpu_ref import OracleScene

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
_ORACLE = {}


def oracle_frame(xml, cam):
    if (xml, cam) not in _ORACLE:
        _ORACLE[(xml, cam)] = OracleScene(xml).render(cam, threads=THREADS)
    return _ORACLE[(xml, cam)]


def same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0] * 8])
@pytest.mark.parametrize("name", ["c1", "hf_side", "soup1", "soup_depth3", "single_sphere"])
def test_multi_device_scene_matches_oracle(scene_dir, name, devices):
    import ceng795_amd
    xml = scenes.write(name, scene_dir)
    with ceng795_amd.Scene(xml, devices=devices) as s:
        assert s.device_count == len(devices)
        for cam in range(s.num_cameras):
            ref, st = oracle_frame(xml, cam)
            got, gst = s.render_image(cam)
            assert same(got, ref), (name, devices, cam)
            assert gst.primary_rays == st.primary_rays and gst.shadow_rays == st.shadow_rays
            assert gst.secondary_rays == st.secondary_rays


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0] * 8])
@pytest.mark.parametrize("name", ["msaa4", "msaa5", "msaa9_depth2", "msaa16"])
def test_multi_device_msaa_matches_single_device(scene_dir, name, devices):
    """MSAA over several devices (the Gaussian splat of HW2/Scene.cpp:51-63
    crosses tile borders): each device renders the samples of its band of rows plus a one-row
    halo, resolves its band, and the bands are gathered.  Every frame must be the one-device
    frame bit for bit (which test_msaa_matches_oracle pins to the oracle), with the same ray
    counts — halo rows are not counted twice."""
    import ceng795_amd
    xml = scenes.write(name, scene_dir)
    for seed in (0, 12345):
        with ceng795_amd.Scene(xml) as one:
            one.set_msaa_seed(seed)
            refs = [one.render_image(c) for c in range(one.num_cameras)]
        with ceng795_amd.Scene(xml, devices=devices) as s:
            s.set_msaa_seed(seed)
            for cam, (ref, st) in enumerate(refs):
                got, gst = s.render_image(cam)
                assert same(got, ref), (name, devices, cam, seed)
                assert (gst.primary_rays, gst.shadow_rays, gst.secondary_rays, gst.primary_hits) == \
                    (st.primary_rays, st.shadow_rays, st.secondary_rays, st.primary_hits)


def test_multi_device_msaa_on_caller_stream(scene_dir):
    """rt_render_device of an MSAA camera on a multi-device scene: bands gathered into the
    caller's HBM frame, ordered on the caller's stream."""
    import torch
    import ceng795_amd
    xml = scenes.write("msaa4", scene_dir)
    o = OracleScene(xml)
    ref, _ = o.render_msaa(0, seed=7, threads=THREADS)
    with ceng795_amd.Scene(xml, devices=[0, 0, 0]) as s:
        s.set_msaa_seed(7)
        st = torch.cuda.Stream()
        bufs = []
        for _ in range(2):
            b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
            st.wait_stream(torch.cuda.current_stream())
            s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
            bufs.append(b)
        torch.cuda.synchronize()
        for b in bufs:
            assert same(b.cpu().numpy(), ref)


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
@pytest.mark.parametrize("start,stride", [(3, 5), (0, 64), (47, 1)])
def test_multi_device_row_subsets(scene_dir, devices, start, stride):
    """render_image(cam, px, starting_row, height_increase) keeps its row contract when the
    rows are split over devices."""
    import ceng795_amd
    xml = scenes.write("soup1", scene_dir)
    ref, _ = oracle_frame(xml, 0)
    with ceng795_amd.Scene(xml, devices=devices) as s:
        sentinel = np.full(ref.shape, -7.0, np.float32)
        got, _ = s.render_image(0, sentinel, start, stride)
    rows = np.arange(ref.shape[0])
    sel = (rows >= start) & ((rows - start) % stride == 0)
    assert same(got[sel], ref[sel])
    assert np.all(got[~sel] == -7.0)


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_multi_device_render_device_on_caller_stream(scene_dir, devices):
    """rt_render_device on a multi-device scene: the whole frame into HBM on the first device,
    ordered on the caller's stream (three frames queued back to back, no host sync)."""
    import torch
    import ceng795_amd
    xml = scenes.write("hf_side", scene_dir)
    ref, _ = oracle_frame(xml, 0)
    with ceng795_amd.Scene(xml, devices=devices) as s:
        st = torch.cuda.Stream()
        bufs = []
        for _ in range(3):
            b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
            st.wait_stream(torch.cuda.current_stream())
            s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
            bufs.append(b)
        torch.cuda.synchronize()
        for b in bufs:
            assert same(b.cpu().numpy(), ref)
        with pytest.raises(ceng795_amd.RTError):  # tile subsets are the single-device API
            s.render_device(0, bufs[0].data_ptr(), tile_begin=1, tile_step=2, tile_major=True,
                            stream=st.cuda_stream)


@pytest.mark.parametrize("devices", [[0], [0] * 8])
def test_multi_device_frames_in_flight_on_streams(scene_dir, devices):
    """Frames in flight through a multi-device scene: each caller stream renders on contexts of
    its own (device streams and buffers per caller stream, include/ceng795_rt.h), so three
    frames per stream on three streams overlap on every device — each bit-identical to the
    oracle; releasing a stream hands its contexts back and it renders correctly again."""
    import torch
    import ceng795_amd
    xml = scenes.write("soup_depth3", scene_dir)
    ref, _ = oracle_frame(xml, 0)
    with ceng795_amd.Scene(xml, devices=devices) as s:
        streams = [torch.cuda.Stream() for _ in range(3)]
        for rnd in range(2):
            bufs = []
            for k in range(3):
                for st in streams:
                    b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
                    st.wait_stream(torch.cuda.current_stream())
                    s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
                    bufs.append(b)
            torch.cuda.synchronize()
            for b in bufs:
                assert same(b.cpu().numpy(), ref), (devices, rnd)
            for st in streams:
                s.release_stream(st.cuda_stream)


def test_multi_device_c3_frame_matches_reference_hash(scene_dir):
    """C3 through the multi-device path (RCCL self send / receive on one GPU) hashes to the
    frame the unmodified reference rendered (tests/golden/golden.json)."""
    import hashlib
    import json
    import ceng795_amd
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    xml = scenes.write_c3(scene_dir)
    gc = golden["c3"]["cameras"][0]
    for devices in ([0], [0] * 8):
        with ceng795_amd.Scene(xml, devices=devices) as s:
            got, st = s.render_image(0)
        assert hashlib.sha256(got.tobytes()).hexdigest() == gc["frame_sha256"], devices
        assert st.rays() == gc["rays"]


@pytest.mark.parametrize("name", ["soup1", "hf_side", "soup_depth3"])
def test_threads_render_disjoint_rows_like_the_reference(scene_dir, name):
    """HW2/main.cpp:33-36: T threads call render_image(cam, pixels, i, T) on one const Scene
    and one Pixel array.  ctypes releases the GIL for the call, so the T rt_render calls run
    concurrently in the library (each takes its own render context)."""
    import ceng795_amd
    xml = scenes.write(name, scene_dir)
    ref, _ = oracle_frame(xml, 0)
    for T in (2, 8):
        with ceng795_amd.Scene(xml) as s:
            img = np.full(ref.shape, np.nan, np.float32)
            errors = []

            def work(i):
                try:
                    for _ in range(3):  # repeated: contexts are reused across calls
                        s.render_image(0, img, i, T)
                except Exception as e:  # noqa: BLE001 — reported below
                    errors.append(e)

            ts = [threading.Thread(target=work, args=(i,)) for i in range(T)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            assert not errors, errors
            assert same(img, ref), (name, T)


def test_threads_render_device_on_own_streams(scene_dir):
    """rt_render_device from several host threads at once, each on a new stream of its own:
    every stream's scratch is created while the others render (the table grows under them)."""
    import torch
    import ceng795_amd
    names = ["hf_side", "soup2"]
    xmls = [scenes.write(n, scene_dir) for n in names]
    with ceng795_amd.Scene(xmls[0]) as s:
        ref, _ = oracle_frame(xmls[0], 0)
        T, N = 6, 5
        outs = [[None] * N for _ in range(T)]
        errors = []
        barrier = threading.Barrier(T)

        def work(i):
            try:
                st = torch.cuda.Stream()
                barrier.wait()
                for k in range(N):
                    b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
                    st.wait_stream(torch.cuda.current_stream())
                    s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
                    outs[i][k] = b
                st.synchronize()
                s.release_stream(st.cuda_stream)
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ts = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        assert not errors, errors
        for i in range(T):
            for k in range(N):
                assert same(outs[i][k].cpu().numpy(), ref), (i, k)


def test_release_stream_scratch(scene_dir):
    """A released stream renders correctly again (fresh scratch); releasing a stream the scene
    never used is a no-op."""
    import torch
    import ceng795_amd
    xml = scenes.write("soup_depth3", scene_dir)
    ref, _ = oracle_frame(xml, 0)
    with ceng795_amd.Scene(xml) as s:
        st = torch.cuda.Stream()
        s.release_stream(torch.cuda.Stream().cuda_stream)
        for _ in range(2):
            b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
            st.wait_stream(torch.cuda.current_stream())
            s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
            st.synchronize()
            assert same(b.cpu().numpy(), ref)
            s.release_stream(st.cuda_stream)


@pytest.mark.parametrize("devices", [[0, 0, 0], [0] * 8])
def test_multi_device_back_to_back_frames_on_one_stream(scene_dir, tmp_path, devices):
    """Consecutive frames of two cameras on ONE caller stream, never synchronised in between:
    with a device listed twice the shares are gathered by peer copies on the first device's
    stream while the next frame already renders on the others' streams; each context waits for
    the copy out of its buffers before rendering into them again, so every frame
    stays the oracle's."""
    import torch
    import gen_scene as G
    import ceng795_amd
    xml = str(tmp_path / "hf2cam.xml")
    with open(xml, "w") as f:
        f.write(G.heightfield_scene(40, 120, 72, cameras=2).to_xml())
    refs = [oracle_frame(xml, c)[0] for c in range(2)]
    assert not np.array_equal(refs[0], refs[1])
    with ceng795_amd.Scene(xml, devices=devices) as s:
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        bufs = []
        for k in range(8):
            b = torch.full(refs[0].shape, -1.0, dtype=torch.float32, device="cuda")
            st.wait_stream(torch.cuda.current_stream())
            s.render_device(k % 2, b.data_ptr(), stream=st.cuda_stream)
            bufs.append(b)
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            assert same(b.cpu().numpy(), refs[k % 2]), (devices, k)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_many_caller_streams_stay_bounded(scene_dir, devices):
    """A caller that makes a new stream per frame: beyond the library's per-replica table
    (64 streams) the least recently used stream's scratch / contexts are released after its
    work has finished, and every frame is still right."""
    import torch
    import ceng795_amd
    xml = scenes.write("hf_side", scene_dir)
    ref, _ = oracle_frame(xml, 0)
    kw = {"devices": devices} if devices else {"device": 0}
    with ceng795_amd.Scene(xml, **kw) as s:
        bufs, streams = [], []
        for k in range(80):
            st = torch.cuda.Stream()
            b = torch.full(ref.shape, -1.0, dtype=torch.float32, device="cuda")
            st.wait_stream(torch.cuda.current_stream())
            s.render_device(0, b.data_ptr(), stream=st.cuda_stream)
            bufs.append(b)
            streams.append(st)
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            assert same(b.cpu().numpy(), ref), k
