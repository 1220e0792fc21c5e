#!/usr/bin/env python3
"""Same-box timing of the C ABI's multi-device frames against the one-device path (the
rehearsal of the 8-GPU deal / gather / untile on one GPU: device 0 listed N times).

    python tools/multi_inflight.py [--workload c3] [--frames 40] [--devices 8]

Prints one JSON line: ms per C3 frame for (a) a one-device scene, frames on 1 and 4 streams;
(b) a multi-device scene over device 0 listed N times (peer-copy gather, untile), frames on 1
and 4 caller streams (each caller stream has its own contexts, so its frames overlap)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def timed(scene, cam, bufs, streams, frames):
    import torch
    for k in range(len(streams)):  # warm: every stream's scratch / contexts exist
        scene.render_device(cam, bufs[k].data_ptr(), stream=streams[k].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(frames):
        st = streams[k % len(streams)]
        scene.render_device(cam, bufs[k % len(bufs)].data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / frames * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--devices", type=int, default=8)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    xml = bench.scene_path(a.workload, 1)
    out = {"workload": a.workload, "frames": a.frames}
    for label, devs in (("one_device", None), (f"multi_{a.devices}x_dev0", [0] * a.devices)):
        kw = {"device": 0} if devs is None else {"devices": devs}
        with ceng795_amd.Scene(xml, **kw) as s:
            c = s.camera(0)
            bufs = [torch.empty((c.height, c.width, 3), device="cuda") for _ in range(4)]
            for n in (1, 4):
                streams = [torch.cuda.Stream() for _ in range(n)]
                out[f"{label}_streams{n}_ms"] = round(timed(s, 0, bufs, streams, a.frames), 4)
                for st in streams:
                    s.release_stream(st.cuda_stream)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
