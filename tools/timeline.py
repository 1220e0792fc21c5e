#!/usr/bin/env python3
"""Wave-occupancy timeline of the traversal kernels (development tool; needs the RT_TIMELINE
experiment build: make -C ceng795_amd/csrc exp EXP= EXTRA=-DRT_TIMELINE NAME=timeline).

    CENG795_LIB=timeline python tools/timeline.py [--workload c3] [--slots 8192]

Renders the frame a few times, then reads the last launch's per-wave (start, end) ticks of the
100 MHz clock and reports per kernel: waves, span, wave-duration percentiles, the number of
resident waves over time (20 bins), and slot utilisation = sum of wave lifetimes / (slots x span),
where slots = waves the GPU can hold (256 CUs x 4 SIMDs x 8 waves)."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--slots", type=int, default=8192)
    ap.add_argument("--bins", type=int, default=20)
    ap.add_argument("--save", help="npz of per-tile wave durations (us), one map per kernel")
    ap.add_argument("--world", type=int, default=1,
                    help="> 1: render rank --rank's share of the block deal (tile-major), as one "
                         "rank of an N-GPU run does")
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import _lib
    xml = bench.scene_path(a.workload, 1)
    n = 2 * (1 << 18) * 3
    buf = (C.c_ulonglong * n)()
    out = {}
    with ceng795_amd.Scene(xml, device=0) as s:
        cam = s.camera(0)
        fb = torch.empty((cam.height, cam.width, 3), device="cuda")
        for _ in range(3):  # the last launch's waves are read back (warm order from the 2nd on)
            if a.world > 1:
                s.render_device(0, fb.data_ptr(), tile_begin=a.rank, tile_step=a.world,
                                tile_major=True, blocks=True,
                                stream=torch.cuda.current_stream().cuda_stream)
            else:
                s.render_device(0, fb.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = _lib.lib().rt_debug_timeline(buf, n)
        if got <= 0:
            raise SystemExit("not an RT_TIMELINE build (CENG795_LIB=timeline)")
    tl = np.frombuffer(buf, dtype=np.uint64).reshape(2, 1 << 18, 3).astype(np.int64)
    tiles_x = (cam.width + 7) // 8
    maps = {}
    for k, name in enumerate(["trace_primary_kernel", "trace_shadow_kernel"]):
        t = tl[k]
        t = t[t[:, 0] > 0]
        if not len(t):  # (the fused build records its one kernel as the first)
            continue
        m = np.zeros(((cam.height + 7) // 8, tiles_x), np.float32)
        sel = (t[:, 2] & 0xffffffff).astype(np.uint32).astype(np.int32)
        est = (t[:, 2] >> 32) & 0xffffffff
        ok = sel >= 0
        m.flat[sel[ok]] = (t[ok, 1] - t[ok, 0]) * 0.01  # us per tile
        maps[name] = m
        t0 = t[:, 0].min()
        smap = np.zeros_like(m)
        smap.flat[sel[ok]] = (t[ok, 0] - t0) * 0.01  # start, us
        maps[name + "_start"] = smap
        if est[ok].any():  # the probe's cost estimates (ordered primary launches)
            emap = np.zeros_like(m)
            emap.flat[sel[ok]] = est[ok]
            maps[name + "_estimate"] = emap
        st, en = (t[:, 0] - t0) * 10, (t[:, 1] - t0) * 10  # ns
        span = en.max()
        dur = en - st
        edges = np.linspace(0, span, a.bins + 1)
        mids = (edges[:-1] + edges[1:]) / 2
        resident = [int(((st <= m) & (en > m)).sum()) for m in mids]
        out[name] = {
            "waves": int(len(t)), "span_us": round(span / 1e3, 1),
            "wave_us_p10_p50_p90_max": [round(float(np.percentile(dur, q)) / 1e3, 1)
                                        for q in (10, 50, 90, 100)],
            "last_start_us": round(float(st.max()) / 1e3, 1),
            "slot_utilisation": round(float(dur.sum()) / (a.slots * span), 3),
            "resident_waves_by_time": resident,
        }
    if a.save:
        np.savez_compressed(a.save, **maps)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
