#!/usr/bin/env python3
"""Rank 0's exchange work alone (development tool): the resolve of n-1 ranks' pixel records
and the RGB untile, `--steps` steps each with 4 streams, after 100 ms of preconditioning; and
rt_resolve_rows of (n-1)/n of the frame's rows, one stream.
Run under rocprofv3 --kernel-trace --stats for the kernels' own durations."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    with ceng795_amd.Scene(bench.scene_path(a.workload, 1), device=0) as s:
        st = torch.cuda.current_stream()
        streams = dist_tiles.render_streams(4)
        R = dist_tiles.FrameRenderer(s, st, inflight=4, streams=streams)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            for _ in range(16):
                R.step()
            R.finish()
            torch.cuda.synchronize()
        out = {}
        for rec in (True, False):
            P = bench.ResolveProbe(s, a.n, st, 4, streams, records=rec)
            for _ in range(5):
                P.step()
            P.finish()
            out["resolve_ms" if rec else "untile_ms"] = round(
                bench.timed_steps(P, a.steps, 1, "cuda") / a.steps * 1e3, 4)
        # rt_resolve_rows over rows [h/8, h) of the row-major records (rank 0's share of the
        # 8-way record bands), one launch per step on one stream
        c = s.camera(0)
        rec = torch.empty((c.height, c.width), dtype=torch.int32, device="cuda")
        frame = torch.empty((c.height, c.width, 3), dtype=torch.float32, device="cuda")
        s.render_device(0, rec.data_ptr(), records=True, stream=st.cuda_stream)
        y0 = c.height // a.n
        for _ in range(20):
            s.resolve_rows(0, y0, c.height, rec.data_ptr(), frame.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            s.resolve_rows(0, y0, c.height, rec.data_ptr(), frame.data_ptr(), stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        out["resolve_rows_ms"] = round(e0.elapsed_time(e1) / a.steps, 4)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
