#!/usr/bin/env python3
"""Per-kernel HIP-event times of whole-frame renders (development tool for same-box A/B runs).

    [CENG795_RT_ORDER=0|1|2] [CENG795_RT_PROBE=0|1] python tools/kt.py [--workload c3]
        [--frames 30] [--inflight 4]

Prints one JSON line: the traversal kernels' average times with one frame at a time (the
primary kernel's time includes the probe + order kernels in front of it: marks 0..1), and the
frames-in-flight throughput (ms per frame over `--frames` frames on `--inflight` streams)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--inflight", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    xml = bench.scene_path(a.workload, 1)
    with ceng795_amd.Scene(xml, device=0) as s:
        st = torch.cuda.current_stream()
        kt, n = bench.isolated_kernel_times(s, st, a.frames)
        out = {"env": {k: os.environ.get(k) for k in ("CENG795_RT_ORDER", "CENG795_RT_PROBE")},
               "one_at_a_time_ms": {k: round(v / n, 4) for k, v in kt.items()}}
        R = dist_tiles.FrameRenderer(s, st, inflight=a.inflight)
        for _ in range(3):
            R.step()
        R.finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            R.step()
        R.finish()
        torch.cuda.synchronize()
        out[f"inflight{a.inflight}_ms_per_frame"] = round((time.perf_counter() - t0) / a.frames * 1e3, 4)
        st_ = s.collect_stats()
        out["rays_per_frame"] = (st_.primary_rays + st_.shadow_rays) // (a.frames + 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
