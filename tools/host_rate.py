#!/usr/bin/env python3
"""The drop-in rt_render (host buffer) on the C3 frame, one frame at a time: ms per frame into a
pageable and into a pinned buffer (bench.host_buffer_rate), for the library CENG795_LIB selects.

usage: python tools/host_rate.py [--workload c3] [--frames 10]   (prints one JSON object)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime shared with torch)
    import bench
    import ceng795_amd
    with ceng795_amd.Scene(bench.scene_path(a.workload, 1), device=0) as s:
        r = bench.host_buffer_rate(s, 2.0 * s.camera(0).width * s.camera(0).height, a.frames)
    r["lib"] = os.environ.get("CENG795_LIB", "") or "base"
    print(json.dumps(r))


if __name__ == "__main__":
    main()
