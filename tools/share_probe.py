#!/usr/bin/env python3
"""One rank's share of the N-way block deal rendered alone on one GPU (what bench.py's share
probe times), with the knobs that could explain share-to-share differences:

    python tools/share_probe.py [--world 8] [--steps 40]

Prints one JSON line: per rank, ms per share with fresh streams (released after each rank)
in two passes (rank order 0..N-1, then reversed), and for ranks 0 and 2 a sweep of the
frames in flight (1, 2, 3, 4, 6, 8)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(scene, world, rank, stream, inflight, steps, torch, dist_tiles, streams=None):
    R = dist_tiles.ShareRenderer(scene, world, rank, stream, inflight=inflight, streams=streams)
    for _ in range(3):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    if streams is None:
        for st in R.streams[1:]:
            scene.release_stream(st.cuda_stream)
    return round(ms, 4)


def timed_inplace(scene, stream, inflight, steps, torch, dist_tiles):
    R = dist_tiles.FrameRenderer(scene, stream, inflight=inflight)
    for _ in range(3):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / steps * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    scene = ceng795_amd.Scene(bench.scene_path("c3", 1), device=0)
    stream = torch.cuda.current_stream()
    out = {"world": a.world}
    N = a.world
    out["inplace_inflight4"] = timed_inplace(scene, stream, 4, a.steps, torch, dist_tiles)
    shared = [torch.cuda.Stream() for _ in range(3)]  # one stream set for every rank
    out["forward_shared_streams"] = [timed(scene, N, r, stream, 4, a.steps, torch, dist_tiles,
                                           shared) for r in range(N)]
    out["forward"] = [timed(scene, N, r, stream, 4, a.steps, torch, dist_tiles) for r in range(N)]
    out["reverse"] = [timed(scene, N, r, stream, 4, a.steps, torch, dist_tiles)
                      for r in reversed(range(N))][::-1]
    for r in sorted({0, min(2, N - 1)}):
        out[f"rank{r}_inflight"] = {k: timed(scene, N, r, stream, k, a.steps, torch, dist_tiles)
                                    for k in (1, 2, 3, 4, 6, 8)}
        print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
