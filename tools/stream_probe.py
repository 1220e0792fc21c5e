#!/usr/bin/env python3
"""Development tool: does the C3 band probe (N = 8) depend on WHICH render streams it runs on?
One process: the bench's FrameRenderer streams (S0), then fresh sets S1, S2, then S0 again;
per set the t1 frame and rank r's RGB band, each timed over `--steps` steps.  Prints JSON."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    with ceng795_amd.Scene(bench.scene_path("c3", 1), device=0) as s:
        st = torch.cuda.current_stream()
        R = dist_tiles.FrameRenderer(s, st, inflight=a.inflight)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            for _ in range(16):
                R.step()
            R.finish()
            torch.cuda.synchronize()
        costs = dist_tiles.measure_tile_costs(s)
        plan = dist_tiles.BandPlan.from_costs([(1920, 1080)], 8, 0, costs)
        sets = {"S0": R.streams, "S1": dist_tiles.render_streams(a.inflight),
                "S2": dist_tiles.render_streams(a.inflight)}
        for name in ["S0", "S1", "S2", "S0", "S1"]:
            S = sets[name]
            row = {"t1": round(bench.timed_probe(s, dist_tiles.FrameRenderer(
                s, st, inflight=a.inflight, streams=S), a.steps), 4)}
            row["bands"] = [round(bench.timed_probe(s, bench.BandProbe(
                s, plan, r, st, a.inflight, S, False), a.steps), 4) for r in range(8)]
            out.setdefault(name, []).append(row)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
