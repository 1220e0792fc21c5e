#!/usr/bin/env python3
"""Cold vs warm single-frame latency of library builds (development tool).

    python tools/cold_ab.py base,x [--rounds 3] [--workload c3]

Each (round, variant) runs in its own process with CENG795_LIB=<variant>: 100 ms of untimed
frames (clock ramp), then bench.cold_frame_ms (the first frame of camera 0 on fresh streams,
median of 5) and bench.one_frame_ms (warm, one frame at a time).  Prints one JSON object."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(workload):
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    with ceng795_amd.Scene(bench.scene_path(workload, 1), device=0) as s:
        st = torch.cuda.current_stream()
        R = dist_tiles.FrameRenderer(s, st, inflight=4)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            for _ in range(16):
                R.step()
            R.finish()
            torch.cuda.synchronize()
        cold = bench.cold_frame_ms(s, 5)
        warm = bench.one_frame_ms(s, st, 20)
    return {"cold_frame_ms": cold, "one_frame_ms": warm, "cold_over_warm": round(cold / warm, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.workload)))
        return
    res = {}
    for _ in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ, CENG795_LIB="" if v == "base" else v)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), v, "--one",
                                "--workload", a.workload], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(v, json.dumps(d), file=sys.stderr, flush=True)
    print(json.dumps({v: {"median": {k: sorted(x[k] for x in runs)[len(runs) // 2] for k in runs[0]},
                          "runs": runs} for v, runs in res.items()}))


if __name__ == "__main__":
    main()
