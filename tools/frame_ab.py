#!/usr/bin/env python3
"""Same-box A/B of library builds on the C3 frame (development tool).

    python tools/frame_ab.py base,x,y [--rounds 3] [--workload c3] [--steps 100]

Each (round, variant) runs in its own process with CENG795_LIB=<variant> ("base" = the
production build): 100 ms of untimed frames (the GPU's clock ramp), then the frame kernel's
HIP-event time one frame at a time (median of 20), and the bench's pipelined rate (6 frames in
flight, `--steps` steps).  Rounds interleave the variants (A B C A B C ...).  Prints one JSON
object: per variant the runs and the medians."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def one(workload: str, steps: int) -> dict:
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    with ceng795_amd.Scene(bench.scene_path(workload, 1), device=0) as s:
        st = torch.cuda.current_stream()
        R = dist_tiles.FrameRenderer(s, st, inflight=6)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            for _ in range(16):
                R.step()
            R.finish()
            torch.cuda.synchronize()
        kt, n = bench.isolated_kernel_times(s, st, 20)
        out = {"frame_kernel_ms": round(kt["frame"] / max(1, n), 4)}
        for _ in range(8):
            R.step()
        R.finish()
        out["ms_per_frame_6inflight"] = round(bench.timed_steps(R, steps, 1, "cuda") / steps * 1e3, 4)
        st_ = s.collect_stats()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--one", action="store_true", help="(internal) one run in this process")
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.workload, a.steps)))
        return
    res = {}
    for _ in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ, CENG795_LIB="" if v == "base" else v)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), v, "--one",
                                "--workload", a.workload, "--steps", str(a.steps)],
                               env=env, capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(v, json.dumps(d), file=sys.stderr, flush=True)
    out = {v: {"median": {k: sorted(r[k] for r in runs)[len(runs) // 2] for k in runs[0]},
               "runs": runs} for v, runs in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
