#!/usr/bin/env python3
"""Same-box A/B of the N-way row-band split's per-rank work (development tool).

    python tools/band_ab.py base,x [--n 8] [--rounds 3] [--steps 100] [--workload c3]

Each (round, variant) runs in its own process with CENG795_LIB=<variant>: t1 = the whole frame
with six frames in flight (preconditioned, `steps` steps), then every rank's RGB band of the
cost-balanced cut (bench.BandProbe, four frames in flight, each preconditioned) — the unit of
work of the bench's N-GPU split.  Reports the slowest and the mean band and t1 / (N x each)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(workload, n, steps):
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    with ceng795_amd.Scene(bench.scene_path(workload, 1), device=0) as s:
        st = torch.cuda.current_stream()
        streams6, _ = dist_tiles.pick_render_streams(s, 6, 1)
        t1 = bench.timed_probe(s, dist_tiles.FrameRenderer(s, st, inflight=6, streams=streams6),
                               steps, 100.0)
        costs = dist_tiles.measure_tile_costs(s)
        sizes = [(s.camera(0).width, s.camera(0).height)]
        plan = dist_tiles.BandPlan.from_costs(sizes, n, 0, costs)
        streams4 = dist_tiles.render_streams(4)
        bands = [bench.timed_probe(s, bench.BandProbe(s, plan, r, st, 4, streams4, False), steps)
                 for r in range(n)]
    mx, mean = max(bands), sum(bands) / n
    return {"t1_ms": round(t1, 4), "band_ms": [round(b, 4) for b in bands],
            "band_max_ms": round(mx, 4), "band_mean_ms": round(mean, 4),
            "eff_max": round(t1 / (n * mx), 4), "eff_mean": round(t1 / (n * mean), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.workload, a.n, a.steps)))
        return
    res = {}
    for _ in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ, CENG795_LIB="" if v == "base" else v)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), v, "--one", "--n",
                                str(a.n), "--steps", str(a.steps), "--workload", a.workload],
                               env=env, capture_output=True, text=True, timeout=400)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(v, json.dumps(d), file=sys.stderr, flush=True)
    keys = ["t1_ms", "band_max_ms", "band_mean_ms", "eff_max", "eff_mean"]
    print(json.dumps({v: {"median": {k: sorted(x[k] for x in runs)[len(runs) // 2] for k in keys},
                          "runs": runs} for v, runs in res.items()}))


if __name__ == "__main__":
    main()
