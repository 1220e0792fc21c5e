#!/usr/bin/env python3
"""Same-box A/B of the one-GPU scaling prediction (bench.py share_probe) and the frame
latencies of library builds (development tool).

    python tools/scale_probe.py base,fused [--workloads c3,c4] [--rounds 2] [--steps 40]

Each (round, workload, variant) runs in its own process with CENG795_LIB=<variant> ("base" = the
production build): one frame at a time (warm), a cold frame, the kernels' HIP-event times one
frame at a time, and t1 / every rank's share at N = 2, 4, 8 over the same steps.  Prints one
JSON object: per variant and workload, the runs and the median of each figure."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def one(workload: str, steps: int, inflight: int) -> dict:
    import torch
    import bench
    import ceng795_amd
    with ceng795_amd.Scene(bench.scene_path(workload, 1), device=0) as s:
        st = torch.cuda.current_stream()
        out = {"one_frame_ms": bench.one_frame_ms(s, st, 20), "cold_frame_ms": bench.cold_frame_ms(s)}
        kt, n = bench.isolated_kernel_times(s, st, 20)
        out["kernel_ms"] = {k: round(v / max(1, n), 4) for k, v in kt.items()}
        p = bench.share_probe(s, st, steps, inflight)
        out["t1_ms"] = p["t1_ms"]
        for k, v in p["per_n"].items():
            out[f"share{k}_ms_max"] = v["share_ms_max"]
            out[f"eff{k}"] = v["predicted_efficiency"]
            out[f"share{k}_per_rank"] = v["share_ms_per_rank"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="?", default="base")
    ap.add_argument("--workloads", default="c3,c4")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--one", help="(internal) one workload in this process")
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.one, a.steps, a.inflight)))
        return
    res = {}
    for _ in range(a.rounds):
        for w in a.workloads.split(","):
            for v in a.variants.split(","):
                env = dict(os.environ, CENG795_LIB="" if v == "base" else v)
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", w,
                                    "--steps", str(a.steps), "--inflight", str(a.inflight)],
                                   env=env, capture_output=True, text=True, timeout=400)
                if r.returncode:
                    print(r.stderr[-3000:], file=sys.stderr)
                    sys.exit(1)
                d = json.loads(r.stdout.strip().splitlines()[-1])
                res.setdefault(v, {}).setdefault(w, []).append(d)
                print(v, w, json.dumps({k: x for k, x in d.items() if "per_rank" not in k}),
                      file=sys.stderr, flush=True)
    summary = {}
    for v, ws in res.items():
        for w, runs in ws.items():
            med = {}
            for k in runs[0]:
                xs = [r[k] for r in runs]
                if all(isinstance(x, (int, float)) for x in xs):
                    med[k] = sorted(xs)[len(xs) // 2]
            summary.setdefault(v, {})[w] = {"median": med, "runs": runs}
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
