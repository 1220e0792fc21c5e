#!/usr/bin/env python3
"""Estimate of the multi-GPU PPM frame (C5) from one GPU: for S = 1, 2, 4, 8 every update
shard s of S is rendered alone (ppm_set_update_shard), which is the work one of S GPUs does
in a multi-device scene (each replica traces the whole photon sequence and updates its own
tiles).  Prints per S: the slowest shard's update-kernel ms and photon-pass ms, and the
estimated frame ms (eye + grid + slowest photon pass + density; the state gather is < 0.1 ms).

    python3 tools/ppm_shard_probe.py [--shards 1,2,4,8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="1,2,4,8")
    args = ap.parse_args()
    import bench_ppm
    from ceng795_amd import ppm
    xml = bench_ppm.scene_path()
    out = []
    for S in [int(x) for x in args.shards.split(",")]:
        rows = []
        for s in range(S):
            with ppm.PhotonScene(xml, seed=1) as g:
                g.set_update_shard(s, S)
                g.render(0, reference_threads=bench_ppm.REFERENCE_THREADS)  # warm-up
                _, st = g.render(0, reference_threads=bench_ppm.REFERENCE_THREADS)
                rows.append({"shard": s, "update_ms": round(st.update_ms, 3),
                             "photon_ms": round(st.photon_ms, 3),
                             "frame_ms": round(st.eye_ms + st.grid_ms + st.photon_ms + st.density_ms, 3),
                             "updates": st.updates})
        worst = max(rows, key=lambda r: r["frame_ms"])
        line = {"shards": S, "slowest_frame_ms": worst["frame_ms"],
                "slowest_update_ms": max(r["update_ms"] for r in rows),
                "updates_total": sum(r["updates"] for r in rows), "per_shard": rows}
        out.append(line)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
