#!/usr/bin/env python3
"""L2 locality of the N-way row-band shares against the whole frame (an
efficiency above 1.0 needs a measured cause).  Two halves of a frame render faster than the whole
when each half's launch re-reads a smaller part of the tree from L2 / HBM; the per-band TCC
hit / miss and FETCH_SIZE counters of the frame kernel show whether that is the cause.

Render side (run under rocprofv3 --pmc, which serialises dispatches, so each launch is counted
alone):  python tools/band_pmc.py render --workload c4 --n 2 --frames 4
  renders the whole frame `frames` times, then rank r's band `frames` times for every r (warm:
  each selection's later launches run in its heavy-first order).
Summary:  python tools/band_pmc.py summary --dirs DIR... --workload c4 --n 2 --frames 4
  groups the frame kernel's dispatches (in order: whole frames, then bands) and reports per warm
  launch the counters, per tile, and the band sum against the whole frame.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def render(a):
    import torch
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    with ceng795_amd.Scene(bench.scene_path(a.workload, 1), device=0) as s:
        c = s.camera(0)
        costs = dist_tiles.measure_tile_costs(s)  # (its own stream and launches, first)
        plan = dist_tiles.BandPlan.from_costs([(c.width, c.height)], a.n, 0, costs)
        st = torch.cuda.Stream()
        frame = torch.empty((c.height, c.width, 3), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(a.frames):
            s.render_device(0, frame.data_ptr(), stream=st.cuda_stream)
        rb = dist_tiles.scene_band_renderer(s)
        cuts = []
        for r in range(a.n):
            for b in plan.per_rank[r]:
                cuts.append([b.tile_begin, b.tile_count])
                for _ in range(a.frames):
                    rb(b, frame, st)
        torch.cuda.synchronize()
        print(json.dumps({"bands": cuts, "tiles": s.num_tiles(0)}))


def dispatches(directory):
    """[(dispatch id, {counter: value})] of trace_frame_kernel, in dispatch order"""
    d = defaultdict(dict)
    for path in glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "trace_frame_kernel" not in row["Kernel_Name"]:
                    continue
                key = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
                d[key][row["Counter_Name"]] = d[key].get(row["Counter_Name"], 0.0) + float(
                    row["Counter_Value"])
    return [v for _, v in sorted(d.items())]


def summary(a):
    meta = json.load(open(a.meta))
    counters = {}
    for directory in a.dirs:
        ds = dispatches(directory)
        need = a.frames * (1 + len(meta["bands"]))
        if len(ds) < need:
            raise SystemExit(f"{directory}: {len(ds)} frame-kernel dispatches, expected {need}")
        ds = ds[-need:]
        for name in ds[0]:
            counters[name] = [x[name] for x in ds]
    warm = range(1, a.frames)  # the first launch of each selection runs in block order

    def avg(vals, g):
        return sum(vals[g * a.frames + i] for i in warm) / len(warm)
    out = {"workload": a.workload, "n": a.n, "frames_per_selection": a.frames,
           "warm_launches_averaged": len(warm), "band_tiles": [b[1] for b in meta["bands"]],
           "frame_tiles": meta["tiles"], "per_launch": {}, "per_tile": {}}
    for name, vals in counters.items():
        whole = avg(vals, 0)
        bands = [avg(vals, 1 + g) for g in range(len(meta["bands"]))]
        out["per_launch"][name] = {"whole": whole, "bands": bands, "band_sum": sum(bands),
                                   "band_sum_over_whole": sum(bands) / whole if whole else None}
        out["per_tile"][name] = {"whole": whole / meta["tiles"],
                                 "bands": [b / t for b, t in zip(bands, out["band_tiles"])]}
    h, m = out["per_launch"].get("TCC_HIT_sum"), out["per_launch"].get("TCC_MISS_sum")
    if h and m:
        out["l2_hit_rate"] = {"whole": h["whole"] / (h["whole"] + m["whole"]),
                              "bands": [x / (x + y) for x, y in zip(h["bands"], m["bands"])]}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["render", "summary"])
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--dirs", nargs="*", default=[])
    ap.add_argument("--meta", default="")
    a = ap.parse_args()
    render(a) if a.mode == "render" else summary(a)


if __name__ == "__main__":
    main()
