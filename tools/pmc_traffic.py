#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter CSVs (separate FETCH_SIZE and WRITE_SIZE passes, as
MI355X_MICROARCH.md §HBM and §rocprofv3 prescribe) into per-launch HBM traffic for the render
kernel, written to profiles/traffic_<workload>.json for bench.py's roofline.traffic.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half of the bytes of a wide coalesced stream, so the read side is
doubled.  Our reads are mostly 64-B scalar loads, an access width the guide leaves
uncalibrated: the doubled figure is therefore an upper estimate and the raw figure is kept
beside it.

usage: pmc_traffic.py <fetch_dir> <write_dir> [<tcc_dir>] --workload c3 --round r01
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# the per-frame render step: every kernel of one rt_render_device call
KERNELS = ("trace_primary_kernel", "trace_shadow_kernel", "shade_kernel", "recursive_kernel",
           "render_kernel")
FRAME_KERNEL = ("trace_primary_kernel", "recursive_kernel", "render_kernel")


def per_launch(directory):
    """Counter totals of the render kernels divided by the number of frames (one
    trace_primary dispatch per frame): bytes per render step."""
    files = glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(float)
    frames = defaultdict(int)
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if any(k in name for k in KERNELS):
                    vals[row["Counter_Name"]] += float(row["Counter_Value"])
                if any(k in name for k in FRAME_KERNEL):
                    frames[row["Counter_Name"]] += 1
    return ({k: v / max(1, frames[k]) for k, v in vals.items()}, dict(frames))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("tcc_dir", nargs="?")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch, nf = per_launch(a.fetch_dir)
    write, nw = per_launch(a.write_dir)
    out = {
        "kernels": list(KERNELS),
        "workload": a.workload,
        "round": a.round,
        "frames": {"fetch_pass": nf.get("FETCH_SIZE", 0), "write_pass": nw.get("WRITE_SIZE", 0)},
        "fetch_size_kib_raw": fetch["FETCH_SIZE"],
        "write_size_kib": write["WRITE_SIZE"],
        "read_bytes_raw": fetch["FETCH_SIZE"] * 1024,
        "read_bytes_corrected": 2 * fetch["FETCH_SIZE"] * 1024,
        "write_bytes": write["WRITE_SIZE"] * 1024,
    }
    out["hbm_bytes_per_launch"] = int(out["read_bytes_corrected"] + out["write_bytes"])
    if a.tcc_dir:
        tcc, _ = per_launch(a.tcc_dir)
        out["tcc"] = tcc
        if "TCC_HIT_sum" in tcc and "TCC_MISS_sum" in tcc:
            out["l2_hit_rate"] = tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"])
    path = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "profiles", f"traffic_{a.workload}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
