#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter CSVs into per-kernel, per-launch numbers for bench.py's
roofline (profiles/traffic_<workload>.json):

  * HBM traffic: separate FETCH_SIZE and WRITE_SIZE passes (one TCC budget each), as
    MI355X_MICROARCH.md §HBM and §rocprofv3 prescribe.  Both counters are in KiB; on gfx950
    FETCH_SIZE reports exactly half of the bytes of a wide coalesced stream, so the read side
    is doubled.  Our reads are mostly 64-B scalar loads, an access width the guide leaves
    uncalibrated: the doubled figure is the upper estimate, and the raw one is kept beside it.
  * instruction issue (optional insts pass): SQ_INSTS_VALU / SALU / SMEM per launch.  A wave64
    VALU instruction occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md, wave scheduling), so
    VALU issue time = 2 * VALU / (1024 SIMDs * clock); the scalar unit (one per CU) issues one
    SALU per cycle: SALU issue time = SALU / (256 CUs * clock).  bench.py divides them by the
    kernel's live duration.
  * wave states (optional sq pass): SQ_WAVE_CYCLES, SQ_WAIT_ANY (parked at s_waitcnt /
    barrier), SQ_WAIT_INST_ANY (issue stall), SQ_ACTIVE_INST_* (quad-cycles).

The summary records the sha256 of the library the passes ran (bench.py ignores it for any other
build) and the git commit.

usage: pmc_traffic.py --fetch DIR --write DIR [--insts DIR] [--sq DIR] [--workload c3]
                      [--round r02] [--out PATH]
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import subprocess
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("trace_frame_kernel", "order_kernel", "recursive_kernel",
           "group_update_kernel", "photon_kernel", "materialize_kernel", "deposit_keys_kernel")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def per_kernel(directory):
    """{kernel: {counter: value per dispatch}}, {kernel: dispatches}"""
    files = glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {directory}")
    rows = []
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if k is not None:
                    rows.append((k, path, row))
    # only each kernel's largest launches (the whole frame): the bench also makes small ones
    # (the cold-frame probe's one-tile render, shares)
    top = defaultdict(int)
    for k, _, row in rows:
        top[k] = max(top[k], int(row.get("Grid_Size", 0) or 0))
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for k, path, row in rows:
        if int(row.get("Grid_Size", 0) or 0) != top[k]:
            continue
        vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add((path, row.get("Dispatch_Id", row.get("Correlation_Id", ""))))
    n = {k: len(v) for k, v in disp.items()}
    return {k: {c: x / max(1, n[k]) for c, x in v.items()} for k, v in vals.items()}, n


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--insts")
    ap.add_argument("--sq")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--round", default="r02")
    ap.add_argument("--lib", default=os.path.join(ROOT, "ceng795_amd", "lib", "libceng795_rt.so"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch, nf = per_kernel(a.fetch)
    write, nw = per_kernel(a.write)
    insts, _ = per_kernel(a.insts) if a.insts else ({}, {})
    sq, _ = per_kernel(a.sq) if a.sq else ({}, {})
    out_path = a.out or os.path.join(ROOT, "profiles", f"traffic_{a.workload}.json")
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True,
                              text=True).stdout.strip()
    except OSError:
        head = ""
    out = {"workload": a.workload, "round": a.round, "path": out_path,
           "lib_sha256": sha256(a.lib), "git_head": head,
           "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950 streaming-read calibration), "
                         "write = WRITE_SIZE KiB x 1024", "per_kernel": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("FETCH_SIZE", 0.0)
        w = write.get(k, {}).get("WRITE_SIZE", 0.0)
        d = {"dispatches": {"fetch_pass": nf.get(k, 0), "write_pass": nw.get(k, 0)},
             "fetch_size_kib_raw": round(f, 1), "write_size_kib": round(w, 1),
             "read_bytes_raw": int(f * 1024), "read_bytes_corrected": int(2 * f * 1024),
             "write_bytes": int(w * 1024), "hbm_bytes": int(2 * f * 1024 + w * 1024)}
        if k in insts:
            i = insts[k]
            d["issue"] = {c: int(v) for c, v in i.items()}
            if "SQ_INSTS_VALU" in i:
                d["issue"]["valu_issue_us_at_2.4GHz"] = round(2 * i["SQ_INSTS_VALU"] / 1024 / 2.4e3, 2)
            if "SQ_INSTS_SALU" in i:
                d["issue"]["salu_issue_us_at_2.4GHz"] = round(i["SQ_INSTS_SALU"] / 256 / 2.4e3, 2)
        if k in sq:
            d["wave_states"] = {c: int(v) for c, v in sq[k].items()}
        out["per_kernel"][k] = d
    with open(out_path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
