#!/usr/bin/env python3
"""Per-launch counter values of the traversal kernels' FULL-FRAME dispatches (grid of the
whole C3 frame), from rocprofv3 --pmc CSVs of bench.py runs, which also hold the share-probe
and one-frame launches of other grid sizes: pmc_frame.py <dir>... [--grid N]

Prints one JSON object: kernel -> counter -> median over the full-frame dispatches."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main(argv):
    grid = None
    if "--grid" in argv:
        i = argv.index("--grid")
        grid = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # k -> grid -> disp/ctr
    for d in argv:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row["Kernel_Name"].split("(")[0].replace("void ", "")
                    if "trace_" not in name and "order_kernel" not in name:
                        continue
                    key = (path, row["Dispatch_Id"], row["Counter_Name"])
                    vals[name][int(row["Grid_Size"])][key] += float(row["Counter_Value"])
    out = {}
    for k, grids in vals.items():
        g = grid or max(grids)  # the largest launch = the full frame
        per = defaultdict(list)
        for (_, _, ctr), v in grids[g].items():
            per[ctr].append(v)
        out[k] = {"grid": g, **{c: statistics.median(v) for c, v in sorted(per.items())},
                  "dispatches": max(len(v) for v in per.values())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
