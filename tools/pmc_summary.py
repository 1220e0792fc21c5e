#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter CSVs: pmc_summary.py <dir>..."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row["Kernel_Name"].split("(")[0].replace("void ", "")
                    if "rocclr" in name:
                        continue
                    vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
