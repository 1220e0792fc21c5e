#!/usr/bin/env python3
"""Isolated per-kernel times from a rocprofv3 kernel trace of tools/kt.py (its first `frames`
renders run one frame at a time; later ones overlap): average / min over those launches."""
import collections
import csv
import sys


def main(path, frames=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    per = collections.defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"].split("(")[0][:48]].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in per.items():
        n = 2 * frames if k.endswith("order_kernel") and len(v) >= 4 * frames else frames
        iso = v[1:1 + n] if len(v) > n else v
        print(f"{k:48s} launches {len(v):4d}  isolated avg {sum(iso) / len(iso):8.1f} us  "
              f"min {min(iso):8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
