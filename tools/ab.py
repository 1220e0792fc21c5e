#!/usr/bin/env python3
"""A/B kernel timing on ONE box: each variant is a library build (lib/libceng795_rt_<v>.so,
"" = the production build) timed by `tools/diag.py timing` in its own process; rounds are
interleaved (A B C A B C ...) so device clock drift hits every variant alike.

    python tools/ab.py base,nocx --rounds 3
    python tools/ab.py t0,t4,occ7@4     (tK / lib@K: treelet size K of the culling tree, 0 = none)
    python tools/ab.py base,base:CENG795_RT_STEAL=0   (lib:VAR=VAL[:VAR=VAL]: extra environment)
"""
import argparse
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", default="c3")
    a = ap.parse_args()
    res = defaultdict(lambda: defaultdict(list))
    for _ in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ)
            v_lib, *assigns = v.split(":")
            for a_ in assigns:
                key, _, val = a_.partition("=")
                env[key] = val
            lib, _, k = v_lib.partition("@")  # <lib>@K: treelet size K of the culling tree
            if lib[:1] == "t" and lib[1:].isdigit():  # tK: production lib
                lib, k = "base", lib[1:]
            env["CENG795_LIB"] = "" if lib == "base" else lib
            if k:
                env["CENG795_RT_TREELET"] = k
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag.py"), "timing",
                                  "--workload", a.workload], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            for k, t in json.loads(out.stdout).items():
                res[v][k].append(t["median_ms"])
            # progress line per run (a GPU box kills a command silent for minutes)
            print(v, json.dumps({k: x[-1] for k, x in res[v].items()}), file=sys.stderr, flush=True)
    summary = {v: {k: round(sorted(x)[len(x) // 2], 4) for k, x in d.items()} for v, d in res.items()}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
