#!/usr/bin/env python3
"""Static instruction counts of ISA line ranges (build/isa/rt_kernels.s from `make isa`), by
issue class: VALU (v_*), SALU (s_* arithmetic / logic / moves), branch (s_cbranch / s_branch),
SMEM (s_load / s_memtime ...), waitcnt (s_waitcnt, s_nop), LDS (ds_*), VMEM (global_* /
buffer_*).  Used for the per-phase attribution of the frame kernel (profiles/r06/attribution.json):
static counts per path x the RT_DIAG event counts (tools/phases.py).

usage: python tools/isa_count.py build/isa/rt_kernels.s 23572-23625 23883-23903 ...
"""
import json
import sys


def classify(op: str) -> str:
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_dcache")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def count(lines, a: int, b: int) -> dict:
    c = {}
    for ln in lines[a - 1:b]:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":") or t.startswith(";;#"):
            continue
        op = t.split()[0]
        k = classify(op)
        c[k] = c.get(k, 0) + 1
    c["issued"] = sum(v for k, v in c.items() if k not in ("other",))
    return c


def main():
    path = sys.argv[1]
    lines = open(path).read().split("\n")
    out = {}
    for r in sys.argv[2:]:
        a, b = (int(x) for x in r.split("-"))
        out[r] = count(lines, a, b)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
