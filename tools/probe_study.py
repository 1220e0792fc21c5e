#!/usr/bin/env python3
"""Replay of the traversal kernels' dispatch from measured per-tile wave times (tools/
timeline.py --save maps): how good would a dispatch order be?  A unit (the workgroup's 2x2
tiles) holds its block slot for its slowest tile; each XCD has 32 CUs x `blocks` slots; units
are dealt to XCDs by region (half rows of units round-robin) and run in the given order.
Prints, per maps file: Spearman correlation of the probe's estimate with the measured time,
and the replayed span for block order, per-XCD LPT by the estimate, and per-XCD LPT by the
measured time (the ideal)."""
import sys

import heapq
import numpy as np


def units(mp):
    ty, tx = mp.shape
    nbx, nby = (tx + 1) // 2, (ty + 1) // 2
    out = []
    for by in range(nby):
        for bx in range(nbx):
            ts = [(by * 2 + w // 2, bx * 2 + w % 2) for w in range(4)]
            out.append([(y, x) for y, x in ts if y < ty and x < tx])
    return out, nbx


def replay(dur, U, lists, slots):
    end = 0.0
    for lst in lists:
        heap = [0.0] * slots
        for u in lst:
            t = heapq.heappop(heap)
            heapq.heappush(heap, t + max(dur[y, x] for y, x in U[u]))
        end = max(end, max(heap))
    return end


def rank(a):
    r = np.empty(len(a))
    r[np.argsort(a, kind="stable")] = np.arange(len(a))
    return r


def main():
    for path in sys.argv[1:]:
        m = np.load(path)
        dur = m["trace_primary_kernel"]
        est = m["trace_primary_kernel_estimate"] if "trace_primary_kernel_estimate" in m else None
        U, nbx = units(dur)
        chunk = (nbx + 1) // 2
        reg = [[] for _ in range(8)]
        for u in range(len(U)):
            reg[(u // chunk) % 8].append(u)
        slots = 32 * 7
        res = {"block": replay(dur, U, reg, slots)}
        ideal = [sorted(r, key=lambda u: -max(dur[y, x] for y, x in U[u])) for r in reg]
        res["lpt_measured"] = replay(dur, U, ideal, slots)
        if est is not None:
            rho = np.corrcoef(rank(est.ravel()), rank(dur.ravel()))[0, 1]
            res["spearman"] = rho
            byest = [sorted(r, key=lambda u: -max(est[y, x] for y, x in U[u])) for r in reg]
            res["lpt_estimate"] = replay(dur, U, byest, slots)
        print(path, {k: round(float(v), 3) for k, v in res.items()})


if __name__ == "__main__":
    main()
