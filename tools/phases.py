#!/usr/bin/env python3
"""Per-phase attribution of the C3 frame kernel: the RT_DIAG build's visit
loop events and 100 MHz real-time clock ticks (rt_debug_phases), one warm frame.

Events per traversal kind (primary / shadow): visits, slots tested, slot hits (some lane
entered), leafy / pair / inner hits, stack pushes and pops, leaf-batch flushes and their
64-test iterations.  Cycles (s_memrealtime, 100 MHz, summed over waves): the whole primary / shadow / shading
phase of each packet, and inside the traversals the node visits (of which the node load: issue
to data), and the leaf-batch flushes.  The clock reads themselves perturb the timing (an SMEM
round trip each), so the cycle split is a proportion, not a kernel time.

usage: CENG795_LIB=diag python tools/phases.py <scene.xml> [--frames 3]   (prints one JSON object)
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EVENTS = ["visits", "slots_tested", "slot_hits", "leafy_hits", "pair_hits", "inner_hits",
          "stack_pushes", "stack_pops", "flushes", "flush_iters"]
CYCLES = ["prim_total", "prim_visit", "prim_load", "prim_flush", "shad_total", "shad_visit",
          "shad_load", "shad_flush", "shade", "frame", "waves"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("xml")
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    if "diag" not in os.environ.get("CENG795_LIB", ""):
        raise SystemExit("run with CENG795_LIB=diag (an RT_DIAG build)")
    import torch
    import ceng795_amd
    from ceng795_amd._lib import lib
    buf = (C.c_ulonglong * 64)()
    with ceng795_amd.Scene(a.xml, device=0) as s:
        c = s.camera(0)
        out = torch.empty((c.height, c.width, 3), device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(a.frames):  # the last one warm (ordered by the previous frame's costs)
            lib().rt_debug_phases(buf, 64)
            s.debug_counters()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.render_device(0, out.data_ptr(), stream=st)
            e1.record()
            torch.cuda.synchronize()
            frame_ms = e0.elapsed_time(e1)
        n = lib().rt_debug_phases(buf, 64)
        d = s.debug_counters()
    if n <= 0:
        raise SystemExit("not a diagnostic build")
    v = list(buf)[:n]
    prim = dict(zip(EVENTS, v[0:10]))
    shad = dict(zip(EVENTS, v[10:20]))
    cyc = dict(zip(CYCLES, v[20:31]))

    def per_visit(e):
        vis = max(1, e["visits"])
        return {k: round(e[k] / vis, 3) for k in EVENTS if k != "visits"}

    frame = max(1, cyc["frame"])
    res = {"scene": os.path.basename(a.xml), "frame": f"{c.width}x{c.height}",
           "primary": prim, "shadow": shad,
           "primary_per_visit": per_visit(prim), "shadow_per_visit": per_visit(shad),
           "leaf_lane_tests": {"primary": d["prim_leaf_lanes"], "shadow": d["shad_leaf_lanes"],
                               "guard_tests": d["guard_tests"]},
           "diag_frame_ms": round(frame_ms, 4),
           "clock": "s_memrealtime (100 MHz): 10 ns per tick",
           "wave_us": {k: round(cyc[k] / max(1, cyc["waves"]) / 100.0, 3) for k in CYCLES
                       if k != "waves"},
           "cycles": cyc,
           "cycle_share_of_frame": {k: round(cyc[k] / frame, 4) for k in CYCLES
                                    if k not in ("frame", "waves")}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
