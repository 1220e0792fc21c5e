#!/usr/bin/env python3
"""The traversal kernels' own work on one frame, from the RT_DIAG build
(lib/libceng795_rt_diag.so, the same kernels plus per-wave counters): node visits, leaf visits
and lane tests per kernel.  bench.py runs this as a child process (CENG795_LIB=diag selects the
diagnostic library; the timed library is never instrumented) to price its roofline:

    algorithmic bytes of a traversal launch = 128 B x 8-wide node visits (one node's scalar
                                              loads per packet visit; 64 B x reference-node
                                              visits without a culling tree)
                                            + 64 B x leaf visits   (one DevLeaf per
                                                                    (packet, leaf) pair: the
                                                                    primitive and its guard box)
                                            + per-pixel records    (primary: 8 B hit record
                                                                    written; shadow: 8 B hit
                                                                    record read + 4 B
                                                                    occlusion word written;
                                                                    shading: 8 B hit record +
                                                                    16 B normal / material + 4 B
                                                                    occlusion read, 12 B RGB
                                                                    written)

The frame kernel runs all three phases per packet: frame_bytes = primary + shadow + shading.

usage: CENG795_LIB=diag python tools/kernel_work.py <scene.xml> [--camera 0] [--traversal fast]
prints one JSON object.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("xml")
    ap.add_argument("--camera", type=int, default=0)
    ap.add_argument("--traversal", default="fast", choices=["fast", "reference"])
    a = ap.parse_args()
    if "diag" not in os.environ.get("CENG795_LIB", ""):
        raise SystemExit("run with CENG795_LIB=diag (an RT_DIAG build)")
    import torch
    import ceng795_amd
    with ceng795_amd.Scene(a.xml, device=0, traversal=a.traversal) as s:
        c = s.camera(a.camera)
        buf = torch.empty((c.height, c.width, 3), device="cuda")
        s.debug_counters()
        s.render_device(a.camera, buf.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        d = s.debug_counters()
        if not d["diag_build"]:
            raise SystemExit("not a diagnostic build")
        pixels = c.width * c.height
        words = max(1, (s.num_lights + 31) // 32)
        node_bytes = lambda n, wide: 64 * (n - wide) + 128 * wide  # noqa: E731
        leaf_b = 64 if d["prim_wide_visits"] else 48  # DevLeaf (culling tree) or DevPrim
        prim = (node_bytes(d["prim_node_visits"], d["prim_wide_visits"])
                + leaf_b * d["prim_leaf_visits"] + 8 * pixels)
        shad = (node_bytes(d["shad_node_visits"], d["shad_wide_visits"])
                + leaf_b * d["shad_leaf_visits"] + (8 + 4 * words) * pixels) if s.num_lights else 0
        shade = (8 + 16 + 4 * words + 12) * pixels
        out = {"pixels": pixels, "packets": ((c.width + 7) // 8) * ((c.height + 7) // 8),
               "counters": d,
               "primary_bytes": prim, "shadow_bytes": shad, "shade_bytes": shade,
               "frame_bytes": prim + shad + shade}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
