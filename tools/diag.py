#!/usr/bin/env python3
"""Traversal diagnostics on the GPU (development tool, not part of the measured path).

    CENG795_LIB=diag python tools/diag.py counters [--workload c3]
        packet-level work from the RT_DIAG build: node visits per packet, active lanes per
        visit (SIMD utilisation), leaf tests, exact slab-test fallbacks; fast vs reference.
    python tools/diag.py timing [--workload c3]
        kernel time of the production build on the full scene and on a primary-only copy
        (no point lights), to split primary from shadow cost.
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def scene_xml(workload):
    import bench
    return bench.scene_path(workload, 1)


def strip_lights(xml):
    out = xml.replace(".xml", "_nolights.xml")
    if not os.path.exists(out):
        with open(xml) as f:
            text = f.read()
        text = re.sub(r"<PointLight.*?</PointLight>", "", text, flags=re.S)
        with open(out, "w") as f:
            f.write(text)
    return out


def counters(workload):
    import torch  # noqa: F401  (shares its HIP runtime)
    import ceng795_amd
    xml = scene_xml(workload)
    res = {}
    for mode in ["fast", "reference"]:
        with ceng795_amd.Scene(xml, device=0, traversal=mode) as s:
            import torch
            cam = s.camera(0)
            buf = torch.empty((cam.height, cam.width, 3), device="cuda")
            s.debug_counters()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            s.render_device(0, buf.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
            b.record()
            torch.cuda.synchronize()
            c = s.debug_counters()

            class St:
                primary_rays = c["primary_rays"]
                shadow_rays = c["shadow_rays"]
                kernel_ms = a.elapsed_time(b)
            st = St()
            packets = ((cam.height + 7) // 8) * ((cam.width + 7) // 8)
            r = {
                "diag_build": c["diag_build"],
                "packets": packets,
                "prim_node_visits_per_packet": c["prim_node_visits"] / packets,
                "prim_active_lanes_per_visit": c["prim_node_lanes"] / max(1, c["prim_node_visits"]),
                "prim_box_tests_per_ray": 2 * c["prim_node_lanes"] / max(1, st.primary_rays),
                "prim_leaf_visits_per_packet": c["prim_leaf_visits"] / packets,
                "prim_leaf_tests_per_ray": c["prim_leaf_lanes"] / max(1, st.primary_rays),
                "shad_node_visits_per_packet": c["shad_node_visits"] / packets,
                "shad_active_lanes_per_visit": c["shad_node_lanes"] / max(1, c["shad_node_visits"]),
                "shad_box_tests_per_ray": 2 * c["shad_node_lanes"] / max(1, st.shadow_rays),
                "shad_leaf_visits_per_packet": c["shad_leaf_visits"] / packets,
                "shad_leaf_tests_per_ray": c["shad_leaf_lanes"] / max(1, st.shadow_rays),
                "exact_box_fallbacks": c["exact_box_fallbacks"],
                "kernel_ms_diag_build": st.kernel_ms,
            }
            res[mode] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}
    print(json.dumps(res, indent=1))


def timing(workload, reps=10):
    import torch
    import ceng795_amd
    xml = scene_xml(workload)
    out = {}
    for label, path in [("full", xml), ("primary_only", strip_lights(xml))]:
        for mode in ["fast", "reference"]:
            with ceng795_amd.Scene(path, device=0, traversal=mode) as s:
                c = s.camera(0)
                buf = torch.empty((c.height, c.width, 3), device="cuda")
                st = torch.cuda.current_stream()
                for _ in range(2):
                    s.render_device(0, buf.data_ptr(), stream=st.cuda_stream)
                evs = []
                for _ in range(reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    s.render_device(0, buf.data_ptr(), stream=st.cuda_stream)
                    b.record(st)
                    evs.append((a, b))
                torch.cuda.synchronize()
                ms = sorted(a.elapsed_time(b) for a, b in evs)
                out[f"{label}/{mode}"] = {"median_ms": round(ms[len(ms) // 2], 4),
                                          "min_ms": round(ms[0], 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["counters", "timing"])
    ap.add_argument("--workload", default="c3")
    a = ap.parse_args()
    counters(a.workload) if a.what == "counters" else timing(a.workload)
