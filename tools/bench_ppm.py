#!/usr/bin/env python3
"""Photon-mapping benchmark (BASELINE.json configs[4], "C5"): the PPM Cornell box at 256x256,
PhotonCountPerIteration 10000 x NumberOfIterations 1000, run as PPM/src/main.cpp does on 8
host threads (1e7 photons traced, normaliser P*(P/T)*T).

One step = one ppm_render: eye pass + hash grid + photon pass (trace, deposit sort, hit-point
updates) + density estimation.  The metric is the reference's own phase: photons traced per
second of the photon pass (main.cpp:64-103 prints it as "Tracing photon rays is completed
in"); the whole-frame time is reported beside it.

    python bench.py --workload c5 [--steps K] [--warmup W]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

REFERENCE_THREADS = 8
METRIC = "Mphotons/s (PPM photon pass, Cornell box, 1e7 photons)"


def scene_path() -> str:
    import gen_ppm_scene as GP
    d = os.environ.get("CENG795_SCENE_DIR", os.path.join(ROOT, "scenes"))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "bench_c5.xml")
    if not os.path.exists(path):
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(GP.cornell(256, 256, photons=10000, iterations=1000))
        os.replace(tmp, path)
    return path


def cpu_baseline(xml: str, threads: int, iterations: int = 100):
    """The reference itself (oracle/_ref/ppm_harness, PPM sources compiled unmodified) on
    `threads` host threads, on a bounded sample: NumberOfIterations cut to `iterations`."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ppm_harness")
    if os.path.exists(harness):
        out = subprocess.run([harness, "render", xml, "0", os.devnull, str(threads),
                              str(iterations)], check=True, capture_output=True, text=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        kind, photons, sec = "reference", r["photons_traced"], r["photon_s"]
    else:
        from oracle.ppm_ref import OraclePPM
        import numpy as np  # noqa: F401
        o = OraclePPM(xml)
        w, h, _ = o.camera(0)
        o.eye_pass(0)
        o.build_hash_grid(w, h)
        photons = 10000 // threads * threads * iterations
        t0 = time.perf_counter()
        o.trace_photons(0, 0, photons)
        sec = time.perf_counter() - t0
        kind, threads = "port", 1
    return {"value": round(photons / sec / 1e6, 4), "unit": "Mphotons/s", "cores": threads,
            "kind": kind,
            "sample": f"photon pass of {photons} photons (NumberOfIterations {iterations} of "
                      f"1000), {sec:.3f} s"}


def run(steps: int, warmup: int, with_cpu: bool) -> dict:
    import torch  # noqa: F401  (shares the HIP runtime; see ceng795_amd/_lib.py)
    from ceng795_amd import ppm

    xml = scene_path()
    scene = ppm.PhotonScene(xml, device=0, seed=1)
    for k in range(warmup):
        img, st = scene.render(0, reference_threads=REFERENCE_THREADS)
    times, photon_ms, phases = [], [], []
    for k in range(steps):
        scene.set_seed(100 + k)
        t0 = time.perf_counter()
        img, st = scene.render(0, reference_threads=REFERENCE_THREADS)
        times.append(time.perf_counter() - t0)
        photon_ms.append(st.photon_ms)
        phases.append((st.eye_ms, st.grid_ms, st.photon_ms, st.density_ms))
    ms_step = 1e3 * sum(times) / len(times)
    ph_ms = sum(photon_ms) / len(photon_ms)
    avg = [sum(p[i] for p in phases) / len(phases) for i in range(4)]
    value = st.photons / (ph_ms / 1e3) / 1e6
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mphotons/s", "n_gpus": 1,
        "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": "C5: PPM Cornell box (10 tris + mirror + glass sphere), 256x256, "
                               "10000 photons x 1000 iterations (BASELINE.json configs[4])",
                   "photons_per_step": st.photons, "hit_points": st.hit_points,
                   "deposits_per_step": st.deposits, "updates_per_step": st.updates,
                   "photon_rays_per_step": st.photon_rays,
                   "phase_ms": {"eye": round(avg[0], 3), "grid": round(avg[1], 3),
                                "photon": round(avg[2], 3), "density": round(avg[3], 3)},
                   "frame_photons_per_s": round(st.photons / (ms_step / 1e3) / 1e6, 2)},
    }
    if with_cpu:
        line["cpu_baseline"] = cpu_baseline(xml, REFERENCE_THREADS)
    return line


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run(a.steps, a.warmup, not a.no_cpu_baseline)))
