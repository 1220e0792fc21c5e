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


def cpu_baseline(xml: str, threads: int, how: str, iterations: int = 1000):
    """The reference itself (oracle/_ref/ppm_harness, PPM sources compiled unmodified) on
    `threads` host threads (the box's CPU quota), the full photon pass (NumberOfIterations
    1000 = 1e7 photons) after a short warm-up run."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ppm_harness")
    if os.path.exists(harness):
        def one(it):
            out = subprocess.run([harness, "render", xml, "0", os.devnull, str(threads), str(it)],
                                 check=True, capture_output=True, text=True).stdout
            return json.loads(out.strip().splitlines()[-1])
        one(10)  # warm-up: page cache, CPU frequency
        r = one(iterations)
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
                      f"1000), {sec:.3f} s, after a 10-iteration warm-up run; threads: {how}"}


def update_roofline(st, launches_per_step: int, ms_per_launch: float):
    """Roofline of the dominant kernel, group_update_kernel, on its ESSENTIAL bytes per launch:
    every deposit's 16-B position record read once (the superset filter) + the 48-B deposit
    record of every candidate it passes to the recurrence (hit-point records and state are
    < 1 %), over its HIP-event duration.  The bytes the kernel's filter actually streams — the
    16-B record per (hit-point tile, deposit) pair, each group list re-read once per tile — are
    reported beside it (`filter_bytes_per_launch`, `frac_filter_bytes`): the excess of those
    over the essential bytes is the re-reading a better design would remove (VERDICT r05 item
    4).  traffic: the committed PMC summary of this library build."""
    import bench
    ess = (16 * st.deposits + 48 * st.update_candidates) / max(1, launches_per_step)
    filt = (16 * st.update_deposit_visits + 48 * st.update_candidates) / max(1, launches_per_step)
    achieved = ess / (ms_per_launch * 1e-3) / 1e9
    prof, traffic = None, None
    path = os.path.join(ROOT, "profiles", "traffic_c5.json")
    if os.path.exists(path):
        from ceng795_amd import ppm
        with open(path) as f:
            prof = json.load(f)
        if prof.get("lib_sha256") == bench.file_sha256(ppm.LIB_PATH):
            traffic = prof["per_kernel"].get("group_update_kernel", {}).get("hbm_bytes")
        else:
            prof = None
    # bound: the kernel lasts as long as its longest tile (a serial per-hit-point chain and
    # one workgroup's compaction of a 2.6 M-record list), not HBM bandwidth;
    # `frac` is measured against the HBM peak it would otherwise hit
    return {"bound": "latency", "peak_of": "hbm", "achieved": round(achieved, 1), "peak": 8000.0,
            "unit": "GB/s",
            "frac": round(achieved / 8000.0, 4), "traffic": traffic,
            "kernel": "group_update_kernel", "kernel_ms_avg": round(ms_per_launch, 4),
            "launches_per_step": launches_per_step,
            "algorithmic_bytes_per_launch": int(ess),
            "bytes_model": "essential: 16 B x deposits (each position record once) + 48 B x "
                           "candidates (ppm_stats.deposits / update_candidates)",
            "filter_bytes_per_launch": int(filt),
            "frac_filter_bytes": round(filt / (ms_per_launch * 1e-3) / 1e9 / 8000.0, 4),
            "filter_bytes_model": "16 B x (hit-point tile, deposit) pairs the filter streams + 48 B "
                                  "x candidates (update_deposit_visits / update_candidates)",
            "work_per_step": {"deposits": st.deposits, "deposit_visits": st.update_deposit_visits,
                              "candidates": st.update_candidates, "updates": st.updates},
            "traffic_source": "profiles/traffic_c5.json" if traffic is not None else None}


def run(steps: int, warmup: int, with_cpu: bool, devices=None) -> dict:
    """devices: None = one GPU (device 0); a list = one multi-device scene over those GPUs of
    this process (ppm_scene_load_xml_multi: every pass on each, the update pass sharded by hit
    point, the state gathered on devices[0])."""
    import torch  # noqa: F401  (shares the HIP runtime; see ceng795_amd/_lib.py)
    from ceng795_amd import ppm

    xml = scene_path()
    scene = ppm.PhotonScene(xml, device=0, seed=1, devices=devices)
    n_gpus = 1 if devices is None else len(devices)
    for k in range(warmup):
        img, st = scene.render(0, reference_threads=REFERENCE_THREADS)
    times, photon_ms, phases, upd_ms = [], [], [], []
    for k in range(steps):
        scene.set_seed(100 + k)
        t0 = time.perf_counter()
        img, st = scene.render(0, reference_threads=REFERENCE_THREADS)
        times.append(time.perf_counter() - t0)
        photon_ms.append(st.photon_ms)
        upd_ms.append(st.update_ms)
        phases.append((st.eye_ms, st.grid_ms, st.photon_ms, st.density_ms))
    ms_step = 1e3 * sum(times) / len(times)
    ph_ms = sum(photon_ms) / len(photon_ms)
    avg = [sum(p[i] for p in phases) / len(phases) for i in range(4)]
    value = st.photons / (ph_ms / 1e3) / 1e6
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mphotons/s", "n_gpus": n_gpus,
        "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "strong" if n_gpus > 1 else "weak",
        "vs_baseline": None, "dtype": "f32",
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
    if devices is not None:
        line["config"]["devices"] = list(devices)
        line["config"]["parallelism"] = (f"ppm_multi{n_gpus}: photon pass replicated, update pass "
                                         "sharded by hit point, state gathered on devices[0]")
        if len(set(devices)) < len(devices):
            line["config"]["rehearsal"] = "a device is listed more than once: replicas share a GPU"
    launches = max(1, st.update_launches)  # one per photon batch (one at this size)
    line["roofline"] = update_roofline(st, launches, sum(upd_ms) / len(upd_ms) / launches)
    if with_cpu:
        import bench
        threads, how = bench.host_cores()
        line["cpu_baseline"] = cpu_baseline(xml, threads, how)
    return line


def run_dist(steps: int, warmup: int, device: str = "cuda", verify: bool = True) -> dict:
    """C5 with one process per GPU (ceng795_amd.dist_ppm): every rank traces the whole photon
    sequence and updates its shard of the hit points; rank 0 gathers the state (RCCL) and runs
    the density estimation.  Timed: whole frames (eye pass, grid, photon pass, gather, density),
    barrier + synchronize on both sides, max over ranks.  Rank 0 checks the last frame against
    a one-GPU render of the same seed (gather_verified).  Returns the line on rank 0, else None."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from ceng795_amd import dist_ppm, ppm

    rank, world = dist.get_rank(), dist.get_world_size()
    xml = scene_path()
    scene = ppm.PhotonScene(xml, device=torch.cuda.current_device(), seed=1)
    for k in range(warmup):
        dist_ppm.render_sharded(scene, 0, REFERENCE_THREADS, device)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    img = traced = None
    for k in range(steps):
        scene.set_seed(100 + k)
        img, traced = dist_ppm.render_sharded(scene, 0, REFERENCE_THREADS, device)
    torch.cuda.synchronize()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    ms_step = 1e3 * float(dt.item()) / steps
    verified = None
    if rank == 0 and verify:
        scene.set_update_shard(0, 1)
        want, _ = scene.render(0, reference_threads=REFERENCE_THREADS)
        verified = bool(np.array_equal(np.asarray(img).view(np.uint32), want.view(np.uint32)))
    scene.close()
    if rank != 0:
        return None
    return {
        "metric": METRIC + ", whole frames", "value": round(traced / (ms_step / 1e3) / 1e6, 2),
        "unit": "Mphotons/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C5: PPM Cornell box, 256x256, 10000 photons x 1000 iterations "
                               "(BASELINE.json configs[4])",
                   "photons_per_step": traced,
                   "parallelism": f"ppm_shards{world}+{dist.get_backend()}_gather",
                   "timed": "whole frame: eye pass, grid, photon pass (whole sequence on every "
                            "rank, update pass sharded by hit point), state gather, density",
                   "gather_verified": verified}}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run(a.steps, a.warmup, not a.no_cpu_baseline)))
