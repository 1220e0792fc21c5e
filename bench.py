#!/usr/bin/env python3
"""Headline benchmark: Mrays/s of HW2's render path (primary + shadow rays) at 1920x1080 on
the ~1M-triangle height field (BASELINE.json configs[2], "C3"), plus the HBM-roofline fraction
of the render kernel and the reference CPU path timed on this box's host cores.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python bench.py --workload c5        (photon mapping, tools/bench_ppm.py)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

One step = one full render of every camera in the job: N frames of 1920x1080 for N ranks.
The 8x8-pixel tiles of all frames are dealt round-robin over the ranks (the reference deals
rows round-robin over threads, HW2/main.cpp:33-36), each rank renders its tiles into HBM, and
rank 0 gathers them over RCCL (torch.distributed "nccl" = RCCL over xGMI) and untiles the
framebuffers.  Per-GPU work is fixed as N grows: "scaling": "weak".  At N = 1 the step is
exactly one C3 frame rendered in place.

Printed by rank 0: ONE JSON line (see the contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "Mrays/s at 1920×1080 (primary+shadow); fraction of HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    # name: (grid n, width, height, description)
    "c3": (708, 1920, 1080, "C3: 999,698-triangle height field, 1920x1080, 1 point light, "
                            "primary + shadow rays (BASELINE.json configs[2])"),
    "c4": (708, 3840, 2160, "C4: 999,698-triangle height field, 3840x2160, 1 point light"),
    "c2": (187, 800, 800, "C2: 69,192-triangle height field, 800x800, 1 point light"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scene_path(workload: str, cameras: int) -> str:
    import gen_scene as G
    n, w, h, _ = WORKLOADS[workload]
    d = os.environ.get("CENG795_SCENE_DIR", os.path.join(ROOT, "scenes"))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"bench_{workload}_{cameras}cam.xml")
    if not os.path.exists(path):
        spec = G.heightfield_scene(n, w, h, name=f"{workload}.png", cameras=cameras)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(spec.to_xml())
        os.replace(tmp, path)
    return path


def algorithmic_bytes(xml: str, threads: int):
    """B_ray = 32 N_box + 36 N_tri + 16 [hit], with the REFERENCE-order visit
    counts (no culling, HW2/Bounding_volume_hierarchy.cpp:31-55) measured by the oracle's
    instrumented restatement over the whole frame of camera 0, plus 12 B of fp32 RGB output
    per pixel.  Returns (bytes per frame, oracle stats dict)."""
    from oracle.cpu_ref import OracleScene
    o = OracleScene(xml)
    _, st = o.render(0, threads=threads)
    s = st.as_dict()
    box = sum(s["box_tests"])
    tri = sum(s["prim_tests"])
    pixels = s["primary_rays"]
    b = 32 * box + 36 * tri + 16 * s["primary_hits"] + 12 * pixels
    o.close()
    return b, s


def cpu_baseline(xml: str, threads: int):
    """The reference itself (oracle/_ref/ref_harness: HW2 sources compiled unmodified) on this
    box's host cores, rows interleaved over `threads` std::threads as HW2/main.cpp:33-36;
    falls back to the oracle restatement (kind "port") when the reference build is absent."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    reps = 3
    if os.path.exists(harness):
        out = subprocess.run([harness, "time", xml, "0", str(threads), str(reps), "1"],
                             check=True, capture_output=True, text=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        sec, rays, kind = r["seconds_median"], r["rays"], "reference"
    else:
        from oracle.cpu_ref import OracleScene
        o = OracleScene(xml)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            _, st = o.render(0, threads=threads)
            times.append(time.perf_counter() - t0)
        sec = sorted(times)[len(times) // 2]
        rays, kind = st.primary_rays + st.shadow_rays, "port"
    return {"value": round(rays / sec / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "kind": kind,
            "sample": f"full camera-0 frame, median of {reps} renders ({rays} rays, "
                      f"{sec:.3f} s each), render region only as HW2/main.cpp:26-41"}


def stream_copy_gbps(device) -> float:
    """Measured device-to-device copy bandwidth (read + write bytes / time) on this GPU: the
    attainable-HBM reference SURVEY.md §8(d) asks for beside the 8 TB/s spec peak."""
    import torch
    n = 1 << 29  # 2 GiB of fp32 per buffer, far beyond the 256 MB Infinity Cache
    x = torch.empty(n, dtype=torch.float32, device=device).fill_(1.0)
    y = torch.empty_like(x)
    for _ in range(2):
        y.copy_(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    reps = 10
    for _ in range(reps):
        y.copy_(x)
    b.record()
    torch.cuda.synchronize()
    gbps = 2 * 4 * n * reps / (a.elapsed_time(b) * 1e-3) / 1e9
    del x, y
    torch.cuda.empty_cache()
    return gbps


def pmc_traffic(workload: str):
    """HBM bytes per render launch from a committed rocprofv3 --pmc pass (profiles/), corrected
    as MI355X_MICROARCH.md §HBM prescribes; None when no such profile exists."""
    path = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS) + ["c5"],
                    help="c5: the photon-mapping Cornell box (tools/bench_ppm.py), 1 GPU")
    ap.add_argument("--traversal", default="fast", choices=["fast", "reference"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearsal of the N>1 path on one GPU (ranks share device 0)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip rank 0's bit-for-bit check of the gathered frames")
    ap.add_argument("--gather-rehearsal", action="store_true",
                    help="run the N>1 tile/gather pipeline even at WORLD_SIZE=1 (a one-rank "
                         "process group; exercises the comm-stream gather on one GPU)")
    args = ap.parse_args()
    if args.workload == "c5":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            log("c5 (photon mapping) is a one-GPU configuration (BASELINE.json configs[4])")
            return 2
        import bench_ppm
        print(json.dumps(bench_ppm.run(args.steps, args.warmup, not args.no_cpu_baseline)))
        return 0

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    use_pg = world > 1 or args.gather_rehearsal
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")

    import ceng795_amd
    from ceng795_amd import dist_tiles

    n_cams = world
    if rank == 0:
        xml = scene_path(args.workload, n_cams)
    if world > 1:
        dist.barrier()
    xml = scene_path(args.workload, n_cams)
    t0 = time.perf_counter()
    scene = ceng795_amd.Scene(xml, device=device, traversal=args.traversal)
    log(f"[rank {rank}] scene loaded + uploaded in {time.perf_counter() - t0:.2f} s, "
        f"BVH depth {scene.bvh_depth}")
    plan = dist_tiles.TilePlan(scene, world, rank, force=use_pg)
    stream = torch.cuda.current_stream()
    renderer = dist_tiles.FrameRenderer(scene, plan, stream, gather=use_pg,
                                        host_staging=args.dist_backend == "gloo")

    # warmup (also yields the per-step ray count from the device counters)
    for _ in range(args.warmup):
        renderer.step()
    torch.cuda.synchronize()
    st = scene.collect_stats()
    rays_local = (st.primary_rays + st.shadow_rays + st.secondary_rays) / max(1, args.warmup)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    rays_step = torch.tensor([rays_local], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(rays_step)
    rays_step = float(rays_step.item())

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        renderer.step(events=ev[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    kernel_ms_avg = sum(kernel_ms) / len(kernel_ms)
    scene.collect_stats()  # reset counters

    verified = None
    if use_pg and rank == 0 and not args.no_verify:
        # the gathered framebuffers must equal single-GPU renders of the same cameras, bit for bit
        verified = True
        for c, f in enumerate(renderer.frames):
            ref = torch.empty_like(f)
            scene.render_device(c, ref.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize()
            verified &= bool(torch.equal(ref.view(torch.int32), f.view(torch.int32)))
        log(f"[rank 0] gathered frames bit-identical to single-GPU renders: {verified}")

    if rank == 0:
        value = rays_step * args.steps / elapsed / 1e6
        threads = min(16, os.cpu_count() or 1)
        roof = None
        try:
            bytes_frame, ostats = algorithmic_bytes(xml, threads)
            # one launch renders this rank's share of the job's frames
            per_launch = bytes_frame * (rays_local / (ostats["primary_rays"] + ostats["shadow_rays"]))
            achieved = per_launch / (kernel_ms_avg * 1e-3) / 1e9
            traffic = pmc_traffic(args.workload) if world == 1 else None
            copy_gbps = stream_copy_gbps(device)
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    "traffic": traffic,
                    "algorithmic_bytes_per_launch": int(per_launch),
                    "kernel_ms_avg": round(kernel_ms_avg, 4),
                    "stream_copy_GBps_measured": round(copy_gbps, 1),
                    "ref_order_visits_per_ray": {
                        "primary_box": round(ostats["box_tests"][0] / ostats["primary_rays"], 2),
                        "primary_tri": round(ostats["prim_tests"][0] / ostats["primary_rays"], 2),
                        "shadow_box": round(ostats["box_tests"][1] / max(1, ostats["shadow_rays"]), 2),
                        "shadow_tri": round(ostats["prim_tests"][1] / max(1, ostats["shadow_rays"]), 2)}}
        except Exception as e:  # the oracle is a checker; never let it hide the measurement
            log(f"roofline accounting failed: {e!r}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(xml, threads)
            except Exception as e:
                log(f"cpu baseline failed: {e!r}")
        n, w, h, desc = WORKLOADS[args.workload]
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": desc, "frame": f"{w}x{h}", "frames_per_step": n_cams,
                       "triangles": 2 * (n - 1) ** 2, "rays_per_step": int(rays_step),
                       "traversal": args.traversal,
                       "parallelism": f"tiles{world}" + (f"+{'rccl' if args.dist_backend == 'nccl' else 'gloo'}_gather" if use_pg else ""),
                       "gather_verified": verified},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()
    scene.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
