#!/usr/bin/env python3
"""Headline benchmark: Mrays/s of HW2's render path (primary + shadow rays) at 1920x1080 on
the ~1M-triangle height field (BASELINE.json configs[2], "C3"), plus the roofline of the
dominant kernel and the reference CPU path timed on this box's host cores.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python bench.py --workload c5        (photon mapping alone, tools/bench_ppm.py)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

One step = one full render of every camera in the job (default: one 1920x1080 C3 frame).
`--gpus N` with N > 1 and no launcher starts N rank processes itself (torch.distributed.run,
before any GPU call).  N = 1: the step is one C3 frame rendered in place, `--inflight`
consecutive steps (default 6) on as many render streams, picked by timing.  N > 1 (default
`--split bands`, "scaling": "strong"): each frame is cut into one row band per rank at cuts
balanced by the frame's measured tile costs (the reference deals rows round-robin over
threads, HW2/main.cpp:33-36); each rank renders its band in place, ranks > 0 send it to rank 0
point to point over RCCL (torch.distributed "nccl" = RCCL over xGMI) as 32-bit pixel records
that rank 0 shades into its frame (`--exchange rgb`: as RGB), four steps in flight per rank;
`--split tiles` deals 2x2-tile blocks and untiles on rank 0, `--split frames` gives each rank
whole frames.  Rank 0 verifies the frame bit for bit, times the same frame rendered alone to
report t1 / (N * tN), and the line carries a weak-scaling measurement (one whole frame per
rank per step) as an extra key.  At N = 1 the line predicts the split's efficiency for N = 2,
4, 8 from every rank's work timed on this GPU (C3 and C4) and carries the C5 photon-mapping
benchmark (tools/bench_ppm.py) as a `c5` sub-object.

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
# frames in flight: whole frames on one GPU gain from six (10,918-10,989 vs 10,635-10,700
# Mrays/s with four, same box), a rank's 1/N-frame launches from four
# (profiles/r05/hwq_inflight/runs.txt)
INFLIGHT_N1, INFLIGHT_SPLIT = 6, 4
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


def host_cores():
    """Host threads for the CPU baseline: the CPUs this process may run on (affinity), capped
    by the cgroup CPU quota when one is set.  On the GPU box nproc / os.cpu_count() report the
    whole machine while a job gets a share of it (16 CPUs per GPU); more threads than the
    share would only time-slice.  Returns (threads, how it was determined)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"sched_getaffinity {n}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
            how += f", cgroup cpu.max quota {quota}"
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return max(1, n), how + f", nproc {os.cpu_count()}"


def cpu_baseline(xml: str, threads: int, how: str, reps: int = 5, warm: int = 1):
    """The reference itself (oracle/_ref/ref_harness: HW2 sources compiled unmodified) on this
    box's host cores, rows interleaved over `threads` std::threads as HW2/main.cpp:33-36,
    median of `reps` renders after `warm` untimed ones; falls back to the oracle restatement
    (kind "port") when the reference build is absent."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        out = subprocess.run([harness, "time", xml, "0", str(threads), str(reps), "1", str(warm)],
                             check=True, capture_output=True, text=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        sec, rays, kind = r["seconds_median"], r["rays"], "reference"
    else:
        from oracle.cpu_ref import OracleScene
        o = OracleScene(xml)
        times = []
        for k in range(warm + reps):
            t0 = time.perf_counter()
            _, st = o.render(0, threads=threads)
            if k >= warm:
                times.append(time.perf_counter() - t0)
        sec = sorted(times)[len(times) // 2]
        rays, kind = st.primary_rays + st.shadow_rays, "port"
    return {"value": round(rays / sec / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "kind": kind,
            "sample": f"full camera-0 frame, median of {reps} renders after {warm} warm-up "
                      f"({rays} rays, {sec:.3f} s each), render region only as "
                      f"HW2/main.cpp:26-41; threads: {how}"}


def dropin_ms(xml: str, threads: int):
    """The drop-in at the reference's own seam: oracle/_ref/hw2_gpu — the unmodified HW2 Scene /
    Pixel / lodepng sources with the binding of INTEGRATION.md §2 (the reference's parsed Scene
    and its own BVH handed over as an rt_scene_desc) — timed by its own clock over HW2/main.cpp's
    region (:26-41: T threads of render_image_gpu, i.e. rt_render into a pinned frame plus the
    reference's Pixel::add_color per pixel).  One render per camera, as the reference does (a
    cold frame).  Returns {threads: ms} for T = 1 and `threads`, or None without the binary."""
    import re
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "hw2_gpu")
    if not os.path.exists(exe):
        return None
    out = {}
    for t in sorted({1, threads}):
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([exe, xml, "--threads", str(t)], cwd=d, capture_output=True,
                               text=True, timeout=300)
        m = re.search(r"in ([0-9.eE+-]+) ms", r.stdout)
        if r.returncode or not m:
            log(f"hw2_gpu failed ({r.returncode}): {r.stderr[-500:]}")
            return None
        out[str(t)] = round(float(m.group(1)), 3)
    return {"ms_by_threads": out,
            "binary": "oracle/_ref/hw2_gpu (reference HW2 sources + oracle/ref/Scene_gpu.cpp)",
            "region": "HW2/main.cpp:26-41 as the reference times it: render_image_gpu on T "
                      "threads (rt_render into a pinned frame, then Pixel::add_color per pixel); "
                      "one cold frame per camera"}


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


def file_sha256(path: str) -> str:
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def pmc_profile(workload: str):
    """The committed rocprofv3 --pmc summary for this workload (tools/pmc_traffic.py, separate
    FETCH_SIZE / WRITE_SIZE / instruction-count passes, corrected as MI355X_MICROARCH.md §HBM
    prescribes) — used only when it was measured on this very library build (sha256 of
    libceng795_rt.so recorded in it); otherwise None, and traffic is reported as null."""
    from ceng795_amd import _lib
    path = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        prof = json.load(f)
    if prof.get("lib_sha256") != file_sha256(_lib.LIB_PATH):
        log(f"{path} was measured on another library build; traffic reported as null")
        return None
    return prof


def kernel_work(xml: str):
    """Per-frame work of the traversal kernels (tools/kernel_work.py on the RT_DIAG build, in
    a child process): node / leaf visits and the algorithmic bytes they imply."""
    env = dict(os.environ, CENG795_LIB="diag")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_work.py"), xml],
                         check=True, capture_output=True, text=True, env=env, timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])


def isolated_kernel_times(scene, stream, frames: int):
    """HIP-event kernel times of `frames` whole-frame renders of camera 0, one at a time on one
    stream (no other frame in flight): each kernel's own duration, for the roofline."""
    import torch
    cam = scene.camera(0)
    buf = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    scene.render_device(0, buf.data_ptr(), stream=stream.cuda_stream)  # warm
    torch.cuda.synchronize()
    scene.read_kernel_times()
    scene.set_kernel_timing(True)
    for _ in range(frames):
        scene.render_device(0, buf.data_ptr(), stream=stream.cuda_stream)
    torch.cuda.synchronize()
    scene.set_kernel_timing(False)
    kt, n = scene.read_kernel_times()
    scene.collect_stats()
    return kt, n


def host_buffer_rate(scene, rays_frame: float, frames: int = 5):
    """The drop-in host-buffer call (rt_render = Scene::render_image filling a host Image, HW2/
    Scene.h:34-35) on camera 0, one frame at a time: render + device-to-host copy of the float
    RGB frame, into a pageable numpy array and into a pinned one.  Mrays/s; never `value`."""
    import numpy as np
    import torch
    cam = scene.camera(0)
    out = {}
    pinned = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, pin_memory=True)
    for kind, arr in (("pageable", np.empty((cam.height, cam.width, 3), np.float32)),
                      ("pinned", pinned.numpy())):
        scene.render_image(0, arr)  # warm
        t0 = time.perf_counter()
        for _ in range(frames):
            scene.render_image(0, arr)
        sec = (time.perf_counter() - t0) / frames
        out[kind] = {"Mrays_s": round(rays_frame / sec / 1e6, 1), "ms_per_frame": round(sec * 1e3, 3)}
    out["frame_bytes"] = cam.height * cam.width * 3 * 4
    return out


def roofline_line(xml, world, local_share, kt, launches, prof, kt_iso=None, n_iso=0):
    # local_share: fraction of one frame's pixels a timed launch renders
    """Roofline of the dominant kernel, trace_frame_kernel (primary rays, shadow rays and
    shading of every packet in one launch): algorithmic bytes per launch (the kernel's own node
    / leaf fetches of both traversals and its per-pixel records, tools/kernel_work.py) over its
    HIP-event duration.  With frames in flight the timed region's launches share the GPU with
    other frames' kernels, which stretches their start-to-end times; the roofline then uses the
    same launches run one frame at a time right after the timed region (kt_iso), and reports the
    timed-region average beside it.  traffic = HBM bytes per launch of that kernel from the PMC
    profile of this build (or null); issue = its instruction counts from the same profile."""
    work = kernel_work(xml)
    per_launch = work["frame_bytes"] * local_share
    ms_timed = kt["frame"] / launches if launches else None  # (--kernel-timing only)
    if kt_iso is not None and n_iso:
        kt, launches, per_launch = kt_iso, n_iso, work["frame_bytes"]
    ms = kt["frame"] / max(1, launches)
    achieved = per_launch / (ms * 1e-3) / 1e9
    c = work["counters"]
    roof = {"bound": "latency", "peak_of": "hbm", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
            "kernel": "trace_frame_kernel",
            "kernel_ms_avg": round(ms, 4),
            "kernel_ms_avg_timed_region": round(ms_timed, 4) if ms_timed else None,
            "kernel_timing": "one frame at a time after the timed region" if kt_iso is not None
                             and n_iso else "timed region",
            "algorithmic_bytes_per_launch": int(per_launch),
            "algorithmic_bytes_split": {"primary": work["primary_bytes"],
                                        "shadow": work["shadow_bytes"],
                                        "shading": work["shade_bytes"]},
            "bytes_model": "per traversal: 128 B x 8-wide node visits + 64 B x leaf visits "
                           "(DevLeaf: primitive + guard box); per pixel: 8 B hit record written, "
                           "8 B read + 4 B occlusion word written by the shadow phase, 8 B hit "
                           "record + 16 B normal/material + 4 B occlusion read and 12 B RGB "
                           "written by the shading (tools/kernel_work.py, RT_DIAG build, same "
                           "frame)",
            "work_per_frame": {"primary_wide_node_visits": c.get("prim_wide_visits"),
                               "primary_leaf_visits": c["prim_leaf_visits"],
                               "primary_lanes_per_node_visit": round(
                                   c["prim_node_lanes"] / max(1, c["prim_node_visits"]), 2),
                               "primary_leaf_lane_tests": c["prim_leaf_lanes"],
                               "shadow_wide_node_visits": c.get("shad_wide_visits"),
                               "shadow_leaf_visits": c["shad_leaf_visits"],
                               "shadow_leaf_lane_tests": c["shad_leaf_lanes"]},
            "other_kernels_ms_avg": {"order_kernel": round(kt["order"] / max(1, launches), 4)}}
    if prof is not None and world == 1:
        k = prof["per_kernel"].get("trace_frame_kernel", {})
        roof["traffic"] = k.get("hbm_bytes")
        roof["traffic_source"] = os.path.join("profiles", os.path.basename(prof["path"]))
        if "issue" in k:
            i = k["issue"]
            visits = (c.get("prim_wide_visits") or 0) + (c.get("shad_wide_visits") or 0)
            roof["issue"] = {
                "source": roof["traffic_source"],
                "wave_insts": i.get("SQ_INSTS"),
                "valu_wave_insts": i.get("SQ_INSTS_VALU"), "salu_wave_insts": i.get("SQ_INSTS_SALU"),
                "smem_wave_insts": i.get("SQ_INSTS_SMEM"),
                "insts_per_wide_visit": round(i["SQ_INSTS"] / visits, 1)
                if i.get("SQ_INSTS") and visits else None,
                # 2 cycles per wave64 VALU instruction on a SIMD-32, 1024 SIMDs; 1 SALU per
                # cycle per CU, 256 CUs; at 2.4 GHz, over the live kernel time
                "valu_issue_frac": round(i["valu_issue_us_at_2.4GHz"] / (ms * 1e3), 3)
                if "valu_issue_us_at_2.4GHz" in i else None,
                "salu_issue_frac": round(i["salu_issue_us_at_2.4GHz"] / (ms * 1e3), 3)
                if "salu_issue_us_at_2.4GHz" in i else None}
        if "wave_states" in k:
            roof["wave_states"] = k["wave_states"]
    return roof


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch(n: int) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes with torch.distributed.run
    (one per GPU, rendezvous on 127.0.0.1) as a child process and exit with its code.  Called
    before anything touches the GPU; rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    log(f"--gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd[1:6])} ...")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (see Environment)
    return subprocess.run(cmd, env=env).returncode


def timed_steps(renderer, steps: int, world: int, coll_dev: str, events=None):
    """Barrier + synchronize, EXACTLY `steps` renderer steps, finish + synchronize + barrier;
    returns the max over ranks of the wall time (s)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        renderer.step(events=events[k] if events else None)
    renderer.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def n1_steps(scene, stream, inflight: int, steps: int, warmup: int, precondition_ms: float, dev):
    """The N = 1 bench of another scene exactly as main() times its own: render streams picked
    by timing, `inflight` frames in flight, preconditioned for `precondition_ms`, `warmup`
    untimed steps, then `steps` timed steps.  Returns ms per step and Mrays/s."""
    from ceng795_amd import dist_tiles
    rstreams, _ = dist_tiles.pick_render_streams(scene, inflight, 1, device=dev)
    R = dist_tiles.FrameRenderer(scene, stream, inflight=inflight, streams=rstreams)
    precondition(R, precondition_ms)
    scene.collect_stats()
    for _ in range(max(1, warmup)):
        R.step()
    R.finish()
    st = scene.collect_stats()
    rays = (st.primary_rays + st.shadow_rays + st.secondary_rays) / max(1, warmup)
    el = timed_steps(R, steps, 1, "cuda")
    scene.collect_stats()
    return {"ms_per_step": round(el / steps * 1e3, 4),
            "Mrays_s": round(rays * steps / el / 1e6, 2), "steps": steps,
            "frames_in_flight": inflight, "precondition_ms": precondition_ms}


def one_frame_ms(scene, stream, frames: int):
    """Wall time per frame of camera 0 rendered ONE frame at a time (one stream, nothing else
    in flight): the single-frame latency beside the pipelined `value`."""
    import torch
    from ceng795_amd import dist_tiles
    R = dist_tiles.FrameRenderer(scene, stream, inflight=1)
    for _ in range(3):
        R.step()
    R.finish()
    ms = timed_steps(R, frames, 1, "cuda") / frames * 1e3
    scene.collect_stats()
    return round(ms, 4)


def cold_frame_ms(scene, frames: int = 3):
    """Wall time of a COLD frame of camera 0: the first whole frame of that selection on a fresh
    stream, so its primary kernel runs in block order (no previous frame's tile costs to order
    it by).  The stream's scratch is allocated beforehand by a one-tile render
    of another selection (that allocation is a one-time cost, not a frame's); median of
    `frames` fresh streams."""
    import torch
    cam = scene.camera(0)
    buf = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    out = []
    for _ in range(frames):
        st = torch.cuda.Stream()
        scene.render_device(0, buf.data_ptr(), tile_count=1, stream=st.cuda_stream)
        st.synchronize()
        t0 = time.perf_counter()
        scene.render_device(0, buf.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
        scene.release_stream(st.cuda_stream)
    scene.collect_stats()
    return round(sorted(out)[len(out) // 2], 4)


# Steps per timed probe of the one-GPU scaling prediction (at least): a 1/8 band of C3 takes
# ~0.045 ms, so 20 steps timed 1 ms of work and the per-rank times scattered by several % from
# run to run; 100 steps (each probe also preconditioned, precondition()) hold them within ~1-2 %.
PROBE_STEPS = 100


def precondition(R, ms: float):
    """Untimed steps of renderer R for `ms` of wall time (the GPU's clock ramp after an idle
    gap: profiles/r05/warmup_sweep.txt measured 7.5 % on 3 warm-up steps), then its queue
    drained."""
    import torch
    t0 = time.perf_counter()
    while True:
        for _ in range(8):
            R.step()
        R.finish()
        torch.cuda.synchronize()
        if (time.perf_counter() - t0) * 1e3 >= ms:
            return


def timed_probe(scene, R, steps: int, precondition_ms: float = 30.0) -> float:
    """ms per step of probe renderer R, one GPU: preconditioned like the bench's own timed
    region (untimed steps of R for `precondition_ms`), then `steps` timed steps."""
    precondition(R, precondition_ms)
    ms = timed_steps(R, steps, 1, "cuda") / steps * 1e3
    scene.collect_stats()
    return ms


def calibrated_band_plan(scene, n: int, costs, rho, stream, inflight: int, streams,
                        records: bool, steps: int = PROBE_STEPS, rounds: int = 4):
    """Row bands balanced on measured band times.  The cuts start from the measured tile costs
    (records: rank 0's band shrunk by its resolve of the others', root_band_weights(n, rho));
    then every rank's band is timed on this GPU (`inflight` frames in flight, preconditioned) and
    each rank's weight — its share of the tile costs, band_cuts — is scaled by mean / its time,
    up to `rounds` times or until the slowest band is within 1.5 % of the mean.  The plan with
    the smallest slowest band is kept.  Returns (plan, weights, [per-round band times])."""
    from ceng795_amd import dist_tiles
    sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
    w = list(dist_tiles.root_band_weights(n, rho)) if records and rho is not None else [1.0] * n
    plan = dist_tiles.BandPlan.from_costs(sizes, n, 0, costs, w)
    if n == 1:
        return plan, w, []
    best = (float("inf"), plan, list(w))
    hist = []
    for _ in range(rounds):
        t = [timed_probe(scene, BandProbe(scene, plan, r, stream, inflight, streams, records), steps)
             for r in range(n)]
        hist.append([round(x, 4) for x in t])
        if max(t) < best[0]:
            best = (max(t), plan, list(w))
        mean = sum(t) / n
        if max(t) <= 1.015 * mean:
            break
        w = [wi * mean / ti for wi, ti in zip(w, t)]
        plan = dist_tiles.BandPlan.from_costs(sizes, n, 0, costs, w)
    return best[1], best[2], hist


# Measured causes of band efficiencies above 1.0, by frame: per-launch PMC of the frame kernel
# (tools/band_pmc.py, dispatches serialised) for the whole frame and every band of the cut.
BAND_LOCALITY = {
    "3840x2160": "profiles/r06/band_locality.json: the C4 bands' launches together fetch 0.78x "
                 "(N = 2) / 0.73x (N = 8) of the whole frame's HBM bytes, L2 hit rate 0.71 -> "
                 "0.75 / 0.77 (a band's rays walk a smaller part of the tree, which stays in L2); "
                 "C3's bands fetch 1.11x at N = 8 and predict below 1.0",
}


def efficiency_check(frame: str, per_n: dict) -> str:
    """Every prediction of the line (the chosen split and payload, and the RGB bands, record
    bands and tile deal beside it) above 1.0, with its measured cause or flagged."""
    over = []
    for n, v in per_n.items():
        for name, e in (("line", v.get("predicted_efficiency")),
                        ("rgb bands", v.get("bands", {}).get("predicted_efficiency")),
                        ("record bands", v.get("bands_records", {}).get("predicted_efficiency")),
                        ("tile deal", v.get("tiles", {}).get("predicted_efficiency"))):
            if e is not None and e > 1.0:
                over.append(f"N = {n} {name} {e}")
    if not over:
        return "ok: no prediction above 1.0"
    if frame in BAND_LOCALITY:
        return f"above 1.0 ({'; '.join(over)}), measured cause: {BAND_LOCALITY[frame]}"
    return (f"SUSPECT: above 1.0 ({'; '.join(over)}) with no measured cause; treat as a probe "
            "artifact")


def share_probe(scene, stream, steps: int, inflight: int, ns=(2, 4, 8), exchange: str = "rgb",
                split: str = "bands", streams=None, inflight_n: int = INFLIGHT_SPLIT,
                t1_line_ms=None):
    """Prediction of strong scaling on one GPU (no N-GPU node needed).  t1 = the whole frame
    rendered in place with `inflight` frames in flight, and for each N every rank's work of the
    N-way split alone on this GPU — ALL timed over the same `steps` steps after the same warm-up,
    with one set of render streams (each rank of an N-GPU run creates its streams in a fresh
    process).  bands: rank r's cost-balanced row band in place (payload rgb; payload records:
    ranks > 0 render pixel records, rank 0 its smaller band plus the resolve of the others');
    tiles: rank r's block share, plus rank 0's untile / resolve of the others.  The N-GPU step
    can be no shorter than the slowest rank's work: t1 / (N * that step) bounds the efficiency
    from above (the link transfer, overlapped with the rendering of the frames in flight, is
    reported in bytes, not timed).

    t1_line_ms: the N = 1 line's own ms_per_step for this frame (its timed region, after its
    preconditioning), the t1 every efficiency is priced against; the re-probed t1 is reported
    beside it (`t1_probe_ms`) as a check of the probe conditions.  Every probe is preconditioned
    (timed_probe)."""
    from ceng795_amd import dist_tiles
    # t1 on the bench's own render streams (`streams`) with the N = 1 line's frames in flight;
    # every rank's work of an N-way split with the split's frames in flight (`inflight_n`) on
    # a stream set picked the way a rank of the N-GPU run picks its own (pick_render_streams)
    streams = dist_tiles.render_streams(inflight, streams=streams)

    def timed(R):
        return timed_probe(scene, R, steps)

    one = dist_tiles.FrameRenderer(scene, stream, inflight=inflight, streams=streams)
    t1_probe = timed(one)
    t1 = t1_line_ms if t1_line_ms else t1_probe
    inflight = inflight_n
    records = exchange == "records" and dist_tiles.records_ok(scene)
    costs = dist_tiles.measure_tile_costs(scene)
    rho = dist_tiles.measure_resolve_frac(scene) if dist_tiles.records_ok(scene) else None
    sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
    out = {}
    for n in ns:
        streams, set_ms = dist_tiles.pick_render_streams(scene, inflight, n)
        # the band split (bench default): each rank's cost-balanced row band alone, in place;
        # rank 0 receives the others' bands into its frame (records: and shades them, its own
        # band shrunk by that work) — both payloads
        bands_by = {}
        for rec in ((False, True) if rho is not None else (False,)):
            # cuts calibrated on measured band times (records: rank 0's band against its
            # resolve of the others' records too)
            plan, wts, hist = calibrated_band_plan(scene, n, costs, rho, stream, inflight, streams,
                                                   rec, steps)
            bands = [timed(BandProbe(scene, plan, r, stream, inflight, streams, rec))
                     for r in range(n)]
            bc = plan.band_costs(costs)
            band = {"band_ms_per_rank": [round(x, 4) for x in bands],
                    "band_ms_max": round(max(bands), 4),
                    "band_cost_max_over_mean": round(float(
                        bc[1:].max() / bc[1:].mean() if rec and n > 1 else bc.max() / bc.mean()), 4),
                    "band_tile_row_cuts": plan.cuts[0] if len(plan.cuts) == 1 else plan.cuts,
                    "predicted_efficiency": round(t1 / (n * max(bands)), 4),
                    "peer_link_MB_per_step_max": round(max(
                        (4 if rec else 12) *
                        sum((b.y1 - b.y0) * plan.sizes[b.camera][0] for b in plan.per_rank[r])
                        for r in range(1, n)) / 1e6, 3)}
            band["weights"] = [round(x, 4) for x in wts]
            band["calibration_band_ms"] = hist
            if rec:
                band["resolve_frac_of_frame"] = round(rho, 4)
            bands_by["records" if rec else "rgb"] = (band, max(bands))
        band_step = bands_by["records" if records else "rgb"][1]
        # ranks > 0 render what the N-GPU bench exchanges (RGB or pixel records); rank 0's
        # share is the same tile work (it renders in place)
        per = [timed(dist_tiles.ShareRenderer(scene, n, r, stream, inflight=inflight,
                                              streams=streams, records=records and r > 0))
               for r in range(n)]
        # rank 0 also assembles the other ranks' shares into its frame: the RGB untile
        # (rt_untile_device) or the records' shading (rt_resolve_device) — both timed
        untile = timed(ResolveProbe(scene, n, stream, inflight, streams, records=False))
        resolve = (timed(ResolveProbe(scene, n, stream, inflight, streams, records=True))
                   if dist_tiles.records_ok(scene) else None)
        root = resolve if records else untile
        slow = max(max(per), per[0] + root)
        L = dist_tiles.TilePlan(scene, n, 0)
        link = sum(sh.slot for sh in L.shares) * 64 * 4  # bytes per peer per step, per 4 B/px
        tiles = {"share_ms_max": round(max(per), 4), "share_ms_min": round(min(per), 4),
                 "share_ms_per_rank": [round(x, 4) for x in per],
                 "root_untile_ms": round(untile, 4),
                 "root_resolve_ms": None if resolve is None else round(resolve, 4),
                 "peer_link_MB_per_step": {"rgb": round(3 * link / 1e6, 3),
                                           "records": round(link / 1e6, 3)},
                 "predicted_step_ms": round(slow, 4),
                 "predicted_efficiency": round(t1 / (n * slow), 4)}
        step = band_step if split == "bands" else slow
        out[str(n)] = {"split": split, "payload": "records" if records else "rgb",
                       "render_stream_sets_ms": set_ms,
                       "predicted_step_ms": round(step, 4),
                       "predicted_efficiency": round(t1 / (n * step), 4),
                       "predicted_Mrays_s_factor": round(t1 / step, 3),
                       "bands": bands_by["rgb"][0], "tiles": tiles}
        if "records" in bands_by:
            out[str(n)]["bands_records"] = bands_by["records"][0]
    cam = scene.camera(0)
    eff = [v["predicted_efficiency"] for v in out.values()]
    return {"frame": f"{cam.width}x{cam.height}", "t1_ms": round(t1, 4),
            "t1_source": ("the N = 1 line's ms_per_step (same process, same preconditioning)"
                          if t1_line_ms else "re-probed"),
            "t1_probe_ms": round(t1_probe, 4),
            "t1_probe_over_t1": round(t1_probe / t1, 4),
            "efficiency_check": efficiency_check(f"{cam.width}x{cam.height}", out),
            "steps": steps,
            "frames_in_flight": {"t1": one.inflight, "per_rank": inflight_n},
            "split": split,
            "tiles_exchange": "records" if records else "rgb",
            "per_n": out,
            "note": "PREDICTION from one GPU: t1 and every rank's work of one frame, timed over "
                    "the same number of steps with the same frames in flight and render streams, "
                    "each preconditioned; efficiencies priced against the line's own N = 1 step. "
                    "bands (the bench's N>1 split): each rank's cost-balanced row band in place; "
                    "step = the slowest band.  tiles: each rank's block share, plus rank 0's "
                    "untile (or resolve of pixel records) of the others; step = max(slowest "
                    "share, rank 0's share + untile).  Efficiency t1 / (N * step); the transfer "
                    "to rank 0 (MB per xGMI link per step, overlapped with the rendering of the "
                    "frames in flight) is not included"}


class BandProbe:
    """Rank r's bands of a BandPlan rendered in place (no exchange): the per-rank render work of
    the band split, on one GPU.  records: ranks > 0 render pixel records, and rank 0 renders RGB
    and then shades every other band's records (from a whole-frame record buffer rendered once)."""

    def __init__(self, scene, plan, r, stream, inflight, streams, records=False):
        import torch
        from ceng795_amd import dist_tiles
        self.scene, self.stream, self.streams = scene, stream, streams
        self.bands = plan.per_rank[r]
        self.records = records and r > 0
        self.resolve = dist_tiles.scene_row_resolver(scene) if records and r == 0 else None
        self.render = dist_tiles.scene_band_renderer(scene, self.records)
        shape = (lambda w, h: (h, w)) if self.records else (lambda w, h: (h, w, 3))
        dt = torch.int32 if self.records else torch.float32
        self.frames = [[torch.empty(shape(w, h), dtype=dt, device="cuda")
                        for (w, h) in plan.sizes] for _ in range(inflight)]
        self.recs = None
        if self.resolve is not None:
            self.recs = []
            for c, (w, h) in enumerate(plan.sizes):
                t = torch.empty((h, w), dtype=torch.int32, device="cuda")
                scene.render_device(c, t.data_ptr(), records=True,
                                    stream=torch.cuda.current_stream().cuda_stream)
                self.recs.append(t)
            torch.cuda.synchronize()
        for st in streams:
            st.wait_stream(stream)
        self.k = 0

    def step(self, events=None):
        s = self.k % len(self.streams)
        self.k += 1
        st = self.streams[s]
        for c, b in enumerate(self.bands):
            if b.rows > 0:
                self.render(b, self.frames[s][c], st)
            if self.resolve is not None:
                h = self.frames[s][c].shape[0]
                for y0, y1 in ((0, b.y0), (b.y1, h)):
                    if y1 > y0:
                        self.resolve(c, y0, y1, self.recs[c], self.frames[s][c], st)

    def finish(self):
        for st in self.streams:
            self.stream.wait_stream(st)


class ResolveProbe:
    """Rank 0's shading of the other n-1 ranks' pixel records (rt_resolve_device with skip_root,
    every camera), on records rendered once beforehand: the exchange's extra GPU work on rank 0
    (records=False: the RGB untile, rt_untile_device, instead)."""

    def __init__(self, scene, n, stream, inflight, streams, records=True):
        import torch
        from ceng795_amd import dist_tiles
        self.scene, self.stream = scene, stream
        self.layout = L = dist_tiles.TilePlan(scene, n, 0)
        self.streams = streams
        dev = torch.device("cuda", torch.cuda.current_device())
        self.gathered = []
        for c, sh in enumerate(L.shares):
            g = torch.zeros((n, sh.slot, dist_tiles.TILE_RECORDS if records else
                             dist_tiles.TILE_FLOATS), dtype=torch.float32, device=dev)
            for r in range(1, n):
                sr = L.per_rank[r][c]
                if sr.count:
                    scene.render_device(c, g[r].data_ptr(), tile_begin=sr.tile_begin,
                                        tile_step=sr.tile_step, tile_major=True,
                                        blocks=sr.blocks, records=records,
                                        stream=torch.cuda.current_stream().cuda_stream)
            self.gathered.append(g)
        self.frames = [[torch.empty((h, w, 3), dtype=torch.float32, device=dev)
                        for (w, h) in L.sizes] for _ in range(inflight)]
        torch.cuda.synchronize()
        self.untile = dist_tiles.scene_tile_untiler(scene, L, records=records)
        for st in streams:
            st.wait_stream(stream)
        self.k = 0

    def step(self, events=None):
        s = self.k % len(self.streams)
        self.k += 1
        st = self.streams[s]
        for c in range(len(self.gathered)):
            self.untile(c, self.gathered[c], self.frames[s][c], st, skip_root=True)

    def finish(self):
        for st in self.streams:
            self.stream.wait_stream(st)


def band_bytes(renderer) -> int:
    """Bytes rank 0 receives per step in the band split: the other ranks' bands as fp32 RGB (12 B
    per pixel) or as pixel records (4 B)."""
    plan = renderer.plan
    per_px = 4 if renderer.records else 12
    return int(sum(per_px * (b.y1 - b.y0) * plan.sizes[b.camera][0]
                   for r in range(1, plan.world) for b in plan.per_rank[r]))


def band_exchange_text(world, comm, renderer, band_costs):
    import numpy as np
    plan = renderer.plan
    txt = ("rank 0 renders its row band in place; batch_isend_irecv (RCCL send / receive) of "
           "the other ranks' bands straight into rank 0's frame rows (no untile)" if world > 1
           else "one-rank rehearsal: rank 0's row band through an RCCL self send / receive pair "
                "(batch_isend_irecv) into the frame")
    if renderer.records:
        txt += ("; the bands travel as 32-bit pixel records (hit primitive + shadow bits, 4 B per "
                "pixel) that rank 0 shades into its frame (rt_resolve_rows); rank 0's band is "
                "shrunk by that work")
    out = {"how": txt + ("" if comm == "rccl" else " (gloo: through host copies)"),
           "band_tile_row_cuts": plan.cuts, "payload": "records" if renderer.records else "rgb"}
    if getattr(renderer, "resolve_frac", None) is not None:
        out["resolve_frac_of_frame"] = round(renderer.resolve_frac, 4)
    if getattr(renderer, "stream_set_ms", None) is not None:
        out["render_stream_sets_ms"] = renderer.stream_set_ms
    if band_costs is not None and len(band_costs) > 1:
        out["band_cost_max_over_mean"] = round(float(max(band_costs) / np.mean(band_costs)), 4)
    return out


def renderer_records(renderer) -> bool:
    return getattr(renderer, "tile_words", 0) == 64


def exchange_bytes(renderer) -> int:
    """Bytes rank 0 receives per step in the tile split: every other rank's slots."""
    L = renderer.layout
    return int(4 * renderer.tile_words * sum(sh.slot for sh in L.shares) * (L.world - 1))


def synthetic_frame(w: int, h: int, seed: int = 795):
    """Stand-in framebuffer for the CPU rehearsal: deterministic fp32 values per pixel."""
    import numpy as np
    return np.random.default_rng(seed).standard_normal((h, w, 3)).astype(np.float32)


def cpu_rehearsal_bands(args, truth, world, rank, desc) -> int:
    """cpu_rehearsal of the band split: bands cut from a synthetic cost map (the frame's own
    values per tile, so the bands are uneven), each rank's band copied from the synthetic frame
    into its frame instead of rendered, the BandGatherRenderer exchange over gloo, and rank 0's
    frame checked bit for bit."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from ceng795_amd import dist_tiles
    h, w, _ = truth.shape
    tx, ty = dist_tiles.tiles_of((w, h))
    pad = np.zeros((ty * 8, tx * 8), np.float64)
    pad[:h, :w] = np.abs(truth).sum(2)
    costs = pad.reshape(ty, 8, tx, 8).sum((1, 3)).reshape(-1) + 1.0
    plan = dist_tiles.BandPlan.from_costs([(w, h)], world, rank, [costs])
    src = torch.from_numpy(truth)
    rendered = []

    def render(b, frame, stream):
        rendered.append(b.y1 - b.y0)
        frame[b.y0:b.y1].copy_(src[b.y0:b.y1])

    R = dist_tiles.BandGatherRenderer(plan, None, render, host_staging=True, device="cpu")
    for _ in range(args.warmup):
        R.step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frames = R.step()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    b = plan.bands[0]
    assert sum(rendered) == (args.warmup + args.steps) * (b.y1 - b.y0)
    if rank == 0:
        ok = bool(np.array_equal(frames[0].numpy().view(np.uint32), truth.view(np.uint32)))
        print(json.dumps({"metric": "cpu rehearsal of the N>1 exchange (no rendering)",
                          "value": round(w * h * args.steps / float(el.item()) / 1e6, 3),
                          "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "scaling": "strong",
                          "data": "synthetic frame, cpu-rehearsal",
                          "config": {"workload": desc, "parallelism": f"bands{world}+gloo_p2p",
                                     "band_cuts": plan.cuts[0],
                                     "band_costs": [round(x, 1) for x in plan.band_costs([costs])],
                                     "gather_verified": ok}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def band_cuts_for(scene, world: int, rank: int, coll_dev: str, records: bool = False,
                  inflight: int = 4, streams=None):
    """Rank 0 measures every camera's tile costs (whole frames on this GPU) and cuts the bands
    (records: rank 0's band shrunk by its resolve of the others', root_band_weights), then
    balances them on measured band times (calibrated_band_plan); the cuts are broadcast so
    every rank holds the same plan.  Returns (cuts, tile costs or None, the
    resolve fraction or None)."""
    import torch
    import torch.distributed as dist
    from ceng795_amd import dist_tiles
    sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
    costs = rho = None
    flat = []
    if rank == 0:
        costs = dist_tiles.measure_tile_costs(scene)
        if records:  # rank 0's band sized against its resolve of the others' records
            rho = dist_tiles.measure_resolve_frac(scene)
        st = torch.cuda.current_stream()
        # the cuts balanced on this GPU's measured band times (calibrated_band_plan)
        plan, _, _ = calibrated_band_plan(scene, world, costs, rho, st, inflight,
                                          dist_tiles.render_streams(inflight, streams=streams),
                                          records)
        flat = [x for cc in plan.cuts for x in cc]
    t = torch.tensor(flat if rank == 0 else [0] * (len(sizes) * (world + 1)),
                     dtype=torch.int64, device=coll_dev)
    if world > 1:
        dist.broadcast(t, 0)
    v = t.cpu().tolist()
    return [v[c * (world + 1):(c + 1) * (world + 1)] for c in range(len(sizes))], costs, rho


def cpu_rehearsal(args) -> int:
    """The N>1 default path with no GPU (gloo, host tensors): the frame's tiles dealt over the
    ranks, each rank's share written tile-major into its slot (cut from a synthetic frame
    instead of rendered), the pipelined TileGatherRenderer exchange, rank 0's untile and a
    bit-for-bit check against the synthetic frame.  For the multi-rank CPU tests of the
    launcher and the exchange; "value" is pixels per second of that exchange, not Mrays/s."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from ceng795_amd import dist_tiles
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("gloo")
    _, w, h, desc = WORKLOADS[args.workload]
    truth = synthetic_frame(w, h)
    if args.split == "bands":
        return cpu_rehearsal_bands(args, truth, world, rank, desc)
    L = dist_tiles.TileLayout([(w, h)], world, rank)
    tx, ty = dist_tiles.tiles_of((w, h))
    pad = np.zeros((ty * 8, tx * 8, 3), np.float32)
    pad[:h, :w] = truth
    tiles = torch.from_numpy(pad.reshape(ty, 8, tx, 8, 3).transpose(0, 2, 1, 3, 4)
                             .reshape(tx * ty, dist_tiles.TILE_FLOATS).copy())
    rendered = []

    share = torch.from_numpy(L.share_tiles(0, rank))  # frame tile of each slot tile (-1: none)

    def render(sh, slot, stream):
        rendered.append(len(share))
        part = tiles[share.clamp(min=0)]
        part[share < 0] = 0.0
        slot[:len(share)].copy_(part)

    R = dist_tiles.TileGatherRenderer(L, None, render, host_staging=True, device="cpu")
    for _ in range(args.warmup):
        R.step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frames = R.step()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    assert sum(rendered) == (args.warmup + args.steps) * L.local_tiles
    if rank == 0:
        ok = bool(np.array_equal(frames[0].numpy().view(np.uint32), truth.view(np.uint32)))
        print(json.dumps({"metric": "cpu rehearsal of the N>1 exchange (no rendering)",
                          "value": round(w * h * args.steps / float(el.item()) / 1e6, 3),
                          "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "scaling": "strong",
                          "data": "synthetic tiles, cpu-rehearsal",
                          "config": {"workload": desc, "parallelism": f"tiles{world}+gloo_gather",
                                     "gather_verified": ok}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS) + ["c5"],
                    help="c5: the photon-mapping Cornell box alone (tools/bench_ppm.py); "
                         "--gpus N: one multi-device scene over devices 0..N-1 of this process; "
                         "under a launcher (WORLD_SIZE > 1) or --gather-rehearsal: one process "
                         "per GPU, update pass sharded, state gathered over RCCL")
    ap.add_argument("--devices", default="",
                    help="c5: comma-separated device list of the multi-device scene (e.g. 0,0 "
                         "rehearses two replicas on one GPU)")
    ap.add_argument("--traversal", default="fast", choices=["fast", "reference"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true",
                    help="N=1: skip the C5 (photon mapping) sub-object of the line")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearsal of the N>1 path through host copies")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip rank 0's bit-for-bit check of the gathered frames")
    ap.add_argument("--gather-rehearsal", action="store_true",
                    help="run the N>1 tile / gather pipeline even at WORLD_SIZE=1 (a one-rank "
                         "process group; exercises the comm-stream gather on one GPU)")
    ap.add_argument("--frames", type=int, default=1,
                    help="frames (cameras) per step; --split tiles deals their tiles over the "
                         "ranks (strong scaling at 1 frame), --split frames gives each rank "
                         "whole frames (default then: one per rank)")
    ap.add_argument("--split", default="bands", choices=["bands", "tiles", "frames"],
                    help="N>1: bands = each frame cut into one row band per rank at measured-"
                         "cost-balanced cuts, received by rank 0 straight into its frame; tiles = "
                         "2x2 tile blocks dealt round-robin, gathered and untiled by rank 0; "
                         "frames = whole frames per rank (weak scaling)")
    ap.add_argument("--no-weak", action="store_true",
                    help="N>1: skip the extra weak-scaling measurement (one frame per rank)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--gather-stream", choices=("render", "comm"), default="render",
                    help="N>1 tile split: enqueue a step's gather + untile on its own render "
                         "stream (default) or on one communication stream")
    ap.add_argument("--exchange", choices=("rgb", "records"), default="records",
                    help="N>1: the bands / shares travel as 32-bit pixel records (default where "
                         "the scene allows: 4 B per pixel, shaded by rank 0 — a third of the link "
                         "bytes for rank 0 re-reading the hit primitives; with bands, rank 0's "
                         "band is calibrated smaller by that work) or as fp32 RGB (12 B)")
    ap.add_argument("--root-gather", action="store_true",
                    help="N>1 tile split: rank 0 renders its share tile-major and gathers it "
                         "with the others (default: in place, point-to-point receives only)")
    ap.add_argument("--step-events", action="store_true",
                    help="per-step timing events in the timed region (render_ms_avg; they cost "
                         "a few %% of the step)")
    ap.add_argument("--kernel-timing", action="store_true",
                    help="HIP events around the kernels inside the timed region too (the "
                         "roofline always uses one-frame-at-a-time times after it)")
    ap.add_argument("--split-inflight", type=int, default=INFLIGHT_SPLIT,
                    help="frames in flight per rank of the N>1 split (and of the N=1 line's "
                         "prediction of it)")
    ap.add_argument("--no-share-probe", action="store_true",
                    help="N=1: skip the one-GPU prediction of strong scaling (share probe)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: the N>1 tile deal / gather / untile with synthetic tiles over "
                         "gloo (tests of the launcher and the exchange)")
    ap.add_argument("--precondition-ms", type=float, default=100.0,
                    help="untimed steps for this long before the warm-up steps (the GPU's clock "
                         "ramp; 0 = none)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight per GPU: consecutive steps on that many streams / "
                         "buffer sets, so one frame's sparsely occupied last waves (and, N>1, "
                         "its exchange) overlap the next frame; 1 = one frame at a time "
                         "(default: 6 for one GPU's whole frames, 4 for the N>1 split's "
                         "smaller per-rank launches; profiles/r05/hwq_inflight/)")
    args = ap.parse_args()
    if args.workload == "c5" and (int(os.environ.get("WORLD_SIZE", "1")) > 1
                                  or args.gather_rehearsal):
        # one process per GPU (launcher, or --gpus N relaunched below): the update pass
        # sharded over the ranks, the hit-point state gathered to rank 0 (dist_ppm)
        import torch
        import torch.distributed as dist
        import bench_ppm
        local = int(os.environ.get("LOCAL_RANK", "0"))
        device = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29577))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        line = bench_ppm.run_dist(args.steps, args.warmup, "cuda", not args.no_verify)
        if line is not None:
            print(json.dumps(line), flush=True)
        dist.destroy_process_group()
        return 0
    if args.workload == "c5":
        import bench_ppm
        devices = None
        if args.devices:
            devices = [int(d) for d in args.devices.split(",")]
        elif args.gpus > 1:
            devices = list(range(args.gpus))
        print(json.dumps(bench_ppm.run(args.steps, args.warmup,
                                       not args.no_cpu_baseline and devices is None, devices)))
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(args.gpus)
    if args.cpu_rehearsal:
        return cpu_rehearsal(args)

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
    if args.inflight is None:
        args.inflight = INFLIGHT_N1 if not use_pg else args.split_inflight
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29577))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    host_staging = args.dist_backend == "gloo"

    import ceng795_amd
    from ceng795_amd import dist_tiles

    if args.split == "frames" and args.frames < world:
        args.frames = world
    n_cams = max(1, args.frames)
    tiled = use_pg and args.split == "tiles"
    banded = use_pg and args.split == "bands"
    strong = (tiled or banded) and n_cams < world  # one frame (or a few) split over more ranks
    if rank == 0:
        xml = scene_path(args.workload, n_cams)
    if world > 1:
        dist.barrier()
    xml = scene_path(args.workload, n_cams)
    t0 = time.perf_counter()
    scene = ceng795_amd.Scene(xml, device=device, traversal=args.traversal)
    log(f"[rank {rank}] scene loaded + uploaded in {time.perf_counter() - t0:.2f} s, "
        f"BVH depth {scene.bvh_depth}")
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", device)
    band_costs = None
    if not use_pg:
        # render streams picked by timing whole frames (pick_render_streams: the first set a
        # process creates rendered C3 frames ≈1.5 % slower than later ones)
        rstreams, stream_ms = dist_tiles.pick_render_streams(scene, args.inflight, 1, device=dev)
        renderer = dist_tiles.FrameRenderer(scene, stream, inflight=args.inflight,
                                            streams=rstreams)
        renderer.stream_set_ms = stream_ms
    elif banded:
        # the bands travel as 32-bit pixel records (a third of RGB's link bytes) shaded by rank 0
        # (rt_resolve_rows), whose band is shrunk by that work
        records = args.exchange == "records" and dist_tiles.records_ok(scene)
        # the render streams first, picked by measurement (pick_render_streams): the
        # calibration runs on the streams the steps will use
        rstreams, stream_ms = ((None, None) if host_staging else
                               dist_tiles.pick_render_streams(scene, args.inflight, world,
                                                              device=dev))
        cuts, costs, resolve_frac = band_cuts_for(scene, world, rank, coll_dev, records,
                                                  args.inflight, rstreams)
        plan = dist_tiles.BandRenderPlan(scene, world, rank, cuts)
        if costs is not None:
            band_costs = plan.band_costs(costs)
        renderer = dist_tiles.BandGatherRenderer(
            plan, stream, dist_tiles.scene_band_renderer(scene), inflight=args.inflight,
            host_staging=host_staging, device=dev,
            # one-rank rehearsal: rank 0's band through a real RCCL self send / receive
            self_exchange=args.gather_rehearsal and world == 1,
            render_records=dist_tiles.scene_band_renderer(scene, True) if records else None,
            resolve=dist_tiles.scene_row_resolver(scene) if records else None,
            streams=rstreams)
        renderer.resolve_frac = resolve_frac
        renderer.stream_set_ms = stream_ms
    elif tiled:
        layout = dist_tiles.TilePlan(scene, world, rank)
        # shares travel as 32-bit pixel records (a third of RGB's bytes) where the scene allows;
        # rank 0 shades them into the frame (rt_resolve_device)
        records = (not host_staging and args.exchange == "records"
                   and dist_tiles.records_ok(scene))
        renderer = dist_tiles.TileGatherRenderer(
            layout, stream, dist_tiles.scene_tile_renderer(scene, records), inflight=args.inflight,
            host_staging=host_staging, device=dev,
            untile=None if host_staging else dist_tiles.scene_tile_untiler(scene, layout, records),
            gather_stream=args.gather_stream,
            render_inplace=None if (host_staging or args.root_gather)
            else dist_tiles.scene_inplace_renderer(scene),
            # one-rank rehearsal: rank 0's share through a real RCCL self send / receive + untile
            self_exchange=args.gather_rehearsal and world == 1,
            tile_words=dist_tiles.TILE_RECORDS if records else dist_tiles.TILE_FLOATS)
    else:
        owners = dist_tiles.FrameOwners(n_cams, world, rank)
        sizes = [(scene.camera(c).width, scene.camera(c).height) for c in range(scene.num_cameras)]
        renderer = dist_tiles.FrameGatherRenderer(scene, owners, sizes, stream,
                                                  host_staging=host_staging,
                                                  inflight=args.inflight, device=dev)

    # device preconditioning: untimed steps for --precondition-ms of wall time before the
    # warm-up.  Five warm-up steps are 2 ms of GPU work, too short for the GPU to leave its idle
    # clock: the same 20 timed steps measured 0.431-0.441 ms per step after 5 warm-up steps and
    # 0.395-0.401 after 50 or 200 (profiles/r05/warmup_sweep.txt).  Its rays are not counted.
    pre_steps = 0
    if args.precondition_ms > 0:
        t_pre = time.perf_counter()
        while True:  # rounds of steps; with several ranks every rank runs as many as rank 0
            for _ in range(4 * renderer.inflight):
                renderer.step()
                pre_steps += 1
            renderer.finish()
            torch.cuda.synchronize()
            go = torch.tensor([float((time.perf_counter() - t_pre) * 1e3 < args.precondition_ms)],
                              dtype=torch.float64, device=coll_dev)
            if world > 1:
                dist.broadcast(go, 0)
            if go.item() == 0.0:
                break
        scene.collect_stats()  # (discard the preconditioning's rays)
    # warmup (also yields the per-step ray count from the device counters)
    for _ in range(args.warmup):
        renderer.step()
    renderer.finish()
    torch.cuda.synchronize()
    st = scene.collect_stats()
    rays_local = (st.primary_rays + st.shadow_rays + st.secondary_rays) / max(1, args.warmup)
    rays_step = torch.tensor([rays_local], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(rays_step)
    rays_step = float(rays_step.item())

    ev = None if not args.step_events else [
        (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for _ in range(args.steps)]
    scene.read_kernel_times()  # discard
    # HIP events around each traversal kernel, on its stream
    scene.set_kernel_timing(args.kernel_timing)
    elapsed = timed_steps(renderer, args.steps, world, coll_dev, ev)
    scene.set_kernel_timing(False)
    kt, launches = scene.read_kernel_times()
    render_ms = [a.elapsed_time(b) for a, b in ev] if ev else [0.0]
    scene.collect_stats()  # reset counters

    verified = None
    t1_ms = None
    if use_pg and rank == 0:
        if not args.no_verify:
            # the gathered framebuffers must equal single-GPU renders of the same cameras
            verified = True
            for c, f in enumerate(renderer.frames):
                ref = torch.empty_like(f)
                scene.render_device(c, ref.data_ptr(), stream=stream.cuda_stream)
                torch.cuda.synchronize()
                verified &= bool(torch.equal(ref.view(torch.int32), f.view(torch.int32)))
            log(f"[rank 0] gathered frames bit-identical to single-GPU renders: {verified}")
        if strong:
            # t1: the same job rendered by this GPU alone, in place, as the N = 1 bench renders
            # it (its frames in flight, a picked stream set)
            one_streams, _ = dist_tiles.pick_render_streams(scene, INFLIGHT_N1, 1, device=dev)
            one = dist_tiles.FrameRenderer(scene, stream, inflight=INFLIGHT_N1,
                                           streams=one_streams)
            for _ in range(max(1, args.warmup)):
                one.step()
            one.finish()
            t1_ms = timed_steps(one, args.steps, 1, coll_dev) / args.steps * 1e3
            scene.collect_stats()
    weak = None
    if world > 1 and strong and not args.no_weak:
        # extra: weak scaling, one whole frame per rank per step (camera 0 everywhere)
        owners = dist_tiles.FrameOwners(world, world, rank)
        c0 = scene.camera(0)
        wr = dist_tiles.FrameGatherRenderer(
            scene, owners, [(c0.width, c0.height)] * world, stream, host_staging=host_staging,
            inflight=args.inflight, device=dev,
            render=lambda c, out, s: scene.render_device(0, out.data_ptr(), stream=s.cuda_stream))
        for _ in range(args.warmup):
            wr.step()
        wr.finish()
        el_w = timed_steps(wr, args.steps, world, coll_dev)
        scene.collect_stats()
        weak = {"value": round(world * rays_step / n_cams * args.steps / el_w / 1e6, 2),
                "unit": "Mrays/s", "ms_per_step": round(el_w / args.steps * 1e3, 4),
                "frames_per_step": world,
                "parallelism": f"frames{world}+{'rccl' if coll_dev == 'cuda' else 'gloo'}_gather",
                "note": "one whole frame per rank per step, gathered to rank 0 (weak scaling)"}
    if world > 1:
        dist.barrier()

    if rank == 0:
        value = rays_step * args.steps / elapsed / 1e6
        threads, how = host_cores()
        roof = None
        if not args.no_roofline:
            try:
                # fraction of one frame's work in one launch (one rt_render_device call)
                share = rays_local / max(1.0, rays_step / n_cams) / max(1.0, launches / args.steps)
                prof = pmc_profile(args.workload) if world == 1 else None
                kt_iso, n_iso = isolated_kernel_times(scene, stream, max(3, args.steps // 2))
                roof = roofline_line(xml, world, share, kt, launches, prof, kt_iso, n_iso)
                roof["timed_launches"] = launches
                roof["stream_copy_GBps_measured"] = round(stream_copy_gbps(device), 1)
                bytes_ref, ostats = algorithmic_bytes(xml, threads)
                roof["ref_order_effective_GBps"] = round(
                    bytes_ref * n_cams / (elapsed / args.steps) / 1e9, 1)
                roof["ref_order_model"] = ("SURVEY §8(d): 32 B x box tests + 36 B x triangle "
                                           "tests + 16 B per hit + 12 B per pixel with the "
                                           "reference's own visit counts (no culling), over "
                                           "the step time; not a roofline (the kernel does not "
                                           "make those fetches)")
            except Exception as e:  # the checker must never hide the measurement
                log(f"roofline accounting failed: {e!r}")
        single = cold = None
        probe = probe_c4 = None
        if world == 1 and not use_pg:
            try:
                single = one_frame_ms(scene, stream, max(10, args.steps // 2))
                cold = cold_frame_ms(scene)
                if not args.no_share_probe:
                    # every efficiency is priced against this line's own N = 1 step
                    probe = share_probe(scene, stream, max(PROBE_STEPS, args.steps), args.inflight,
                                        exchange=args.exchange, split=args.split,
                                        streams=renderer.streams,
                                        inflight_n=args.split_inflight,
                                        t1_line_ms=elapsed / args.steps * 1e3)
                    if args.workload == "c3":
                        # the north star's 8-GPU configuration: C4 (3840x2160), same mesh; its
                        # t1 = the C4 frame's N = 1 steps timed here exactly as this line's
                        with ceng795_amd.Scene(scene_path("c4", 1), device=device,
                                               traversal=args.traversal) as s4:
                            c4_n1 = n1_steps(s4, stream, args.inflight, args.steps, args.warmup,
                                             args.precondition_ms, dev)
                            probe_c4 = share_probe(s4, stream, max(PROBE_STEPS, args.steps), args.inflight,
                                                   exchange=args.exchange, split=args.split,
                                                   streams=renderer.streams,
                                                   inflight_n=args.split_inflight,
                                                   t1_line_ms=c4_n1["ms_per_step"])
                            probe_c4["n1_line"] = c4_n1
            except Exception as e:
                log(f"one-frame / share probe failed: {e!r}")
        host_rate = None
        if world == 1:
            try:
                host_rate = host_buffer_rate(scene, rays_step / n_cams)
            except Exception as e:
                log(f"host-buffer rate failed: {e!r}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(xml, threads, how)
            except Exception as e:
                log(f"cpu baseline failed: {e!r}")
        dropin = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                dropin = dropin_ms(xml, threads)
            except Exception as e:
                log(f"drop-in timing failed: {e!r}")
        n, w, h, desc = WORKLOADS[args.workload]
        ms_step = elapsed / args.steps * 1e3
        comm = "rccl" if coll_dev == "cuda" else "gloo"
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            # N = 1 is the base of the default N > 1 run, the tile split of one frame (strong)
            "scaling": "strong" if (strong or world == 1) else "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": desc, "frame": f"{w}x{h}", "frames_per_step": n_cams,
                       "triangles": 2 * (n - 1) ** 2, "rays_per_step": int(rays_step),
                       "traversal": args.traversal,
                       "parallelism": (f"tiles{world}+{comm}_gather" if tiled else
                                       f"bands{world}+{comm}_p2p" if banded else
                                       f"frames{world}+{comm}_gather" if use_pg else "frames1"),
                       "frames_in_flight": renderer.inflight,
                       "render_stream_sets_ms": getattr(renderer, "stream_set_ms", None),
                       "dispatch": "heavy-first per XCD region; the primary kernel by the tile "
                                   "costs of the previous frame on its stream (warm order, "
                                   "DESIGN.md 4.8), every frame's rays all traced",
                       "gather_verified": verified,
                       "exchange": band_exchange_text(world, comm, renderer, band_costs)
                       if banded else None if not tiled else (
                           ("dist.gather (RCCL) of every rank's tile-major share, whole-frame untile"
                            if args.root_gather or host_staging else
                            "rank 0 in place + batch_isend_irecv (RCCL send / receive) of the other "
                            "ranks' shares, untile around rank 0's units" if world > 1 else
                            "one-rank rehearsal: rank 0's tile-major share through an RCCL self "
                            "send / receive pair (batch_isend_irecv), whole-frame untile")
                           + ("; shares as 32-bit pixel records (hit primitive + shadow bits, "
                              "4 B per pixel) shaded on rank 0 (rt_resolve_device)"
                              if renderer_records(renderer) else "; shares as fp32 RGB")),
                       "exchange_bytes_per_step": (exchange_bytes(renderer) if tiled else
                                                   band_bytes(renderer) if banded else None),
                       "render_ms_avg": round(sum(render_ms) / len(render_ms), 4) if ev else None,
                       "timed_region": "the steps alone: no timing events inside it (kernel "
                                       "and one-frame times are measured after it)",
                       "preconditioning": {"ms": args.precondition_ms, "steps": pre_steps,
                                           "note": "untimed steps before the warm-up: the "
                                                   "GPU's clock ramp"}},
            "roofline": roof, "cpu_baseline": cpu, "pcie_inclusive": host_rate,
            "dropin_ms": dropin,
        }
        if single is not None:
            line["one_frame_ms"] = single
            line["one_frame_Mrays_s"] = round(rays_step / n_cams / (single * 1e-3) / 1e6, 2)
            line["one_frame_note"] = ("one frame at a time on one stream, warm (the previous "
                                      "frame's tile costs order its primary work)")
        if cold is not None:
            line["cold_frame_ms"] = cold
            line["cold_frame_note"] = ("the first frame of camera 0 on a fresh stream (block "
                                       "order, nothing else in flight), median of 3 streams")
        if probe is not None:
            line["predicted_strong_scaling"] = probe
        if probe_c4 is not None:
            line["predicted_strong_scaling_c4"] = probe_c4
        if strong and t1_ms is not None:
            line["strong_scaling"] = {"t1_ms": round(t1_ms, 4), "tN_ms": round(ms_step, 4),
                                      "efficiency_t1_over_N_tN": round(t1_ms / (world * ms_step), 4)}
        if weak is not None:
            line["weak_scaling"] = weak
        if world == 1 and not use_pg and not args.no_c5:
            try:
                import bench_ppm
                c5 = bench_ppm.run(max(3, args.steps // 4), 1, not args.no_cpu_baseline)
                line["c5"] = {k: c5[k] for k in ("metric", "value", "unit", "ms_per_step",
                                                 "steps", "warmup", "config", "roofline")}
                line["c5"]["cpu_baseline"] = c5.get("cpu_baseline")
            except Exception as e:
                log(f"c5 sub-benchmark failed: {e!r}")
        print(json.dumps(line), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()
    scene.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
