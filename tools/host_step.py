#!/usr/bin/env python3
"""Host cost of one bench step: the Python/driver time to ENQUEUE a step of the in-place
renderer and of the N>1 tile-gather renderer (one-rank RCCL group, the --gather-rehearsal
path), against the GPU time per step.  If the enqueue time approaches the step time, the
exchange path is host-bound, and so would every rank of an N-GPU run be.

    python tools/host_step.py [--steps 60] [--inflight 4]

Prints one JSON line: per renderer, host ms per step spent in step() calls (no syncs inside
the loop) and wall ms per step once the GPU has drained; and a breakdown of the tile-gather
step (render calls, the gather + untile on the communication stream)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def measure(R, steps, torch):
    for _ in range(5):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        R.step()
    t1 = time.perf_counter()
    R.finish()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"host_ms_per_step": round((t1 - t0) / steps * 1e3, 4),
            "wall_ms_per_step": round((t2 - t0) / steps * 1e3, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--inflight", type=int, default=4)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    import ceng795_amd
    from ceng795_amd import dist_tiles
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench.free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    scene = ceng795_amd.Scene(bench.scene_path("c3", 1), device=0)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", 0)
    out = {}
    out["inplace"] = measure(dist_tiles.FrameRenderer(scene, stream, inflight=a.inflight),
                             a.steps, torch)
    layout = dist_tiles.TilePlan(scene, 1, 0)
    for label, untile, gs in (
            ("tile_gather_render_stream", dist_tiles.scene_tile_untiler(scene, layout), "render"),
            ("tile_gather_comm_stream", dist_tiles.scene_tile_untiler(scene, layout), "comm"),
            ("tile_gather_index_untile", None, "render"),
            ("tile_root_inplace", dist_tiles.scene_tile_untiler(scene, layout), "inplace")):
        R = dist_tiles.TileGatherRenderer(
            layout, stream, dist_tiles.scene_tile_renderer(scene), inflight=a.inflight,
            device=dev, untile=untile, gather_stream="render" if gs == "inplace" else gs,
            render_inplace=dist_tiles.scene_inplace_renderer(scene) if gs == "inplace" else None)
        out[label] = measure(R, a.steps, torch)
    out["inplace_again"] = measure(dist_tiles.FrameRenderer(scene, stream, inflight=a.inflight),
                                   a.steps, torch)
    # the pieces of one tile-gather step, host time only
    R = dist_tiles.TileGatherRenderer(layout, stream, dist_tiles.scene_tile_renderer(scene),
                                      inflight=a.inflight, device=dev,
                                      untile=dist_tiles.scene_tile_untiler(scene, layout),
                                      gather_stream="comm")
    for _ in range(5):
        R.step()
    R.finish()
    torch.cuda.synchronize()
    sh = layout.shares[0]
    t0 = time.perf_counter()
    for k in range(a.steps):
        R.render(sh, R._slot(k % R.inflight, sh), R.rstreams[k % R.inflight])
    t1 = time.perf_counter()
    with torch.cuda.stream(R.comm):
        for k in range(a.steps):
            R._gather(k % R.inflight, R.comm)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    out["pieces_host_ms"] = {"render_call": round((t1 - t0) / a.steps * 1e3, 4),
                             "gather_and_untile": round((t2 - t1) / a.steps * 1e3, 4)}
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
