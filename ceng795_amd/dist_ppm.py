"""Progressive photon mapping over GPUs with one process per GPU ("PPM photons
shard freely, but the hit-point flux state is shared").

The reference's T threads share every hit point under a per-hit-point mutex
(PPM/src/Scene.cpp:131-168, PPM/include/Hit_point.h:22).  Here each rank owns a shard of the hit
points instead: every rank runs the eye pass, the hash grid and the whole photon sequence on its
GPU, and applies the update pass to its own shard only (ppm_set_update_shard(rank, world): the
grid's update tiles dealt round-robin).  A hit point's result depends on no other hit point, so
each shard's values are the one-GPU values bit for bit; rank 0 gathers the ranks' (flux, r^2, n)
arrays (one torch.distributed gather: RCCL over xGMI for "nccl", host memory for "gloo"), takes
every hit point from its owner (merge_shard_states) and runs the density estimation.  The C ABI
offers the same split in one process (ppm_scene_load_xml_multi).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .ppm import merge_shard_states


def gather_merged_state(state: np.ndarray, owners: np.ndarray, device: str = "cpu",
                        group=None) -> Optional[np.ndarray]:
    """Every rank passes its hit-point state (n x 5 float32, ppm hit_state()) after its
    sharded update pass and the owner map (hit_point_shards(), identical on every rank);
    rank 0 receives the merged state, the other ranks None.  `device`: where the collective's
    tensors live ("cuda" for the nccl backend)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = torch.from_numpy(np.ascontiguousarray(state, np.float32)).to(device)
    if world == 1:
        return merge_shard_states([t.cpu().numpy()], owners)
    if rank == 0:
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t, bufs, dst=0, group=group)
        return merge_shard_states([b.cpu().numpy() for b in bufs], owners)
    dist.gather(t, dst=0, group=group)
    return None


def photons_and_normaliser(per_iteration: int, iterations: int, height: int, threads: int):
    """PPM/src/main.cpp:72-98 on `threads` host threads: photons traced, normaliser P*(P/T)*T
    (the same rule ppm_render applies)."""
    per_thread = per_iteration // threads
    traced = per_iteration * iterations if height < threads else per_thread * iterations * threads
    return traced, per_iteration * per_thread * threads


def render_sharded(scene, camera: int = 0, reference_threads: int = 8, device: str = "cpu",
                   group=None):
    """One PPM frame of `scene` (a ceng795_amd.ppm.PhotonScene on this rank's GPU) with the
    update pass sharded over the process group.  Returns (image or None, photons traced): the
    image on rank 0 only."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    scene.set_update_shard(rank, world)
    cam = scene.camera(camera)
    scene.eye_trace_lines(camera)
    scene.build_hash_grid(cam.width, cam.height)
    P, I, _ = scene.settings()
    traced, normaliser = photons_and_normaliser(P, I, cam.height, reference_threads)
    scene.trace_photons(0, traced)
    merged = gather_merged_state(scene.hit_state(), scene.hit_point_shards(), device, group)
    if merged is None:
        return None, traced
    scene.write_hit_state(merged)
    return scene.density_estimation(normaliser, camera), traced
