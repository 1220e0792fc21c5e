#!/usr/bin/env python3
"""Offline study of the cold-frame order (CPU only, development tool): how well the projected-
primitive count per tile (rt_api.hip cold_costs: each primitive weighted by 1 / |cos| of its
view angle, or unweighted) orders a C3 frame, replayed against measured per-tile times.

  python tools/cold_study.py [--costs profiles/r05/tile_cost_map_split_w1.npz]

The estimate is recomputed here in numpy for the C3 height field (tools/gen_scene.py, camera
through rt_camera_from_view); the measured map is a round-5 RT_TIMELINE run (primary + shadow
time per tile).  The replay: 2x1-tile units (one 2-wave workgroup, cost = its slower tile), the
frame's units cut into 16 chunks, chunk c to XCD c mod 8 (block order: 8 runs, one per XCD, as a
launch without an order list), each XCD a list schedule over `slots`
workgroup slots in the given order; prints each order's makespan (slowest XCD, model units) and
the estimate's correlation with the measured times."""
import argparse
import ctypes as C
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def estimate(n=708, width=1920, height=1080, weighted=True):
    import gen_scene as G
    from ceng795_amd import _lib
    V = np.array([[float(x) for x in ln.split()] for ln in G.heightfield_vertices(n)])
    T = np.array([[int(x) for x in ln.split()] for ln in G.heightfield_faces(n)]) - 1
    cam = _lib.rt_camera()
    F3 = C.c_float * 3
    assert _lib.lib().rt_camera_from_view(F3(0, 1.5, -5), F3(0, -1, 0), F3(0, 0, -1),
                                          (C.c_float * 4)(-0.9, 0.9, -0.5, 0.5), C.c_float(1.0),
                                          width, height, 1, C.byref(cam)) == 0
    e, tl = np.array(cam.e[:]), np.array(cam.top_left[:])
    su, sv = np.array(cam.s_u[:]), np.array(cam.s_v[:])
    D = V - e
    M = np.stack([D, np.broadcast_to(-su, D.shape), np.broadcast_to(sv, D.shape)], axis=2)
    lam, fx, fy = np.linalg.solve(M, np.broadcast_to(tl - e, D.shape)[..., None])[..., 0].T
    tx, ty = (width + 7) // 8, (height + 7) // 8
    ok = (lam[T] > 0).all(1) & (fx[T].max(1) >= 0) & (fy[T].max(1) >= 0) & \
        (fx[T].min(1) < width) & (fy[T].min(1) < height)
    x0 = np.clip(np.floor(fx[T].min(1) / 8).astype(int), 0, tx - 1)
    x1 = np.clip(np.floor(fx[T].max(1) / 8).astype(int), 0, tx - 1)
    y0 = np.clip(np.floor(fy[T].min(1) / 8).astype(int), 0, ty - 1)
    y1 = np.clip(np.floor(fy[T].max(1) / 8).astype(int), 0, ty - 1)
    w = np.ones(len(T))
    if weighted:  # 1 / |cos(normal, view direction)|, at most 20 (as cold_costs)
        nrm = np.cross(V[T[:, 0]] - V[T[:, 1]], V[T[:, 0]] - V[T[:, 2]])
        d = V[T].mean(1) - e
        cosv = np.abs((nrm * d).sum(1)) / (np.linalg.norm(nrm, axis=1) * np.linalg.norm(d, axis=1))
        w = 1.0 / np.maximum(cosv, 0.05)
    est = np.ones((ty, tx))
    for i in np.nonzero(ok)[0]:
        est[y0[i]:y1[i] + 1, x0[i]:x1[i] + 1] += w[i]
    return est


def replay(cost, key, slots=448, chunks=2):
    ty, tx = cost.shape
    U = np.maximum(cost[:, 0::2], cost[:, 1::2]).ravel()
    K = None if key is None else np.maximum(key[:, 0::2], key[:, 1::2]).ravel()
    n = len(U)
    cs = -(-n // (8 * chunks))
    worst = 0.0
    for x in range(8):
        units = [u for c in range(x, 8 * chunks, 8) for u in range(c * cs, min(n, (c + 1) * cs))]
        if K is not None:
            units.sort(key=lambda u: -K[u])
        h = [0.0] * slots
        end = 0.0
        for u in units:
            t = heapq.heappop(h) + U[u]
            end = max(end, t)
            heapq.heappush(h, t)
        worst = max(worst, end)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--costs", default=os.path.join(ROOT, "profiles/r05/tile_cost_map_split_w1.npz"))
    a = ap.parse_args()
    m = np.load(a.costs)
    cost = m["trace_primary_kernel"] + m["trace_shadow_kernel"]
    est, cnt = estimate(), estimate(weighted=False)
    print({"corr_weighted": round(float(np.corrcoef(est.ravel(), cost.ravel())[0, 1]), 3),
           "corr_count": round(float(np.corrcoef(cnt.ravel(), cost.ravel())[0, 1]), 3),
           "block_order": round(float(replay(cost, None, chunks=1)), 1),  # (one run per XCD)
           "count_order": round(float(replay(cost, cnt)), 1),
           "weighted_order": round(float(replay(cost, est)), 1),
           "measured_order": round(float(replay(cost, cost)), 1)})


if __name__ == "__main__":
    main()
