#!/usr/bin/env python3
"""Study of the C5 update pass's work (CPU, from the oracle's logged photon pass).

    python tools/ppm_list_study.py [--photons 10000000] [--segments 4,8,16,32]

The oracle (oracle/ppm_ref.cpp, ppmref_trace_photons_logged) replays the single-threaded
reference run and logs every deposit (position, normal, photon) and every update (hit point,
deposit).  From that this script reports, for the C5 scene:
  * the bucket-list design of ppm_kernels.hip: groups (hit points with one cell range), their
    list lengths, tiles of 3, and the (tile, deposit) filter reads it makes;
  * a per-hit-point gather design: the photon stream cut into S segments, each hit point
    collecting the segment's deposits within the radius it has at the segment start (a superset
    of its updates there, the radius only shrinks), found through a uniform grid of cell c:
    candidates, deposits visited (those in the cells its radius box overlaps), and the longest
    per-segment candidate chain (the serial gate of one hit point).
Analysis only; nothing here is used by the product or the tests.
"""
import argparse
import ctypes as C
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenes  # noqa: E402
from oracle import ppm_ref  # noqa: E402

ALPHA = np.float32(0.7)


def logged_run(photons):
    cache = f"/tmp/ppm_log_{photons}.npz"
    if os.path.exists(cache):
        z = np.load(cache)
        return {k: z[k] for k in z.files}
    with tempfile.TemporaryDirectory() as d:
        xml = scenes.write_c5(d)
        o = ppm_ref.OraclePPM(xml)
        w, h, _ = o.camera(0)
        o.eye_pass(0, seed=0)
        info = o.build_hash_grid(w, h)
        hps = o.hit_points()
        L = ppm_ref.lib()
        f = L.ppmref_trace_photons_logged
        f.restype = C.c_longlong
        f.argtypes = [C.c_void_p, C.c_ulonglong, C.c_longlong, C.c_longlong, C.c_void_p,
                      C.c_longlong, C.c_void_p, C.c_longlong, C.POINTER(C.c_longlong)]
        cap_d = int(photons * 1.3) + 1000
        cap_u = int(photons * 8) + 1000
        dep = np.zeros((cap_d, 8), np.float32)
        upd = np.zeros((cap_u, 2), np.int64)
        nu = C.c_longlong()
        t0 = time.time()
        nd = f(o._h, 0, 0, photons, dep.ctypes.data, cap_d, upd.ctypes.data, cap_u, C.byref(nu))
        print(f"logged {photons} photons: {nd} deposits, {nu.value} updates, {time.time()-t0:.1f} s",
              flush=True)
        assert nd <= cap_d and nu.value <= cap_u
        out = dict(dep=dep[:nd], upd=upd[:nu.value], hps=hps, info=np.array(info))
    np.savez(cache, **out)
    return out


def cells_of(x, bmin, scale):
    return np.abs(((x - bmin) * scale).astype(np.int32))


def bucket(ix, iy, iz, num_hash):
    a = ix.astype(np.uint32) * np.uint32(73856093)
    b = iy.astype(np.uint32) * np.uint32(19349663)
    c = iz.astype(np.uint32) * np.uint32(83492791)
    return (a ^ b ^ c) % np.uint32(num_hash)


def r2_table(r0, n):
    """r^2 after k updates (k < n): the reference's float recurrence (Scene.cpp:139-140)."""
    t = np.empty(n, np.float32)
    r2 = np.float32(r0 * r0)
    for k in range(n):
        t[k] = r2
        nf = np.float32(k) * ALPHA
        rr = np.float32((np.float64(nf + ALPHA)) / (np.float64(nf) + 1.0))
        r2 = np.float32(r2 * rr)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--photons", type=int, default=10_000_000)
    ap.add_argument("--segments", default="1,4,8,16,32")
    ap.add_argument("--cell", default="0.5,1.0")  # fine cell size in units of the segment's median r
    a = ap.parse_args()
    z = logged_run(a.photons)
    dep, upd, hps, info = z["dep"], z["upd"], z["hps"], z["info"]
    r0, scale = np.float32(info[0]), np.float32(info[1])
    bmin = info[2:5].astype(np.float32)
    H, D = hps.shape[0], dep.shape[0]
    num_hash = H
    pos = hps[:, 0:3]
    print(f"hit points {H}, deposits {D}, updates {upd.shape[0]}, r0 {r0:.3f}, cell {1/scale:.3f}")
    # ---- bucket-list design
    lo = cells_of((pos - r0), bmin, scale)
    hi = cells_of((pos + r0), bmin, scale)
    key = lo[:, 0].astype(np.int64) | lo[:, 1].astype(np.int64) << 16 | lo[:, 2].astype(np.int64) << 32 \
        | (hi - lo)[:, 0].astype(np.int64) << 48 | (hi - lo)[:, 1].astype(np.int64) << 53 \
        | (hi - lo)[:, 2].astype(np.int64) << 58
    gkeys, ginv, gsize = np.unique(key, return_inverse=True, return_counts=True)
    G = gkeys.shape[0]
    dcell = cells_of(dep[:, 0:3], bmin, scale)
    dbucket = bucket(dcell[:, 0], dcell[:, 1], dcell[:, 2], num_hash)
    bcount = np.bincount(dbucket, minlength=num_hash)
    glist = np.zeros(G, np.int64)
    first = np.zeros(G, np.int64)
    first[ginv[::-1]] = np.arange(H)[::-1]
    for g in range(G):
        h = first[g]
        bs = set()
        for iz in range(lo[h, 2], hi[h, 2] + 1):
            for iy in range(lo[h, 1], hi[h, 1] + 1):
                for ix in range(lo[h, 0], hi[h, 0] + 1):
                    bs.add(int(bucket(np.array([ix]), np.array([iy]), np.array([iz]), num_hash)[0]))
        glist[g] = sum(int(bcount[b]) for b in bs)
    tiles = (gsize + 2) // 3
    print(f"groups {G}: size p50 {np.median(gsize):.0f} max {gsize.max()}, tiles {tiles.sum()}, "
          f"list p50 {np.median(glist):.0f} max {glist.max()}, pairs {glist.sum()}, "
          f"(tile, deposit) reads {int((tiles * glist).sum())}")
    # ---- per-hit-point gather
    from scipy.spatial import cKDTree
    nupd = upd.shape[0]
    order = np.lexsort((upd[:, 1], upd[:, 0]))
    u_h, u_d = upd[order, 0], upd[order, 1]
    tab = r2_table(r0, 100000)
    hp_starts = np.searchsorted(u_h, np.arange(H + 1))
    for S in [int(s) for s in a.segments.split(",")]:
        bounds = np.linspace(0, D, S + 1).astype(np.int64)
        tot_c, tot_v, chain = 0, {c: 0 for c in a.cell.split(",")}, 0
        chain_sum = 0
        t0 = time.time()
        for s in range(S):
            b0, b1 = bounds[s], bounds[s + 1]
            # updates of each hit point before deposit b0
            n = np.array([np.searchsorted(u_d[hp_starts[h]:hp_starts[h + 1]], b0) for h in range(H)])
            r = np.sqrt(tab[np.minimum(n, tab.shape[0] - 1)].astype(np.float64))
            tree = cKDTree(dep[b0:b1, 0:3].astype(np.float64))
            cnt = np.array([len(x) for x in tree.query_ball_point(pos, r * (1 + 1e-6))])
            tot_c += int(cnt.sum())
            chain = max(chain, int(cnt.max()))
            chain_sum += int(cnt.max())
            rmed = float(np.median(r))
            for cs in a.cell.split(","):
                c = float(cs) * rmed
                # deposits in the cells the radius box overlaps: box [p - r - c, p + r + c] (upper bound)
                cnt_v = np.array([len(x) for x in tree.query_ball_point(pos, r + c, p=np.inf)])
                tot_v[cs] += int(cnt_v.sum())
        print(f"segments {S:3d}: candidates {tot_c} ({tot_c/D:.1f}/deposit), longest chain {chain}, "
              f"sum of per-segment longest {chain_sum}, visited "
              + ", ".join(f"c={k}r: {v}" for k, v in tot_v.items()) + f"  ({time.time()-t0:.0f} s)",
              flush=True)


if __name__ == "__main__":
    main()
