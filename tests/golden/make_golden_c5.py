#!/usr/bin/env python3
"""Golden fixture for BASELINE config C5 at its configured size: the PPM Cornell box at
256x256 with PhotonCountPerIteration 10000 x NumberOfIterations 1000 (PPM/src/main.cpp:72-98,
1e7 photons), rendered by the CPU oracle (oracle/ppm_ref.cpp, pinned to the reference by
tests/test_ppm_oracle.py) exactly as ppm_render runs it: eye pass, hash grid, photons
[0, P/T*T*I) with T = 8 reference threads, density estimation with the P*(P/T)*T normaliser.

The single-threaded oracle needs about a minute for the 1e7-photon pass here, which is too long
to repeat inside a GPU test, so the result is committed as data: the sha256 of every hit
point's final (flux, r^2, n), of the frame and of the hit-point records, the pass statistics,
and a seeded sample of hit-point states / pixels for diagnosing a mismatch.

usage: python tests/golden/make_golden_c5.py      (writes tests/golden/golden_c5.{json,npz})
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import scenes  # noqa: E402
from oracle.ppm_ref import OraclePPM  # noqa: E402

SEED = 21
THREADS = 8
SAMPLES = 1024


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import tempfile
    d = tempfile.mkdtemp()
    xml = scenes.write_c5(d)
    o = OraclePPM(xml)
    t0 = time.time()
    frame, st = o.render(0, seed=SEED, threads=THREADS)
    dt = time.time() - t0
    state = o.hit_state()
    hps = o.hit_points()
    rng = np.random.default_rng(795)
    hp_idx = np.sort(rng.choice(state.shape[0], SAMPLES, replace=False))
    h, w, _ = frame.shape
    px_idx = np.sort(rng.choice(h * w, SAMPLES, replace=False))
    meta = {
        "scene": "C5: gen_ppm_scene.cornell(256, 256, photons=10000, iterations=1000)",
        "xml_sha256": hashlib.sha256(open(xml, "rb").read()).hexdigest(),
        "seed": SEED, "reference_threads": THREADS,
        "stats": st.as_dict(),
        "hit_points": int(state.shape[0]),
        "hit_points_sha256": sha(hps),
        "hit_state_sha256": sha(state),
        "frame_sha256": sha(frame),
        "oracle_seconds": round(dt, 1),
    }
    np.savez_compressed(os.path.join(HERE, "golden_c5.npz"), hp_idx=hp_idx,
                        hp_state=state[hp_idx], px_idx=px_idx,
                        px=frame.reshape(-1, 3)[px_idx])
    with open(os.path.join(HERE, "golden_c5.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
