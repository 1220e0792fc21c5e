#!/usr/bin/env python3
"""Development check of the traversal build in CENG795_LIB: renders a few scenes once, prints
time, ray counts and the shared-piece counter, and compares the frame with the oracle."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenes  # noqa: E402
import ceng795_amd  # noqa: E402
from oracle.cpu_ref import OracleScene  # noqa: E402

d = tempfile.mkdtemp()
for name in sys.argv[1:] or ["soup_small", "hf_side", "c2"]:
    xml = scenes.write(name, d)
    ref, rst = OracleScene(xml).render(0, threads=16)
    with ceng795_amd.Scene(xml) as s:
        s.debug_counters()
        t = time.time()
        img, st = s.render_image(0)
        dt = time.time() - t
        bad = int((img.view(np.uint32) != ref.view(np.uint32)).any(-1).sum())
        print(f"{name}: {dt:.3f} s, rays {st.primary_rays}+{st.shadow_rays} (oracle "
              f"{rst.primary_rays}+{rst.shadow_rays}), hits {st.primary_hits} "
              f"(oracle {rst.primary_hits}), {bad} pixels differ", flush=True)
