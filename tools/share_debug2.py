import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
import numpy as np, scenes, ceng795_amd
d = tempfile.mkdtemp()
for name in ["soup1", "c2", "c2", "graze_hf", "c2"]:
    xml = scenes.write(name, d)
    with ceng795_amd.Scene(xml) as s:
        for i in range(4):
            img, st = s.render_image(0)
            dc = s.debug_counters()
            print(name, i, st.primary_rays, st.shadow_rays, st.primary_hits, dc["shared_pieces"], flush=True)
