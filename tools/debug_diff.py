"""Debug helper: where does the GPU frame differ from the oracle? (development tool)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import scenes, tempfile
import ceng795_amd
from oracle.cpu_ref import OracleScene
d = tempfile.mkdtemp()
name = sys.argv[1] if len(sys.argv) > 1 else "c1"
xml = scenes.write(name, d)
o = OracleScene(xml)
for mode in ["fast", "reference"]:
    with ceng795_amd.Scene(xml, traversal=mode) as s:
        for cam in range(s.num_cameras):
            ref, _ = o.render(cam, threads=8)
            got, _ = s.render_image(cam)
            bad = np.argwhere((got != ref).any(-1))
            print(mode, cam, "bad pixels:", len(bad))
            if len(bad):
                tiles = sorted(set((int(y) // 8) * ((got.shape[1] + 7) // 8) + int(x) // 8 for y, x in bad))
                print("  tiles:", tiles[:20], "parity:", sorted(set(t % 2 for t in tiles)))
                for y, x in bad[:8]:
                    print("  ", y, x, got[y, x], ref[y, x])
