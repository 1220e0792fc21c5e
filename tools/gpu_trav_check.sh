#!/bin/bash
# Traversal check: a C2 canary render under a short limit, the parity suites, the
# occupancy timeline and a same-box A/B of library variants (AB_VARIANTS, default base,noshare).
set -o pipefail
O=gpurun_out/${1:-r02g}; mkdir -p $O
timeout -k 10 120 python3 -u -c "
import sys, time; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import torch, bench, ceng795_amd
xml = bench.scene_path('c2', 1)
with ceng795_amd.Scene(xml) as s:
    for i in range(3):
        t = time.time(); img, st = s.render_image(0); print('c2 render', i, round(time.time() - t, 3), 's', st.rays(), flush=True)
    print(s.debug_counters(), flush=True)
" > $O/canary.out 2>&1 || { cat $O/canary.out; exit 1; }
cat $O/canary.out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_configs_gpu.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -2 $O/gpu_tests.out
CENG795_LIB=timeline timeout -k 10 200 python3 tools/timeline.py --save $O/tile_us.npz > $O/timeline.json || exit 1
python3 -c "import json; d=json.load(open('$O/timeline.json')); [print(k, {a:b for a,b in v.items() if a!='resident_waves_by_time'}, v['resident_waves_by_time']) for k,v in d.items()]"
timeout -k 10 600 python3 -u tools/ab.py ${AB_VARIANTS:-base,noshare} --rounds 3 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab.json
