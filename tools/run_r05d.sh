#!/bin/bash
# Round 5, fourth call: heavy-tile split (quadrant waves) — GPU suite, A/B against no split,
# timelines of a warm frame and a warm 1/8 share.
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 900 python3 -u tools/scale_probe.py base,nosplit --rounds 2 > $O/scale.json 2> $O/scale.err \
  || { tail -20 $O/scale.err; exit 1; }
tail -8 $O/scale.err
for W in 1 8; do
  CENG795_LIB=timeline timeout -k 10 120 python3 tools/timeline.py --world $W --save $O/map_w$W.npz \
    > $O/tl_w$W.json 2> $O/tl_w$W.err || { tail -5 $O/tl_w$W.err; exit 1; }
done
echo all done
