#!/bin/bash
# Round 5, fifth call: split tuning A/B (C3 shares), C4 with / without split.
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/scale_probe.py base,sd8,sd8b9,sd4b8,splitall,nosplit --rounds 2 --workloads c3 \
  > $O/scale_c3.json 2> $O/scale_c3.err || { tail -20 $O/scale_c3.err; exit 1; }
tail -12 $O/scale_c3.err
timeout -k 10 600 python3 -u tools/scale_probe.py base,splitall --rounds 1 --workloads c4 \
  > $O/scale_c4.json 2> $O/scale_c4.err || { tail -20 $O/scale_c4.err; exit 1; }
tail -2 $O/scale_c4.err
echo all done
