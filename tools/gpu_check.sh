#!/bin/bash
# One GPU validation pass (run on the box through gpurun): GPU tests, smoke, the headline
# bench line and, optionally, the packet-level traversal counters of the RT_DIAG build.
#   tools/gpu_check.sh <outdir> [diag]
set -o pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -5 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ "$2" = diag ]; then
  CENG795_LIB=diag timeout -k 10 300 python -u tools/diag.py counters > "$OUT/diag.json" 2>&1 \
    || { echo "diag failed"; exit 1; }
fi
echo "gpu check done"
