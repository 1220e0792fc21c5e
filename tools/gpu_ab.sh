#!/bin/bash
# Same-box A/B of library variants (tools/ab.py), optionally after the GPU parity tests.
#   tools/gpu_ab.sh <outdir> <variants> [rounds] [tests]
set -o pipefail
O=${1:?outdir}; V=${2:?variants}; R=${3:-3}
mkdir -p "$O"
if [ "${4:-}" = tests ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.out" 2>&1 || { tail -30 "$O/gpu_tests.out"; exit 1; }
  tail -2 "$O/gpu_tests.out"
fi
timeout -k 10 900 python3 -u tools/ab.py "$V" --rounds "$R" ${AB_ARGS:-} > "$O/ab.json" 2> "$O/ab.err" || { tail -30 "$O/ab.err"; exit 1; }
cat "$O/ab.json"
