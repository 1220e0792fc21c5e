#!/bin/bash
# PPM photon-batch A/B on one GPU box: parity with the default budget and with 1 MB batches
# (many batches per photon pass), then C5 timings: 8 GiB batches (two per step) vs default.
set -o pipefail
O=${1:-gpurun_out/ppm_batch}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CENG795_PPM_SLOT_MB=1 timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests_1mb.log 2>&1 || { tail -30 $O/tests_1mb.log; exit 1; }
tail -1 $O/tests_1mb.log
for r in 1 2; do for v in 8192 0; do
  CENG795_PPM_SLOT_MB=$v timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v$r.json 2>$O/c5_$v$r.err || { tail -5 $O/c5_$v$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c5_$v$r.json')); print('$v', d['ms_per_step'], d['value'])"
done; done
