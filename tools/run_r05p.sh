#!/bin/bash
# Round 5: rehearsals with the default record-band exchange, smoke.
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_full_configs_gpu.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "rehearsal" > $O/rehearsal.log 2>&1 || { tail -30 $O/rehearsal.log; exit 1; }
tail -1 $O/rehearsal.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 -u bench.py --gather-rehearsal --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/rehearsal_c3.json 2> $O/rehearsal_c3.err || { tail -20 $O/rehearsal_c3.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/rehearsal_c3.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['gather_verified'], d['config']['exchange'])"
