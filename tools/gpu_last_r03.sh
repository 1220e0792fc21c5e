#!/bin/bash
# Last check of the round-3 tree on one GPU box: the whole GPU suite, smoke, the default bench line.
set -o pipefail
O=gpurun_out/${1:-last}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -30 $O/gpu_tests.out; exit 1; }
tail -1 $O/gpu_tests.out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.out 2>&1 || { tail -20 $O/smoke.out; exit 1; }
tail -2 $O/smoke.out
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['c5']
print('c3', d['value'], d['ms_per_step'], r['frac'], r['traffic'], 'c5', c['value'], c['roofline']['bound'], c['roofline']['traffic'])"
