#!/bin/bash
# Quick GPU check: full GPU test suite, C3 bench, kernel stats one frame at a time.
set -o pipefail
O=gpurun_out/${1:-quick}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -1 $O/gpu_tests.out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_c3.json').read().strip().splitlines()[-1]);print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['other_kernels_ms_avg'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $O/prof.out 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
