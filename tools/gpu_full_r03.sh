#!/bin/bash
# Round-3 checkpoint on the GPU box: full GPU suite, smoke, default bench line (C3 + C5
# sub-object + CPU baselines), one-frame-at-a-time kernel stats, the N>1 path rehearsed with a
# one-rank RCCL group, and (optionally, $2 = pmc) the PMC passes for profiles/traffic_c3.json.
set -o pipefail
O=gpurun_out/${1:-full}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -1 $O/gpu_tests.out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.out 2>&1 || { tail -20 $O/smoke.out; exit 1; }
tail -2 $O/smoke.out
timeout -k 10 600 python3 -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c3.json').read().strip().splitlines()[-1])
r=d['roofline']; c=d.get('c5') or {}
print('c3', d['value'], d['ms_per_step'], 'kernel', r['kernel_ms_avg'], 'frac', r['frac'], r['other_kernels_ms_avg'], 'cpu', (d['cpu_baseline'] or {}).get('value'))
print('c5', c.get('value'), c.get('ms_per_step'), (c.get('roofline') or {}).get('kernel_ms_avg'), (c.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-c5 --inflight 1 > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
timeout -k 10 300 python3 -u bench.py --gather-rehearsal --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_rehearsal.json 2> $O/bench_rehearsal.err || { tail -20 $O/bench_rehearsal.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_rehearsal.json').read().strip().splitlines()[-1])
print('rehearsal', d['value'], d['config']['parallelism'], d['config']['gather_verified'])"
if [ "$2" = "pmc" ]; then
  bash tools/pmc_passes.sh $O/pmc traffic sq insts || exit 1
  python3 tools/pmc_traffic.py --fetch $O/pmc/fetch --write $O/pmc/write --insts $O/pmc/insts --sq $O/pmc/sq --round r03 --out $O/traffic_c3.json > /dev/null || exit 1
  echo "pmc summary written"
fi
