#!/bin/bash
# Round-2 closing run on one GPU box: C5 PMC traffic of this build (so the C5 bench line
# carries it), the GPU test suite, smoke, C3 / C5 / C4 benches and rocprofv3 kernel stats.
set -o pipefail
O=${1:-gpurun_out/r02_final4}; mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--workload c5" bash tools/pmc_passes.sh $O/pmc_c5 traffic || exit 1
python3 tools/pmc_traffic.py --fetch $O/pmc_c5/fetch --write $O/pmc_c5/write --workload c5 \
  --lib ceng795_amd/lib/libceng795_ppm.so --out profiles/traffic_c5.json > $O/traffic_c5.out 2>&1 || { tail -5 $O/traffic_c5.out; exit 1; }
cp profiles/traffic_c5.json $O/
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
echo done
