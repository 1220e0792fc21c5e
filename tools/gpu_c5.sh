#!/bin/bash
# C5 on one GPU box: PPM GPU parity (incl. the full-size C5 test), counter passes of the C5
# bench (profiles/traffic_c5.json for this library build), kernel stats, then the C5 bench line.
#   tools/gpu_c5.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/c5}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ppm_gpu.py tests/test_full_configs_gpu.py -k "ppm or c5" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS="--workload c5" timeout -k 10 900 bash tools/pmc_passes.sh "$O/pmc" traffic insts sq > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
timeout -k 10 60 python3 tools/pmc_traffic.py --fetch "$O/pmc/fetch" --write "$O/pmc/write" --insts "$O/pmc/insts" --sq "$O/pmc/sq" --workload c5 --round r02 --lib ceng795_amd/lib/libceng795_ppm.so --out "$O/traffic_c5.json" > /dev/null || exit 1
cp "$O/traffic_c5.json" profiles/traffic_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
