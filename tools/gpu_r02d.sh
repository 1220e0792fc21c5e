set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -2 $O/gpu_tests.out; grep "cull:" $O/gpu_tests.out
for m in fast cull fast cull; do timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --traversal $m > $O/bench_$m.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m',d['value'],d['ms_per_step'])"; done
