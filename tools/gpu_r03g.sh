#!/bin/bash
# PPM GPU tests + probe estimator study + 2-wave workgroup A/B
set -o pipefail
mkdir -p gpurun_out/r03g
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_ppm_gpu.py tests/test_full_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/ppm_tests.out 2>&1 || { tail -30 gpurun_out/r03g/ppm_tests.out; exit 1; }
tail -1 gpurun_out/r03g/ppm_tests.out
bash tools/gpu_probe_est.sh r03f || exit 1
bash tools/gpu_ab_lib.sh r03g/ab "- 2 0" "w2 2 0" "- 2 1" "w2 2 1"
