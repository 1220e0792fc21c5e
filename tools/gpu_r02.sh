#!/bin/bash
# Round-2 GPU session: GPU tests, benches, kernel-trace stats and PMC passes on the shipping
# build.  Every GPU step has its own time limit and the chain stops at the first failure.
#   tools/gpu_r02.sh <outdir> [tests|bench|pmc|all]
set -o pipefail
O=${1:-gpurun_out/r02}
WHAT=${2:-all}
mkdir -p "$O"
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'; } > "$O/host_cpus.txt" 2>&1
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $name failed rc=$rc" >&2
    tail -30 "$O/$name.out" "$O/$name.err" >&2
    exit $rc
  fi
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  tail -3 "$O/gpu_tests.out" >&2
  step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  step bench_c3 400 python3 -u bench.py
  cat "$O/bench_c3.out" >&2
  step bench_c4 300 python3 -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline
  step bench_c5 400 python3 -u bench.py --workload c5 --steps 5 --warmup 1
  cat "$O/bench_c5.out" >&2
fi
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
  # one frame at a time, as the roofline's kernel times are taken (bench.py isolated_kernel_times)
  step prof_c3 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1
  step prof_c3_default 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3_default" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
  BENCH_ARGS="--inflight 1" step pmc 900 bash tools/pmc_passes.sh "$O/pmc" traffic insts sq sqc cycles
  step traffic 60 python3 tools/pmc_traffic.py --fetch "$O/pmc/fetch" --write "$O/pmc/write" --insts "$O/pmc/insts" --sq "$O/pmc/sq" --workload c3 --round r02 --out "$O/traffic_c3.json"
fi
echo "all steps done" >&2
