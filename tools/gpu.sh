#!/bin/bash
# One parameterised launcher for GPU-box steps (run under gpurun; each step has its own time
# limit and the caller chains steps with &&, so the first failure ends the call).
#
#   tools/gpu.sh <out> tests [pytest args]         pytest -m gpu (verbose, per-test timeout)
#   tools/gpu.sh <out> smoke                       __graft_entry__.smoke()
#   tools/gpu.sh <out> bench <name> [bench args]   one bench.py line -> <out>/<name>.json
#   tools/gpu.sh <out> stats <name> [bench args]   rocprofv3 --kernel-trace --stats of bench.py
#   tools/gpu.sh <out> ab <variants> [rounds]      same-box A/B of library builds (tools/ab.py)
#   tools/gpu.sh <out> kt <name> [kt args]         per-kernel HIP-event times (tools/kt.py)
#   tools/gpu.sh <out> pmc <workload> [round]      PMC traffic passes -> <out>/traffic_<w>.json
#   tools/gpu.sh <out> pmcg <name> <groups...>      other counter groups (tools/pmc_passes.sh:
#                                                  sq, insts, cycles, sqc, sqcbusy) of the C3 bench
#   tools/gpu.sh <out> work <name> [workload] [lib] traversal work counters (RT_DIAG build,
#                                                  tools/kernel_work.py; lib default "diag")
#   tools/gpu.sh <out> ppmab "<variants>" [rounds] C5 frames of lib/libceng795_ppm_<v>.so builds
#                                                  ("base" = the shipping one), interleaved
#   tools/gpu.sh <out> py <name> <script> [args]   any tools/ script -> <out>/<name>.json
#   tools/gpu.sh <out> ppmdiag <variant>           C5 per-phase update-pass counters of an exp
#                                                  build made with -DPPM_DIAG_LEVEL=2
#                                                  (-DPPM_PHASE_TIMERS=1 for the phase timers)
#
# <out> is a directory under gpurun_out/.
set -o pipefail
O=gpurun_out/${1:?out}; shift
CMD=${1:?command}; shift
mkdir -p "$O"
export TMPDIR=/tmp
case "$CMD" in
  tests)
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
      > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
    tail -3 "$O/tests.log" ;;
  smoke)
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
      || { tail -20 "$O/smoke.log"; exit 1; }
    tail -2 "$O/smoke.log" ;;
  bench)
    N=${1:?name}; shift
    timeout -k 10 600 python3 -u bench.py "$@" > "$O/$N.json" 2> "$O/$N.err" || { tail -20 "$O/$N.err"; exit 1; }
    tail -c 1500 "$O/$N.json" ;;
  stats)
    N=${1:?name}; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$N" -o run --output-format csv -- \
      python3 bench.py "$@" > "$O/$N.out" 2>&1 || { tail -20 "$O/$N.out"; exit 1; }
    f=$(find "$O/$N" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$O/${N}_kernel_stats.csv"
    head -12 "$O/${N}_kernel_stats.csv" | cut -c1-200 ;;
  ab)
    V=${1:?variants}; R=${2:-3}
    timeout -k 10 900 python3 tools/ab.py "$V" --rounds "$R" > "$O/ab.json" 2> "$O/ab.err" || { tail -20 "$O/ab.err"; exit 1; }
    cat "$O/ab.json" ;;
  kt)
    N=${1:?name}; shift
    timeout -k 10 300 python3 tools/kt.py "$@" > "$O/$N.json" 2> "$O/$N.err" || { tail -20 "$O/$N.err"; exit 1; }
    cat "$O/$N.json" ;;
  pmc)
    W=${1:-c3}; R=${2:-r04}
    BENCH_ARGS="--workload $W" bash tools/pmc_passes.sh "$O/pmc_$W" traffic insts sq || exit 1
    LIB=ceng795_amd/lib/libceng795_rt.so; [ "$W" = c5 ] && LIB=ceng795_amd/lib/libceng795_ppm.so
    python3 tools/pmc_traffic.py --fetch "$O/pmc_$W/fetch" --write "$O/pmc_$W/write" --workload "$W" \
      --insts "$O/pmc_$W/insts" --sq "$O/pmc_$W/sq" \
      --round "$R" --lib "$LIB" --out "$O/traffic_$W.json" || exit 1 ;;
  pmcg)
    N=${1:?name}; shift
    bash tools/pmc_passes.sh "$O/$N" "$@" || exit 1
    ls "$O/$N" ;;
  work)
    N=${1:?name}; W=${2:-c3}; L=${3:-diag}
    X=$(python3 -c "import bench; print(bench.scene_path('$W', 1))") || exit 1
    timeout -k 10 300 env CENG795_LIB=$L python3 tools/kernel_work.py "$X" > "$O/$N.json" 2> "$O/$N.err" \
      || { tail -20 "$O/$N.err"; exit 1; }
    cat "$O/$N.json" ;;
  py)
    N=${1:?name}; S=${2:?script}; shift 2
    timeout -k 10 600 python3 -u "$S" "$@" > "$O/$N.json" 2> "$O/$N.err" || { tail -20 "$O/$N.err"; exit 1; }
    tail -c 2000 "$O/$N.json" ;;
  ppmab)
    V=${1:?variants}; R=${2:-2}
    for r in $(seq "$R"); do for v in $V; do
      L=$v; [ "$v" = base ] && L=
      CENG795_PPM_LIB=$L timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 \
        --no-cpu-baseline > "$O/c5_$v$r.json" 2> "$O/c5_$v$r.err" || { tail -5 "$O/c5_$v$r.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$O/c5_$v$r.json')); print('$v', d['ms_per_step'], d['value'], d['roofline']['kernel_ms_avg'])"
    done; done ;;
  ppmdiag)
    V=${1:?variant}
    CENG795_PPM_LIB=$V timeout -k 10 200 python3 -u bench.py --workload c5 --steps 1 --warmup 1 \
      --no-cpu-baseline > "$O/c5d_$V.json" 2> "$O/c5d_$V.err" || { tail -5 "$O/c5d_$V.err"; exit 1; }
    grep "ppm diag" "$O/c5d_$V.err" | tail -1 ;;
  *)
    echo "unknown command $CMD" >&2; exit 2 ;;
esac
