#!/bin/bash
# Per-kernel times of the C5 photon pass for lib/libceng795_ppm_<v>.so variants ("new" = the
# production build): rocprofv3 --kernel-trace --stats over bench.py --workload c5.
#   tools/ppm_prof.sh <outdir> [variants, default "new"]
set -o pipefail
O=${1:-gpurun_out/ppm_prof}; mkdir -p $O
export TMPDIR=/tmp
for v in ${2:-new}; do
  L=$v; [ $v = new ] && L=
  CENG795_PPM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$v.out 2>&1 || { tail -20 $O/prof_$v.out; exit 1; }
  echo "== $v"
  python3 -c "
import csv
rows = sorted(csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:12]:
    print('%-60s %5s %9.1f us avg %8.2f ms total' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))"
done
