#!/bin/bash
# PMC passes over C5 (one rocprofv3 --pmc pass per counter group, --kernel-trace only) for
# lib/libceng795_ppm_<v>.so variants ("new" = the shipping build); prints the update kernel's
# counters per launch.   tools/ppm_pmc.sh <outdir> "<variants>"
set -o pipefail
O=${1:?outdir}; mkdir -p $O
export TMPDIR=/tmp
for v in ${2:-new}; do
  L=$v; [ $v = new ] && L=
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    CENG795_PPM_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $O/${v}_p$i -o run --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 $O/${v}_p$i.log; exit 1; }
  done
  python3 - $O $v <<'PY'
import csv, glob, sys, collections
O, v = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(f"{O}/{v}_p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if 'group_update' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(v, {k: round(sum(x) / len(x) / 1e6, 2) for k, x in sorted(acc.items())}, '(M per dispatch-row avg)')
PY
done
