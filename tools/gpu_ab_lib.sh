#!/bin/bash
# Same-box A/B of library variants (CENG795_LIB) and dispatch settings with tools/kt.py.
# usage: tools/gpu_ab_lib.sh <outdir> "<lib> <order> <probe>" ...   (lib "-" = shipping build)
set -o pipefail
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
export TMPDIR=/tmp
CFGS=("$@")
for rep in 1 2 3; do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    L=$1; [ "$L" = "-" ] && L=""
    CENG795_LIB=$L CENG795_RT_ORDER=$2 CENG795_RT_PROBE=$3 timeout -k 10 120 python3 tools/kt.py > $O/one.json 2>> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/one.json'));d['lib']='$1';print(json.dumps(d))" | tee -a $O/kt.jsonl
  done
done
