#!/bin/bash
# Region chunking of the per-XCD heavy-first order (CENG795_RT_ORDER_CHUNKS: chunks per XCD
# region, 0 = half rows): kernel times (tools/kt.py, 3 interleaved reps) and the traversal
# kernels' FETCH_SIZE (one pass each).
set -o pipefail
O=gpurun_out/${1:-chunks}; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 0 1 2 4; do
    CENG795_RT_ORDER_CHUNKS=$c timeout -k 10 120 python3 tools/kt.py > $O/one.json 2>> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/one.json'));d['chunks']=$c;print(json.dumps(d))" | tee -a $O/kt.jsonl
  done
done
for c in 0 1 2 4; do
  CENG795_RT_ORDER_CHUNKS=$c timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch_c$c -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline --no-c5 --inflight 1 > $O/fetch_c$c.log 2>&1 || { tail -5 $O/fetch_c$c.log; exit 1; }
  python3 - <<PY
import sys; sys.path.insert(0, 'tools')
from pmc_traffic import per_kernel
v, n = per_kernel('$O/fetch_c$c')
print('chunks $c', {k: round(2 * x['FETCH_SIZE'] * 1024 / 1e6, 1) for k, x in v.items()}, 'MB read per launch')
PY
done
