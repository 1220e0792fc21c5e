#!/bin/bash
# Round-5 first GPU call: new tests (binding, copy-gather ordering, stream-table cap, exchange
# rehearsals), the fused frame kernel's parity suite, the scaling A/B, wave timelines.
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_binding_gpu.py tests/test_gpu_multi.py \
  tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "binding or back_to_back or bounded or rehearsal" > $O/new_tests.log 2>&1
echo "new tests rc=$?"; tail -3 $O/new_tests.log
CENG795_LIB=fused timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/parity_fused.log 2>&1 || { tail -20 $O/parity_fused.log; exit 1; }
tail -2 $O/parity_fused.log
timeout -k 10 900 python3 -u tools/scale_probe.py base,fused --rounds 2 > $O/scale.json 2> $O/scale.err \
  || { tail -20 $O/scale.err; exit 1; }
tail -8 $O/scale.err
for L in timeline fusedtl; do
  for W in 1 8; do
    CENG795_LIB=$L timeout -k 10 120 python3 tools/timeline.py --world $W > $O/tl_${L}_w$W.json 2> $O/tl_${L}_w$W.err \
      || { tail -5 $O/tl_${L}_w$W.err; exit 1; }
  done
done
echo done
