set -o pipefail
O=${1:-gpurun_out/s5_lpt}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in ${2:-1 t2 t3 t6}; do
  L=$v; E=1; [ $v = 1 ] && L=
  CENG795_PPM_LPT=$E CENG795_PPM_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v$r.json 2>$O/c5_$v$r.err || { tail -5 $O/c5_$v$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c5_$v$r.json')); print('$v', d['ms_per_step'], d['value'])"
done; done
CENG795_PPM_DIAG=2 timeout -k 10 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5d.json 2>$O/c5d.err && grep "ppm diag" $O/c5d.err | tail -1
