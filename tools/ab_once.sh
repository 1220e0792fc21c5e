set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 600 python3 tools/ab.py base,nocull --rounds 5 > $O/ab_nocull.json 2> $O/ab.err || exit 1
cat $O/ab_nocull.json
CENG795_LIB=nocull_diag timeout -k 10 120 python3 tools/kernel_work.py scenes/bench_c3_1cam.xml > $O/work_nocull.json 2>$O/w1.err || { tail $O/w1.err; exit 1; }
CENG795_LIB=diag timeout -k 10 120 python3 tools/kernel_work.py scenes/bench_c3_1cam.xml > $O/work_base.json 2>$O/w2.err || exit 1
cat $O/work_nocull.json $O/work_base.json
