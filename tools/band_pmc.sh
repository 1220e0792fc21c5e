set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/bpmc
mkdir -p $O
for w in "c4 2" "c4 8" "c3 8"; do
  set -- $w
  tag=$1_n$2
  timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/$tag/tcc -o run --output-format csv -- python3 tools/band_pmc.py render --workload $1 --n $2 > $O/$tag.meta.json 2> $O/$tag.tcc.log || { tail -20 $O/$tag.tcc.log; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/$tag/fetch -o run --output-format csv -- python3 tools/band_pmc.py render --workload $1 --n $2 > $O/$tag.meta2.json 2> $O/$tag.fetch.log || { tail -20 $O/$tag.fetch.log; exit 1; }
  python3 tools/band_pmc.py summary --workload $1 --n $2 --meta $O/$tag.meta.json --dirs $O/$tag/tcc $O/$tag/fetch > $O/$tag.json || exit 1
done
echo done
