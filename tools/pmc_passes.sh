#!/bin/bash
# Counter collection on the GPU box, one rocprofv3 --pmc pass per counter group (each with
# --kernel-trace only, as the pool requires).  Usage: tools/pmc_passes.sh <outdir> <group>...
# Groups: traffic (FETCH_SIZE, WRITE_SIZE, TCC hit/miss), sq (wave states), insts, sqc.
set -o pipefail
OUT=${1:?outdir}
shift
export TMPDIR=/tmp
mkdir -p "$OUT"
CMD="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline --no-c5 --no-share-probe --inflight 1 ${BENCH_ARGS:-}"
run() {
  local name=$1
  shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv \
    -- $CMD > "$OUT/$name.log" 2>&1 || { echo "pass $name failed ($?)"; exit 1; }
}
for g in "$@"; do
  case $g in
    traffic)
      run fetch FETCH_SIZE
      run write WRITE_SIZE
      run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum ;;
    sq)
      run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC ;;
    insts)
      run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD \
        SQ_INST_CYCLES_SMEM SQ_INSTS_VALU_TRANS_F32 SQ_INSTS ;;
    sqc)
      run sqc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_HITS \
        SQC_ICACHE_MISSES SQC_TC_STALL SQC_DCACHE_BUSY_CYCLES SQC_TC_DATA_READ_REQ ;;
    sqcbusy)  # is the scalar data cache (node / prim fetches) the limiter?
      run sqcbusy SQC_DCACHE_BUSY_CYCLES SQC_DCACHE_INPUT_VALID_READYB SQC_DCACHE_REQ \
        SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_TC_STALL \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT ;;
    cycles)   # issue cycles by pipe
      run cycles SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VALU SQ_INSTS_SALU \
        SQ_INSTS_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE ;;
    *) echo "unknown group $g"; exit 2 ;;
  esac
done
echo "pmc passes done"
