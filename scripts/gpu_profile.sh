#!/bin/bash
# GPU profiling run: bench line, rocprofv3 kernel trace + stats, and separate PMC
# passes (never combined with sys/runtime traces).  Usage: bash scripts/gpu_profile.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-prof}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BARGS="$@"
echo "== bench"; timeout -k 10 600 python bench.py --steps 3 --warmup 1 $BARGS > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline $BARGS > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -20 $OUT/kt.log; exit 1; }
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  echo "== pmc $C"
  timeout -k 10 600 rocprofv3 --pmc $C -d $OUT/pmc_$N -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline $BARGS > $OUT/pmc_$N.log 2>&1 || { echo "pmc $C failed"; tail -20 $OUT/pmc_$N.log; exit 1; }
done
find $OUT -name "*.csv" | head -20
echo done
