#!/bin/bash
# Instruction mix of the axis-aligned quad path against the default build (ab/base.so, ab/qaxis.so;
# DESIGN.md §4.2 item 22): one SQ pass each on one sponza frame, then the 64-spp bunny frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r04qm}; mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
for sc in sponza bunny; do
  for n in base qaxis; do
    WGT_LIB_PATH=$PWD/ab/$n.so timeout -s KILL 90 rocprofv3 --pmc $C -d $O/${n}_$sc -o run --output-format csv -- python bench.py --scene $sc --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline --check off --pmc off --stats-reps 1 > $O/${n}_$sc.log 2>&1 || { echo "pmc $n $sc failed"; tail -5 $O/${n}_$sc.log; exit 1; }
  done
done
echo done
