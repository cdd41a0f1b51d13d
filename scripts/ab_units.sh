#!/bin/bash
# Same-box A/B of ab/*.so with WGT_PQ_UNITS values (sample-unit rounds), alternating, fresh processes.
#   bash scripts/ab_units.sh <outdir> "<units list>" "<scene W H spp;...>" [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-abu}; mkdir -p $OUT
UNITS=${2:-"1 4"}; R=${4:-2}
IFS=';' read -ra SCS <<< "${3:-sponza 1920 1080 256;bunny 1920 1080 256}"
for r in $(seq $R); do
  for so in ab/*.so; do
    for u in $UNITS; do
      for sc in "${SCS[@]}"; do
        echo -n "$(basename $so .so)-u$u r$r $sc " | tee -a $OUT/ab.log
        WGT_PQ_UNITS=$u WGT_LIB_PATH=$PWD/$so SWEEP_ONLY=2 timeout -k 10 300 python scripts/sweep_wf.py $sc 2>&1 | grep WGT_KERNEL | tee -a $OUT/ab.log || exit 1
      done
    done
  done
done
