#!/bin/bash
# On the GPU box: time every ab/*.so on the same scenes, alternating, in fresh processes.
# AB_SCENES='scene W H spp;...' overrides the scene list.
#   bash scripts/ab_run.sh <outdir> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT; R=${2:-2}
for r in $(seq $R); do
  for so in ab/*.so; do
    IFS=';' read -ra SCS <<< "${AB_SCENES:-bunny 1920 1080 64;sponza 1920 1080 16}"
    for sc in "${SCS[@]}"; do
      echo -n "$(basename $so) r$r $sc " | tee -a $OUT/ab.log
      WGT_LIB_PATH=$PWD/$so SWEEP_ONLY=${SWEEP_ONLY:-2} timeout -k 10 300 python scripts/sweep_wf.py $sc 2>&1 | tee -a $OUT/ab.log || exit 1
    done
  done
done
