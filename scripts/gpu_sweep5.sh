#!/bin/bash
# Re-tune the persistent kernel's knobs (one process per scene).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep5}; mkdir -p $OUT
ENVS="${ENVS:-WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=14}"
for sc in ${SCENES:-bunny_1920_1080_64 sponza_1920_1080_16}; do
  REPS=3 timeout -k 10 400 python scripts/sweep_env.py $(echo $sc | tr _ " ") "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
done
