#!/bin/bash
# Re-tune the persistent kernel's knobs (one process per scene).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep5}; mkdir -p $OUT
ENVS="${ENVS:-WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=14}"
for sc in "bunny 1920 1080 64" "sponza 1920 1080 16"; do
  REPS=3 timeout -k 10 400 python scripts/sweep_env.py $sc "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
done
