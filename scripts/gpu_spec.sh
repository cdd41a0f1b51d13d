#!/bin/bash
# Speculative-sample check: GPU parity suite with speculation on for every render,
# then a guess-count sweep (single frames).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-spec}; mkdir -p $OUT
WGT_SPEC=4 timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > $OUT/pytest_gpu_spec4.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu_spec4.log
[ $rc -eq 0 ] || exit $rc
ENVS="WGT_SPEC=0;WGT_SPEC=2;WGT_SPEC=4;WGT_SPEC=6;WGT_SPEC=10;WGT_SPEC=0;WGT_SPEC=4"
for sc in bunny_1920_1080_256 sponza_1920_1080_64; do
  REPS=3 timeout -k 10 400 python scripts/sweep_env.py $(echo $sc | tr _ " ") "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
done
