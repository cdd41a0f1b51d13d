#!/bin/bash
# GPU parity tests on the working tree, then same-box A/B of ab/*.so.
#   bash scripts/gpu_ab.sh <tag> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
REPS=${REPS:-3} bash scripts/ab_run.sh ${1:-ab} ${2:-1}
