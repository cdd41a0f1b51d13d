#!/bin/bash
# GPU parity tests (working-tree tests) against every ab/*.so but base.so, then the same-box A/B timing.
#   bash scripts/gpu_ab_all.sh <tag> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
for so in ab/*.so; do
  [ "$(basename $so)" = base.so ] && continue  # HEAD: its own tests ran when it was committed
  n=$(basename $so .so)
  WGT_LIB_PATH=$PWD/$so timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$n.log 2>&1; rc=$?
  echo "$n: $(tail -1 $OUT/pytest_$n.log)"
  [ $rc -eq 0 ] || { tail -30 $OUT/pytest_$n.log; exit $rc; }
done
REPS=${REPS:-3} bash scripts/ab_run.sh ${1:-ab} ${2:-1}
