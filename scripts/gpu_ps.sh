#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ps}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
SWEEP_ONLY=${SWEEP_ONLY:-1,2,0} timeout -k 10 600 python scripts/sweep_wf.py bunny > $OUT/sweep_bunny.log 2>&1 || { tail $OUT/sweep_bunny.log; exit 1; }
cat $OUT/sweep_bunny.log
SWEEP_ONLY=${SWEEP_ONLY:-1,2,0} timeout -k 10 600 python scripts/sweep_wf.py sponza 1920 1080 16 > $OUT/sweep_sponza.log 2>&1 || { tail $OUT/sweep_sponza.log; exit 1; }
cat $OUT/sweep_sponza.log
