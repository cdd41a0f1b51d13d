#!/bin/bash
# L2 request-size calibration (scripts/l2_calib.py under one TCC PMC pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-l2cal}; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/pmc -o run --output-format csv -- python scripts/l2_calib.py > $OUT/l2cal.log 2>&1 || { tail -20 $OUT/l2cal.log; exit 1; }
tail -2 $OUT/l2cal.log
