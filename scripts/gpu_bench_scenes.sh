#!/bin/bash
# One bench line per scene (short): bash scripts/gpu_bench_scenes.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-scenes}
mkdir -p $OUT
for S in bunny sponza cornell; do
  timeout -k 10 300 python bench.py --scene $S --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_$S.log 2>&1 || { echo "bench $S failed"; tail -20 $OUT/bench_$S.log; exit 1; }
  tail -1 $OUT/bench_$S.log
done
