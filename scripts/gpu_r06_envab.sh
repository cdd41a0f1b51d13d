#!/bin/bash
# Same-box A/B of one environment setting (ENV_A vs ENV_B, e.g. "WGT_BVH_SIBLINGS=0"), alternating per
# round: the driver's bench command per scene, timing only.  PYK: a pytest -k parity subset run under
# ENV_B first (skipped when empty).  Usage: ENV_A=... ENV_B=... bash scripts/gpu_r06_envab.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06env}; R=${2:-2}; O=gpurun_out/$T; mkdir -p $O
if [ -n "$PYK" ]; then
  env $ENV_B timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$PYK" > $O/pytest_B.log 2>&1 || { tail -30 $O/pytest_B.log; exit 1; }
  echo "B: $(tail -1 $O/pytest_B.log)"
fi
for r in $(seq $R); do
  for v in A B; do
    if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
    for sc in ${SCENES:-sponza bunny}; do
      st=${STEPS:-12}; [ $sc = bunny ] && st=$((st + 8))
      env $E timeout -k 10 400 python bench.py --scene $sc --steps $st --warmup 3 --pmc off \
        --no-cpu-baseline --stats-reps 1 > $O/bench_${v}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_${v}_${sc}_$r.log; exit 1; }
      echo "$v($E) $sc r$r: $(tail -1 $O/bench_${v}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
    done
  done
done
echo done
