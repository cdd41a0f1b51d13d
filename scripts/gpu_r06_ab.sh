# Round 6 same-box A/B of ab/*.so (each loaded through WGT_LIB_PATH), alternating builds per round:
# the driver's bench command per scene, timing only.  PYK: a pytest -k parity subset run on each
# build first (skipped when empty).  Usage: bash scripts/gpu_r06_ab.sh TAG [rounds]
#   SCENES="sponza bunny" STEPS=12
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06ab}; R=${2:-2}; O=gpurun_out/$T; mkdir -p $O
if [ -n "$PYK" ]; then
  for so in ab/*.so; do
    n=$(basename $so .so)
    WGT_LIB_PATH=$PWD/$so timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "$PYK" > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 1; }
    echo "$n: $(tail -1 $O/pytest_$n.log)"
  done
fi
for r in $(seq $R); do
  for so in ab/*.so; do
    n=$(basename $so .so)
    for sc in ${SCENES:-sponza bunny}; do
      st=${STEPS:-12}; [ $sc = bunny ] && st=$((st + 8))
      WGT_LIB_PATH=$PWD/$so timeout -k 10 400 python bench.py --scene $sc --steps $st --warmup 3 --pmc off \
        --no-cpu-baseline --stats-reps 1 > $O/bench_${n}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_${n}_${sc}_$r.log; exit 1; }
      echo "$n $sc r$r: $(tail -1 $O/bench_${n}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
    done
  done
done
echo done
