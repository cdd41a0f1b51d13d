# Same-box A/B of ab/*.so with the driver's bench command (sponza, 20 steps) and the bunny C3 line:
# the GPU suite on each non-base build first.  Usage: bash scripts/gpu_r04_ab.sh TAG [rounds] [so...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04ab}; R=${2:-2}; shift 2; SOS=${@:-$(ls ab/*.so)}
O=gpurun_out/$T; mkdir -p $O
for so in $SOS; do
  n=$(basename $so .so)
  [ "$n" = base ] && continue
  WGT_LIB_PATH=$PWD/$so timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.log)"
done
for r in $(seq $R); do
  for so in $SOS; do
    n=$(basename $so .so)
    for sc in sponza bunny; do
      st=20; [ $sc = bunny ] && st=30
      WGT_LIB_PATH=$PWD/$so timeout -k 10 600 python bench.py --scene $sc --steps $st --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_${n}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_${n}_${sc}_$r.log; exit 1; }
      echo "$n $sc r$r: $(tail -1 $O/bench_${n}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
    done
  done
done
