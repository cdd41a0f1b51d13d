# The cost pre-pass's path depth (WGT_PQ_DEPTH) on the driver's sponza command and the bunny C3 line,
# rounds alternating the settings.  Usage: bash scripts/gpu_r04_pqdepth.sh TAG [rounds] [depths...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04pq}; R=${2:-3}; shift 2; DS=${@:-50 16 12 8 6}
O=gpurun_out/$T; mkdir -p $O
for r in $(seq $R); do
  for d in $DS; do
    for sc in sponza bunny; do
      st=20; [ $sc = bunny ] && st=30
      WGT_PQ_DEPTH=$d timeout -k 10 300 python bench.py --scene $sc --steps $st --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_d${d}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_d${d}_${sc}_$r.log; exit 1; }
      echo "pq_depth $d $sc r$r: $(tail -1 $O/bench_d${d}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
    done
  done
done
