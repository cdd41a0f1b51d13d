# Same-box timing A/B of ab/*.so (no test suite): the driver's sponza command (20 steps) and the
# bunny C3 line (30 steps), rounds alternating the builds.  Usage: bash scripts/gpu_r04_abtime.sh TAG [rounds] [so...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04abt}; R=${2:-2}; shift 2; SOS=${@:-$(ls ab/*.so)}
O=gpurun_out/$T; mkdir -p $O
for r in $(seq $R); do
  for so in $SOS; do
    n=$(basename $so .so)
    for sc in sponza bunny; do
      st=20; [ $sc = bunny ] && st=30
      WGT_LIB_PATH=$PWD/$so timeout -k 10 300 python bench.py --scene $sc --steps $st --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_${n}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_${n}_${sc}_$r.log; exit 1; }
      echo "$n $sc r$r: $(tail -1 $O/bench_${n}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'], d['simt_utilisation'])")"
    done
  done
done
