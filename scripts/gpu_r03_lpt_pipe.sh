# steady state with frames in flight: the cost pre-pass + LPT order (default) against block order (WGT_PQ_LPT=0),
# the driver's command (20 steps, 2 in flight), alternating, no CPU baseline / PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03lptpipe}; mkdir -p $O
for r in 1 2; do
  for lpt in 1 0; do
    WGT_PQ_LPT=$lpt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/lpt${lpt}_r$r.log 2>&1 || { tail $O/lpt${lpt}_r$r.log; exit 1; }
    echo "lpt=$lpt r$r $(tail -1 $O/lpt${lpt}_r$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["timing"]["isolated_launch_ms"])')"
  done
done
for r in 1 2; do
  for lpt in 1 0; do
    WGT_PQ_LPT=$lpt timeout -k 10 300 python bench.py --scene bunny --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/bunny_lpt${lpt}_r$r.log 2>&1 || { tail $O/bunny_lpt${lpt}_r$r.log; exit 1; }
    echo "bunny lpt=$lpt r$r $(tail -1 $O/bunny_lpt${lpt}_r$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["timing"]["isolated_launch_ms"])')"
  done
done
