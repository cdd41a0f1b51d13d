# Round 5: the SQ pass of the bench line on bunny and sponza (raw figures), and the grid size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r05sq}; mkdir -p $O
for sc in bunny sponza; do
  timeout -k 10 600 python bench.py --scene $sc --steps 6 --warmup 2 --no-cpu-baseline --stats-reps 1 > $O/bench_$sc.log 2>&1 || { tail -20 $O/bench_$sc.log; exit 1; }
  tail -1 $O/bench_$sc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$sc', d['value'], d['persistent_grid_waves'], r['valu_busy'], r['wave_split'], r['sq_raw'])"
done
