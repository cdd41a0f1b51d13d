# Round-4 parked traversal state: the -m gpu suite on the new default,
# then the driver's 20-step bench A/B (WGT_PARK=1 default vs 0, two rounds), the spill/refill
# counts of the default LDS stack on sponza, and WRITE_SIZE / L2 / FETCH passes of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04b}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
for R in 1 2; do
  for P in 1 0; do
    WGT_PARK=$P timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/bench20_p${P}_$R.log 2>&1 || { tail -20 $O/bench20_p${P}_$R.log; exit 1; }
    echo "park=$P round $R: $(tail -1 $O/bench20_p${P}_$R.log | cut -c1-200)"
  done
done
timeout -k 10 300 python scripts/park_stats.py > $O/park_stats.log 2>&1 || { tail -20 $O/park_stats.log; exit 1; }
cat $O/park_stats.log
CH="python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline --check off --pmc off --stats-reps 1"
for P in 1 0; do
  for C in "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    N=$(echo $C | tr ' ' '_' | cut -c1-30)
    WGT_PARK=$P timeout -s KILL 150 rocprofv3 --pmc $C -d $O/p${P}_$N -o run --output-format csv -- $CH > $O/p${P}_$N.log 2>&1 || { echo "pmc $P $C failed"; tail -5 $O/p${P}_$N.log; exit 1; }
  done
done
echo done
