# Round-4 baseline on a fresh box: smoke, the -m gpu suite, the driver's 20-step bench, then the
# write-traffic attribution of DESIGN §5: WRITE_SIZE and L2 hit rate of one
# sponza frame with the 6-wave kernel (68 B/lane of scratch) against the 5-wave one (no scratch).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04a}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-300
CH="python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline --check off --pmc off --stats-reps 1"
for W in 6 5; do
  for C in "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    N=$(echo $C | tr ' ' '_' | cut -c1-30)
    WGT_PS_WAVES=$W timeout -s KILL 150 rocprofv3 --pmc $C -d $O/w${W}_$N -o run --output-format csv -- $CH > $O/w${W}_$N.log 2>&1 || { echo "pmc $W $C failed"; tail -5 $O/w${W}_$N.log; exit 1; }
  done
done
echo done
