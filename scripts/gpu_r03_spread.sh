# The slot spread (pq_cap) on the GPU suite, then the strong-scaling projection with it off/on,
# then full-frame timing with it off/on (full frames have more slots than lanes: no change expected).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03spread}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sp in 0 1; do
  WGT_PQ_SPREAD=$sp timeout -k 10 300 python scripts/strong_projection.py --scene sponza --reps 1 --ns 4 8 > $O/strong_spread$sp.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  cat $O/strong_spread$sp.jsonl | cut -c1-200
done
