# Ray-pool kernel (wgt_pool.hip): the GPU suite with the pool on, then same-box timing
# of k_render_ps (WGT_POOL=0) against the pool kernel at 6 and 5 waves per SIMD.
# Usage: bash scripts/gpu_pool_ab.sh TAG [POOL values...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-pool}; shift; mkdir -p $O
VALS=${@:-0 6 5}
if [ -z "$SKIP_TESTS" ]; then
echo "== pytest -m gpu with WGT_POOL=6"
WGT_POOL=6 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pool6.log 2>&1 || { tail -40 $O/pytest_pool6.log; exit 1; }
tail -2 $O/pytest_pool6.log
fi
for scene in sponza bunny; do
  for rep in 1 2; do
    for P in $VALS; do
      WGT_POOL=$P timeout -k 10 300 python bench.py --scene $scene --steps 6 --warmup 2 --no-cpu-baseline --stats-reps 1 > $O/bench_${scene}_p${P}_r${rep}.log 2>&1 || { echo "bench $scene pool $P failed"; tail -20 $O/bench_${scene}_p${P}_r${rep}.log; exit 1; }
      python - $O/bench_${scene}_p${P}_r${rep}.log $scene $P <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "pool", sys.argv[3], "Mrays/s", d["value"], "launch_ms", d["kernel_ms"], "iso", d["timing"]["isolated_launch_ms"], "simt", d["simt_utilisation"], "nodes", d["per_launch"]["node_visits"])
PY
    done
  done
done
