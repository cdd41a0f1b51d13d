# GPU suite, then the default bench (pipelined) beside --pipeline 1, then the N=2 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r02b}; mkdir -p $O
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== bench p2"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p2.log 2>&1 || { tail -20 $O/bench_p2.log; exit 1; }
tail -1 $O/bench_p2.log | cut -c1-600
echo "== bench p1"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pipeline 1 --no-cpu-baseline > $O/bench_p1.log 2>&1 || { tail -20 $O/bench_p1.log; exit 1; }
tail -1 $O/bench_p1.log | cut -c1-400
echo "== rehearsal"; bash scripts/gpu_dist_rehearsal.sh ${1:-r02b}_dist || exit 1
