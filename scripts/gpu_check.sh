set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== pytest"; timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; tail -5 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc
