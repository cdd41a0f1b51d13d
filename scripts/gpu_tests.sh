# GPU test run: given test files/args (default: the whole -m gpu suite), one pytest process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tests}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v --timeout 300 --timeout-method thread -p no:randomly > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -60
exit $rc
