# Round 5: product tests touched by the decoupled gather, then the wide-form A/B (ab/*.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_product.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "rccl or bench or pipelined or two_ranks" > $O/pytest_product.log 2>&1 || { tail -40 $O/pytest_product.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_product.log | tail -12
SCENES=sponza FORMS="2 4" bash scripts/gpu_r05_ab.sh ${1:-r05c}/ab 1
