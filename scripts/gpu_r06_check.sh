# Round 6: the -m gpu suite on the working tree's libwgt.so (optionally a -k subset: PYK), then the
# same-box A/B of ab/*.so (scripts/gpu_r06_ab.sh).  Usage: bash scripts/gpu_r06_check.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06c}; R=${2:-2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
[ "$R" = 0 ] && exit 0
PYK= bash scripts/gpu_r06_ab.sh $T $R
