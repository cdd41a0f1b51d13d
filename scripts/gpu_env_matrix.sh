#!/bin/bash
# The whole GPU parity suite under each forced kernel knob (node form, wave budget,
# kernel family, queue order): every image stays bit-identical to the oracle.
#   bash scripts/gpu_env_matrix.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for e in WGT_CNODE=1 WGT_CNODE=0 WGT_PS_WAVES=5 WGT_PS_WAVES=6 WGT_KERNEL=1 WGT_PQ_LPT=0; do
  env $e timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/envtest_$e.log 2>&1 || { echo "FAIL $e"; tail -15 gpurun_out/envtest_$e.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/envtest_$e.log)"
done
