#!/bin/bash
# The GPU suite, then bunny (C3) on the compact records (the default since round 6) against the
# size rule's 128-B nodes (WGT_CNODE=2), alternating on one box: the driver's bench command per run.
#   bash scripts/gpu_r06_cnode.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06cn}; R=${2:-3}; O=gpurun_out/$T; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
for r in $(seq $R); do for cn in 2 1; do
  WGT_CNODE=$cn timeout -k 10 400 python bench.py --scene ${SCENE:-bunny} --steps 30 --warmup 3 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bunny_cn${cn}_$r.log 2>&1 || { tail $O/bunny_cn${cn}_$r.log; exit 1; }
  echo "${SCENE:-bunny} cnode=$cn r$r: $(tail -1 $O/bunny_cn${cn}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['per_launch']['bvh_nodes'])")"
done; done
echo done
