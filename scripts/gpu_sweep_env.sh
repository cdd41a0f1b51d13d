#!/bin/bash
# GPU parity tests on the working tree, then an env sweep (scripts/sweep_env.py) per scene.
#   ENVS="K=V,K=V;K=V" SCENES="bunny_1920_1080_64 sponza_1920_1080_16" bash scripts/gpu_sweep_env.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for sc in ${SCENES:-bunny_1920_1080_64 sponza_1920_1080_16}; do
  REPS=${REPS:-2} timeout -k 10 500 python scripts/sweep_env.py $(echo $sc | tr _ " ") "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
done
python - $OUT/sweep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["spp"], d["env"], d["ms"], d["nodes"], d["identical"])
PY
