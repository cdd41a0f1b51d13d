# Same-box A/B of ab/*.so (GPU suite on each non-base build first), then an env sweep on the working tree.
#   AB_SCENES=... ENVS=... SCENES=... bash scripts/gpu_ab_sweep.sh <tag> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
REPS=${REPS:-3} bash scripts/gpu_ab_all.sh ${1:-abs} ${2:-2} > /dev/null || exit 1
OUT=gpurun_out/${1:-abs}
python scripts/ab_table.py $OUT/ab.log 2>/dev/null || grep -A1 "\.so r" $OUT/ab.log | grep -o '"ms": [0-9.]*'
if [ -n "$ENVS" ]; then
  for sc in ${SCENES:-sponza_1920_1080_256 bunny_1920_1080_256}; do
    REPS=2 timeout -k 10 500 python scripts/sweep_env.py $(echo $sc | tr _ " ") "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
  done
  python - $OUT/sweep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["spp"], d["env"], d["ms"], d["nodes"], d["tris"], d["identical"])
PY
fi
