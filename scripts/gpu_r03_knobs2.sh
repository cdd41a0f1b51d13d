# Phase / refill / mode knobs re-swept with two triangles per step (1080p/256 spp, one frame per render, min of 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03knobs2}; mkdir -p $O
E="WGT_PS_SVC_FRAC=16;WGT_PS_TO_TRAV=14,WGT_PS_TO_SERVICE=12;WGT_PS_TO_TRAV=18,WGT_PS_TO_SERVICE=16;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=18;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=12;WGT_PS_TO_TRAV=18,WGT_PS_TO_SERVICE=14;WGT_PS_SVC_FRAC=12;WGT_PS_SVC_FRAC=20;WGT_PQ_REFILL=1;WGT_PQ_REFILL=3;WGT_PS_SVC_FRAC=16"
for sc in bunny sponza; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["trav_util"], d["identical"])
PY
done
