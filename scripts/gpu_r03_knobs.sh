# Phase / refill / mode knobs re-swept on the round-3 build (1080p/256 spp, one frame per render, min of 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03knobs}; mkdir -p $O
E="WGT_PS_SVC_FRAC=16;WGT_PS_TO_TRAV=12,WGT_PS_TO_SERVICE=10;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=18;WGT_PS_TO_TRAV=24,WGT_PS_TO_SERVICE=22;WGT_PS_TO_TRAV=32,WGT_PS_TO_SERVICE=30;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=10;WGT_PS_SVC_FRAC=8;WGT_PS_SVC_FRAC=24;WGT_PQ_REFILL=1;WGT_PQ_REFILL=4;WGT_TRI_RATIO=70;WGT_TRI_RATIO=150;WGT_PS_SVC_FRAC=16"
for sc in bunny sponza; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["trav_util"], d["identical"])
PY
done
