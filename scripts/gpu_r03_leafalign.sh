# Leaf alignment (WGT_LEAF_ALIGN=1: pairs of a triangle step in one 128-B line): GPU suite, then one-frame timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03la}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
E="WGT_LEAF_ALIGN=0;WGT_LEAF_ALIGN=1;WGT_LEAF_ALIGN=0;WGT_LEAF_ALIGN=1;WGT_LEAF_ALIGN=0;WGT_LEAF_ALIGN=1"
for sc in sponza bunny; do
  REUPLOAD=1 REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["trav_util"], d["identical"])
PY
done
