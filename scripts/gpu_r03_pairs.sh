# Two triangles per step adopted: GPU suite, then the mode knob (triangle vs node step ratio) re-swept
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03pairs}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
E="WGT_TRI_RATIO=100;WGT_TRI_RATIO=50;WGT_TRI_RATIO=70;WGT_TRI_RATIO=130;WGT_TRI_RATIO=180;WGT_TRI_RATIO=100"
for sc in bunny sponza; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["trav_util"], d["identical"])
PY
done
