# BVH shape knobs re-swept with two triangles per step (the tree is rebuilt per setting; images must stay identical)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03tree}; mkdir -p $O
E="WGT_DP_TRI=1;WGT_DP_TRI=0.8;WGT_DP_TRI=0.6;WGT_DP_LEAF=4;WGT_DP_LEAF=6;WGT_DP_LEAF=8;WGT_DP_LEAF=8,WGT_DP_TRI=0.7;WGT_SAH_TRAV=1.5;WGT_SAH_TRAV=0.7;WGT_SAH_LEAF=4;WGT_DP_TRI=1"
for sc in sponza bunny; do
  REUPLOAD=1 REPS=2 timeout -k 10 600 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["nodes"], d["tris"], d["bvh"], d["identical"])
PY
done
