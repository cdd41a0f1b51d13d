# Round 2: every config (scripts/gpu_configs.sh) then a knob re-sweep on sponza/bunny 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_configs.sh ${1:-r02cfg} || exit 1
OUT=gpurun_out/${1:-r02cfg}
ENVS=";WGT_TRI_RATIO=60;WGT_TRI_RATIO=80;WGT_TRI_RATIO=130;WGT_TRI_RATIO=170;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=14;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=18;WGT_PS_TO_TRAV=22,WGT_PS_TO_SERVICE=20;WGT_PQ_REFILL=1;WGT_PQ_REFILL=3;"
for sc in sponza_1920_1080_256 bunny_1920_1080_256; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $(echo $sc | tr _ " ") "$ENVS" >> $OUT/sweep.jsonl 2>&1 || exit 1
done
python - $OUT/sweep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["spp"], d["env"], d["ms"], d["nodes"], d["identical"])
PY
