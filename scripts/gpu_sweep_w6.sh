set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r02sw6
for sc in "sponza 1920 1080 256" "bunny 1920 1080 256"; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc ";WGT_PS_TO_TRAV=18,WGT_PS_TO_SERVICE=16;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=18;WGT_PS_TO_TRAV=14,WGT_PS_TO_SERVICE=12;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=12;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=16;WGT_PQ_REFILL=2;WGT_PQ_REFILL=4;WGT_TRI_RATIO=80;WGT_TRI_RATIO=125;WGT_PS_SVC_FRAC=12;WGT_PS_SVC_FRAC=20" >> gpurun_out/r02sw6/sweep.jsonl 2>&1 || exit 1
done
grep '^{' gpurun_out/r02sw6/sweep.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['scene'], d['env'], d['ms'], d['identical'])"
