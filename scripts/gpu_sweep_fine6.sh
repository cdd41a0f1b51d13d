# Fine sweep of the schedule knobs at 6 waves per SIMD (REPS renders per setting, min reported).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r02fine}; mkdir -p $O
E=";WGT_PS_TO_TRAV=15,WGT_PS_TO_SERVICE=13;WGT_PS_TO_TRAV=17,WGT_PS_TO_SERVICE=15;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=13;WGT_PS_TO_TRAV=17,WGT_PS_TO_SERVICE=14;WGT_PS_SVC_FRAC=14;WGT_PS_SVC_FRAC=18;WGT_TRI_RATIO=90;WGT_TRI_RATIO=110;WGT_PQ_SVC_COST=4;WGT_PQ_SVC_COST=5;"
for sc in "sponza 1920 1080 256" "bunny 1920 1080 256"; do
  REPS=3 timeout -k 10 900 python scripts/sweep_env.py $sc "$E" >> $O/sweep.jsonl 2>&1 || exit 1
done
grep '^{' $O/sweep.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['scene'], d['env'], d['ms'], d['identical'])"
