# Node form at 6 waves per SIMD: compact vs 128-B nodes on both stand-ins.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r02cn6; mkdir -p $O
for sc in "sponza 1920 1080 256" "bunny 1920 1080 256"; do
  REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc ";WGT_CNODE=0;WGT_CNODE=1;WGT_PQ_SVC_COST=4;WGT_PQ_SVC_COST=10" >> $O/sweep.jsonl 2>&1 || exit 1
done
grep '^{' $O/sweep.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['scene'], d['env'], d['ms'], d['nodes'], d['identical'])"
