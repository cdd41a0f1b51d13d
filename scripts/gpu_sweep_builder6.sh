# Builder knobs at 6 waves per SIMD (each setting rebuilds the BVH: REUPLOAD=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r02bld}; mkdir -p $O
E="REUPLOAD=1;REUPLOAD=1,WGT_SAH_LEAF=4;REUPLOAD=1,WGT_SAH_LEAF=6;REUPLOAD=1,WGT_DP_LEAF=2;REUPLOAD=1,WGT_DP_LEAF=4;REUPLOAD=1,WGT_SAH_TRAV=0.8;REUPLOAD=1,WGT_SAH_TRAV=1.25;REUPLOAD=1,WGT_DP_TRI=1.5;REUPLOAD=1,WGT_DP_TRI=0.75;REUPLOAD=1"
for sc in "sponza 1920 1080 256" "bunny 1920 1080 256"; do
  REPS=2 timeout -k 10 900 python scripts/sweep_env.py $sc "$E" >> $O/sweep.jsonl 2>&1 || exit 1
done
grep '^{' $O/sweep.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['scene'], d['env'], d['ms'], d['nodes'], d['tris'], d['identical'])"
