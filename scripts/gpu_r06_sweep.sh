# Round 6: the persistent kernel's phase knobs re-swept on the scratch-free build (env knobs, one
# process per scene, isolated 1080p/256spp frames).  Usage: bash scripts/gpu_r06_sweep.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06s}; O=gpurun_out/$T; mkdir -p $O
E=${E:-";WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=18;WGT_PS_TO_TRAV=24,WGT_PS_TO_SERVICE=20;WGT_PS_TO_TRAV=12,WGT_PS_TO_SERVICE=10;WGT_PS_TO_TRAV=18,WGT_PS_TO_SERVICE=16;WGT_PS_TO_TRAV=16,WGT_PS_TO_SERVICE=12;WGT_PS_TO_TRAV=20,WGT_PS_TO_SERVICE=14;WGT_PS_TO_TRAV=14,WGT_PS_TO_SERVICE=12;WGT_TRI_RATIO=70;WGT_TRI_RATIO=150;WGT_PS_SVC_FRAC=8;WGT_PS_SVC_FRAC=24;WGT_PQ_REFILL=4;"}
for sc in sponza bunny; do
  REPS=2 timeout -k 10 400 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/sweep_$sc.jsonl 2>&1 || { tail -20 $O/sweep_$sc.jsonl; exit 1; }
  python -c "
import json,sys
for l in open('$O/sweep_$sc.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$sc', d['ms'], d['trav_util'], d['identical'], d['env'])"
done
echo done
