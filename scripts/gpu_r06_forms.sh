# Round 6: the node form per scene on the scratch-free build (WGT_CNODE), then the A/B of ab/*.so.
#   bash scripts/gpu_r06_forms.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06n}; O=gpurun_out/$T; mkdir -p $O
for sc in sponza bunny; do
  for cn in 2 0 1; do
    st=12; [ $sc = bunny ] && st=20
    WGT_CNODE=$cn timeout -k 10 400 python bench.py --scene $sc --steps $st --warmup 3 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_${sc}_cn$cn.log 2>&1 || { tail -20 $O/bench_${sc}_cn$cn.log; exit 1; }
    echo "$sc cnode=$cn: $(tail -1 $O/bench_${sc}_cn$cn.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['per_launch']['bvh_nodes'])")"
  done
done
bash scripts/gpu_r06_ab.sh $T 2
