# The BVH2 build's SAH node-visit cost (WGT_SAH_TRAV, triangle test = 1) on the current kernel, whose
# triangle steps test two triangles: the driver's sponza command and the bunny C3 line, rounds alternating.
#   bash scripts/gpu_r04_sah.sh TAG [rounds] [costs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04sah}; R=${2:-2}; shift 2; CS=${@:-1.0 1.5 2.0 3.0}
O=gpurun_out/$T; mkdir -p $O
for r in $(seq $R); do
  for c in $CS; do
    for sc in sponza bunny; do
      st=20; [ $sc = bunny ] && st=30
      WGT_SAH_TRAV=$c timeout -k 10 300 python bench.py --scene $sc --steps $st --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_c${c}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_c${c}_${sc}_$r.log; exit 1; }
      echo "sah_trav $c $sc r$r: $(tail -1 $O/bench_c${c}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); pl=d['per_launch']; print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'], 'nodes/ray', round(pl['node_visits']/pl['traced_rays'],3), 'tris/ray', round(pl['tri_tests']/pl['traced_rays'],3))")"
    done
  done
done
