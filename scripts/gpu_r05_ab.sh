# Round 5 same-box A/B of ab/*.so (each loaded through WGT_LIB_PATH): a parity subset on each, the
# wide-form counters, then the driver's bench command per build and node form.
#   bash scripts/gpu_r05_ab.sh TAG [rounds]   (FORMS="2 4", SCENES="sponza bunny", STEPS=20)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05ab}; R=${2:-1}; O=gpurun_out/$T; mkdir -p $O
for so in ab/*.so; do
  n=$(basename $so .so)
  WGT_LIB_PATH=$PWD/$so timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "${PYK:-sponza_render_parity or schedule_invariance}" > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.log)"
  for sc in ${SCENES:-sponza bunny}; do
    WGT_LIB_PATH=$PWD/$so W8_FORMS="4" timeout -k 10 300 python scripts/w8_stats.py $sc 1920 1080 16 > $O/stats_${n}_$sc.log 2>&1 || { tail -20 $O/stats_${n}_$sc.log; exit 1; }
    cat $O/stats_${n}_$sc.log
  done
done
for r in $(seq $R); do
  for so in ab/*.so; do
    n=$(basename $so .so)
    for sc in ${SCENES:-sponza bunny}; do
      for cn in ${FORMS:-2 4}; do
        [ "$cn" != 4 ] && [ "$n" != "$(basename $(ls ab/*.so | head -1) .so)" ] && continue  # BVH4 forms: first build only
        st=${STEPS:-20}; [ $sc = bunny ] && st=$((st + 10))
        WGT_LIB_PATH=$PWD/$so WGT_CNODE=$cn timeout -k 10 600 python bench.py --scene $sc --steps $st --warmup 5 --pmc off \
          --no-cpu-baseline --stats-reps 1 > $O/bench_${n}_${sc}_cn${cn}_$r.log 2>&1 || { tail -20 $O/bench_${n}_${sc}_cn${cn}_$r.log; exit 1; }
        echo "$n $sc cn$cn r$r: $(tail -1 $O/bench_${n}_${sc}_cn${cn}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_launch']; print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'], round(p['node_visits']/p['traced_rays'],3), round(p['tri_tests']/p['traced_rays'],3), d['simt_utilisation'].get('bvh_loop'))")"
      done
    done
  done
done
