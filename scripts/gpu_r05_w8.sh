# Round 5: the wide form on the GPU: parity subset, then the driver's bench command with the
# default node form and with WGT_CNODE=4 (same box).  Usage: bash scripts/gpu_r05_w8.sh TAG [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05w8}; ST=${2:-10}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "${PYK:-sponza_render_parity or full_frame_1080p or schedule_invariance}" > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for sc in ${SCENES:-sponza bunny}; do
  for cn in ${CNODES:-2 4}; do
    WGT_CNODE=$cn timeout -k 10 600 python bench.py --scene $sc --steps $ST --warmup 3 --pmc off --no-cpu-baseline \
      --stats-reps 1 > $O/bench_${sc}_cn$cn.log 2>&1 || { tail -20 $O/bench_${sc}_cn$cn.log; exit 1; }
    tail -1 $O/bench_${sc}_cn$cn.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d.get('per_launch',{}); t=d.get('timing',{}); r=max(p['traced_rays'],1)
print('$sc cn$cn', d['value'], d['ms_per_step'], t.get('isolated_launch_ms'), 'nodes/ray', round(p['node_visits']/r,3), 'tris/ray', round(p['tri_tests']/r,3), p['kernel'], 'simt', d.get('simt_utilisation'))"
  done
done
