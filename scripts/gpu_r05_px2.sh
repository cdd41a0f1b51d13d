# Historical (round 5): k_render_ps2 / WGT_PS_WAVES=4 / WGT_PX2_* were removed after commit 050a6a2.
# Round 5: two pixels per lane (WGT_PS_WAVES=4, k_render_ps2) on the GPU: parity subset, then the
# driver's bench command per variant (same box).  Usage: bash scripts/gpu_r05_px2.sh TAG [steps]
# VARIANTS: space-separated name=ENV,ENV (ENV as K:V), e.g. "base= px2=WGT_PS_WAVES:4"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05px2}; ST=${2:-10}; O=gpurun_out/$T; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "${PYK:-sponza_render_parity or full_frame_1080p or schedule_invariance}" > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for sc in ${SCENES:-sponza bunny}; do
  for v in ${VARIANTS:-base= px2=WGT_PS_WAVES:4}; do
    name=${v%%=*}; envs=${v#*=}
    args=""
    for e in ${envs//,/ }; do args="$args ${e%%:*}=${e#*:}"; done
    env $args timeout -k 10 600 python bench.py --scene $sc --steps $ST --warmup 3 --pmc off --no-cpu-baseline \
      --stats-reps 1 > $O/bench_${sc}_$name.log 2>&1 || { tail -20 $O/bench_${sc}_$name.log; exit 1; }
    tail -1 $O/bench_${sc}_$name.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d.get('per_launch',{}); t=d.get('timing',{}); r=max(p['traced_rays'],1)
print('$sc $name', d['value'], d['ms_per_step'], t.get('isolated_launch_ms'), 'nodes/ray', round(p['node_visits']/r,3), 'tris/ray', round(p['tri_tests']/r,3), p['kernel'], 'simt', d.get('simt_utilisation'))"
  done
done
