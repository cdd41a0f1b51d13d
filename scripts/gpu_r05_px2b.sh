# Historical (round 5): k_render_ps2 / WGT_PS_WAVES=4 / WGT_PX2_* were removed after commit 050a6a2.
# Round 5: why two pixels per lane is slow: STATS counters per variant, then the bench with live
# PMC passes (VALU instructions, wave-cycle split) for the default and the two-pixel kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05px2b}; O=gpurun_out/$T; mkdir -p $O
for sc in bunny sponza; do
  timeout -k 10 300 python scripts/px2_stats.py $sc 16 base= px2=WGT_PS_WAVES:4 px2s1=WGT_PS_WAVES:4,WGT_PX2_SWAP:1 \
    px2s64=WGT_PS_WAVES:4,WGT_PX2_SWAP:64 > $O/stats_$sc.jsonl 2>&1 || { tail -20 $O/stats_$sc.jsonl; exit 1; }
  cat $O/stats_$sc.jsonl
done
for v in base px2; do
  if [ $v = px2 ]; then export WGT_PS_WAVES=4; fi
  timeout -k 10 600 python bench.py --scene bunny --steps 3 --warmup 1 --pmc on --no-cpu-baseline \
    --stats-reps 1 > $O/bench_bunny_$v.log 2>&1 || { tail -20 $O/bench_bunny_$v.log; exit 1; }
  tail -1 $O/bench_bunny_$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$v', d['value'], d['kernel_ms'], r.get('valu_busy'), r.get('wave_split'), (r.get('sq_raw') or {}))"
done
