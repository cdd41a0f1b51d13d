# Historical (round 5): k_render_ps2 / WGT_PS_WAVES=4 / WGT_PX2_* were removed after commit 050a6a2.
# Round 5: two pixels per lane, diagnosis: per 4-wave form (WGT_PX2_MODE 0 = two pixels per lane,
# 1 = k_render_ps2 with one, 2 = k_render_ps at 4 waves) and the default, the frame time and STATS
# counters, then one rocprofv3 --pmc pass of the instruction mix per form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05px2d}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python scripts/px2_stats.py bunny 64 base= px2=WGT_PS_WAVES:4 px2one=WGT_PS_WAVES:4,WGT_PX2_MODE:1 \
  ps4=WGT_PS_WAVES:4,WGT_PX2_MODE:2 > $O/stats_bunny.jsonl 2>&1 || { tail -20 $O/stats_bunny.jsonl; exit 1; }
cat $O/stats_bunny.jsonl
for v in base px2 px2one ps4; do
  case $v in base) E="";; px2) E="WGT_PS_WAVES=4";; px2one) E="WGT_PS_WAVES=4 WGT_PX2_MODE=1";; ps4) E="WGT_PS_WAVES=4 WGT_PX2_MODE=2";; esac
  for e in $E; do export $e; done
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH \
    -d $O/pmc_$v -o run --output-format csv -- python scripts/render_once.py bunny 64 > $O/pmc_$v.log 2>&1 \
    || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  unset WGT_PS_WAVES WGT_PX2_MODE
done
for f in $(find $O -name "*counter_collection.csv" | sort); do
  python -c "
import csv,collections
agg=collections.defaultdict(float)
for r in csv.DictReader(open('$f')):
    n=r['Kernel_Name']
    if 'k_render_ps' in n and '<false, false' in n: agg[(n.split('(')[0], r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print('$f'.split('/')[2], k[0], k[1], '%.4g'%v)
"
done
