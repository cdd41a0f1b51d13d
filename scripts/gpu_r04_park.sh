# Round-4 parked traversal state and the runtime-selected 64-B compact
# records: the -m gpu suite on the new default, then the driver's 20-step bench A/B over
# (WGT_PARK, WGT_CNODE) = (1, 2) default, (0, 2) round 3's kernel, (1, 3) the 64-B records, two
# rounds; the spill/refill counts of the default LDS stack; WRITE_SIZE / L2 / FETCH / SQ passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04b}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
# (WGT_PARK, WGT_CNODE, WGT_PS_WAVES): whole stack (round 3), parked at 6 waves (80-B, 64-B records),
# parked at 7 waves (80-B, 64-B records)
for R in 1 2; do
  for PC in "0 2 6" "1 2 6" "1 3 6" "1 2 7" "1 3 7"; do
    set -- $PC
    WGT_PARK=$1 WGT_CNODE=$2 WGT_PS_WAVES=$3 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/bench20_p$1_c$2_w$3_$R.log 2>&1 || { tail -20 $O/bench20_p$1_c$2_w$3_$R.log; exit 1; }
    echo "park=$1 cnode=$2 waves=$3 round $R: $(tail -1 $O/bench20_p$1_c$2_w$3_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'], d['simt_utilisation'])")"
  done
done
timeout -k 10 300 python scripts/park_stats.py > $O/park_stats.log 2>&1 || { tail -20 $O/park_stats.log; exit 1; }
cat $O/park_stats.log
CH="python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline --check off --pmc off --stats-reps 1"
for PC in "0 2 6" "1 2 6" "1 3 6" "1 2 7"; do
  set -- $PC
  for C in "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"; do
    N=$(echo $C | tr ' ' '_' | cut -c1-30)
    WGT_PARK=$1 WGT_CNODE=$2 WGT_PS_WAVES=$3 timeout -s KILL 150 rocprofv3 --pmc $C -d $O/p$1_c$2w$3_$N -o run --output-format csv -- $CH > $O/p$1_c$2w$3_$N.log 2>&1 || { echo "pmc $PC $C failed"; tail -5 $O/p$1_c$2w$3_$N.log; exit 1; }
  done
done
echo done
