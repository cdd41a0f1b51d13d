#!/bin/bash
# Is the vector-memory address path (TA) what a node step waits on?  One sponza render at 64 spp per
# counter pass (rocprofv3 --pmc, kernel trace for the durations), summarised per kernel.
#   bash scripts/gpu_r06_ta.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06ta}; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python scripts/render_once.py ${SCENE:-sponza} 64 > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
i=0
for G in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- python scripts/render_once.py ${SCENE:-sponza} 64 > $OUT/p$i.log 2>&1 || { echo "pass $i ($G) failed rc=$?"; exit 1; }
done
python scripts/summarize_pmc_mem.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
cat $OUT/kt/*kernel_stats.csv 2>/dev/null | head -5
echo done
