#!/bin/bash
# Vector-memory pipeline counters (TA / TD / TCP) of the sponza render, one pass each.
#   bash scripts/gpu_pmc_mem.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcmem}; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
grep -o -E '\b(TA|TD|TCP|GRBM)_[A-Z0-9_]+' $OUT/avail.txt | sort -u > $OUT/names.txt
wc -l $OUT/names.txt
i=0
for G in "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum" "TA_FLAT_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "GRBM_GUI_ACTIVE GRBM_COUNT" "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- python scripts/render_once.py sponza 1920 1080 16 > $OUT/p$i.log 2>&1 || echo "pass $i ($G) failed rc=$?"
done
python scripts/summarize_pmc_mem.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
echo done
