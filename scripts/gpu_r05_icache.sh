# Round 5: instruction-cache and LDS counters of the default kernel (sponza 1080p/64 spp, one render),
# one rocprofv3 --pmc pass per group, each under its own kill timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05ic}; O=gpurun_out/$T; mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -oE "\b(SQC?_[A-Z0-9_]*ICACHE[A-Z0-9_]*|SQ_LDS_[A-Z_]*|SQ_INSTS_LDS|SQ_INST_CYCLES_[A-Z_]*)\b" $O/counters_list.txt | sort -u > $O/names.txt || true
cat $O/names.txt | tr '\n' ' '; echo
i=0
for ctrs in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctrs -d $O/pmc_$i -o run --output-format csv -- python scripts/render_once.py sponza 64 \
    > $O/pmc_$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $O/pmc_$i.log; continue; }
  python -c "
import csv,glob,collections
agg=collections.defaultdict(float)
for f in glob.glob('$O/pmc_$i/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_render_ps<false, false' in r['Kernel_Name']: agg[r['Counter_Name']]+=float(r['Counter_Value'])
print('pass $i', dict(agg))"
done
