# Parked vs whole-stack kernel: service-region cycle split (scripts/park_regions.py) and the SQ
# instruction mix of one sponza 1080p/64spp frame (SALU, LDS, LDS issue stalls, VALU, scratch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04d}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python scripts/park_regions.py > $O/regions.log 2>&1 || { tail -20 $O/regions.log; exit 1; }
cat $O/regions.log
CH="python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline --check off --pmc off --stats-reps 1 --spp 64"
for P in 0 1; do
  for C in "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES"; do
    N=$(echo $C | tr ' ' '_' | cut -c1-30)
    WGT_PARK=$P WGT_PS_CAP=17 timeout -s KILL 150 rocprofv3 --pmc $C -d $O/p${P}_$N -o run --output-format csv -- $CH > $O/p${P}_$N.log 2>&1 || { echo "pmc $P failed"; tail -5 $O/p${P}_$N.log; exit 1; }
  done
done
echo done
