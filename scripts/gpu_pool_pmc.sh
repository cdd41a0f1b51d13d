# PMC passes (separate runs, no tracing domains) of one sponza 1080p render: k_render_ps vs the
# pool kernel with parking off (no pool traffic) and on.  Usage: bash scripts/gpu_pool_pmc.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-poolpmc}; mkdir -p $O
SPP=${SPP:-16}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR"
for cfg in "0 1" "6 0" "6 1" "5 0"; do
  set -- $cfg
  for pass in A B; do
    C=${!pass}
    D=$O/p$1_park$2_$pass
    WGT_POOL=$1 WGT_POOL_PARK=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $D -o run --output-format csv -- python scripts/render_once.py sponza 1920 1080 $SPP > $D.log 2>&1 || { echo "pmc $cfg $pass failed"; tail -5 $D.log; exit 1; }
  done
  echo "done pool=$1 park=$2"
done
