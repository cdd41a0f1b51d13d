#!/bin/bash
# PMC breakdown per kernel family: bash scripts/gpu_pmc_kernels.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmck}; mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_IFETCH"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU"
G3="SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_IFETCH_LEVEL"
G4="TCC_HIT_sum TCC_MISS_sum"
for K in 2 1; do
  i=0
  for G in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    WGT_KERNEL=$K timeout -k 10 300 rocprofv3 --pmc $G -d $OUT/k${K}_g$i -o run --output-format csv -- python scripts/render_once.py bunny 1920 1080 16 > $OUT/k${K}_g$i.log 2>&1 || { echo "fail k$K g$i"; tail -5 $OUT/k${K}_g$i.log; exit 1; }
  done
done
echo done
