# Region queues (WGT_PQ_REGIONS): GPU suite on the new build, its cost when off against HEAD, then R = 8 / 4 / 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256" REPS=2 \
ENVS="WGT_PQ_REGIONS=0;WGT_PQ_REGIONS=8;WGT_PQ_REGIONS=4;WGT_PQ_REGIONS=2;WGT_PQ_REGIONS=0" \
bash scripts/gpu_ab_sweep.sh ${1:-r03reg} 3 || exit 1
