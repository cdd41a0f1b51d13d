# a hit sibling leaf opened as the pending leaf at a node step (WGT_SIB_LEAF=1: slot 1 only; 3: any slot):
# GPU suite on each build, then same-box timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03sib} 3 || exit 1
