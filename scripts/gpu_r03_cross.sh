# cross-leaf second slot (WGT_TRI_CROSS: the last triangle of the open leaf with the first of the leaf parked on
# the stack top) against HEAD: GPU suite on cross.so, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03cross} 3 || exit 1
