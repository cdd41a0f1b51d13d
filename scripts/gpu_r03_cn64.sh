# 64-B compact node records (WGT_CN64: codes + 24-bit refs with the grid origin in their top bytes) against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;sponza 1920 1080 64;bunny 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03cn64} 3 || exit 1
