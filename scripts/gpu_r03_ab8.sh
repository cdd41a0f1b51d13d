# two triangles per step only in waves where some lane has two left (WGT_TRI_UNIFORM, uni.so) against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab8} 3 || exit 1
