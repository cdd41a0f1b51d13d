# the stack top known without an LDS round trip at a node step's pop (WGT_TOP_PREFETCH): GPU suite on toppf.so,
# then timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03toppf} 3 || exit 1
