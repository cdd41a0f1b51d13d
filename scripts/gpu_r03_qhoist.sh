# a quad record's five scalar loads issued together (WGT_QUAD_HOIST): GPU suite on qhoist.so, then
# same-box timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03qh} 3 || exit 1
