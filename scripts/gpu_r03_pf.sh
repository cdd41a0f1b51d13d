# the next compact node's loads issued right after a traversal step (WGT_NODE_PF): GPU suite on pf.so,
# then same-box timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03pf} 3 || exit 1
