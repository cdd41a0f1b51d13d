# two triangles per step: the generic form (k2gen) against the pairs-shaped merge (k2) and the round-3 build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab7} 4 || exit 1
