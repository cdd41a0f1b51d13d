# up to K triangles per triangle step (WGT_TRI_PER_STEP=2,3,4) against the round-3 build: GPU suite on k2-k4.so, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 64;bunny 1920 1080 64;sponza 1920 1080 256;bunny 1920 1080 256" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab6} 3 || exit 1
