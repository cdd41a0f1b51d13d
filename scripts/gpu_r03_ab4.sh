# -O2 against -O3 at the bench configurations (1080p/256 spp), GPU suite on the -O2 build first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;cornell 1024 1024 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab4} 3 || exit 1
