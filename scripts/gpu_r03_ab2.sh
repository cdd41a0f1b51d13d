# Round-3 A/B batch 2: base (HEAD) vs mtrcp (short 1/det only) vs cur (short 1/det, shade's
# hoisted rand() draws); GPU suite on each; sponza and bunny 1080p at 64 and 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 64;bunny 1920 1080 64;sponza 1920 1080 256" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab2} 3 || exit 1
