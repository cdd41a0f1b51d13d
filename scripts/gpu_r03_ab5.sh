# quad-row prefetch variants (qpf2: normal + (w, d) rows; qpf5: rows 0-4), GPU suite on each, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 64;bunny 1920 1080 64;sponza 1920 1080 256" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab5} 3 || exit 1
