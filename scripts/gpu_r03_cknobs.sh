# the 6-wave scheduling knobs as compile-time constants (WGT_CONST_KNOBS): GPU suite on cknobs.so, then
# same-box timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ck} 3 || exit 1
