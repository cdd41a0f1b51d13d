# Compiler-flag variants (timing only: scheduling / unrolling flags keep the fp32 semantics;
# the chosen one then runs the GPU suite)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03ab3}; mkdir -p $O
AB_SCENES="sponza 1920 1080 64;bunny 1920 1080 64" REPS=2 bash scripts/ab_run.sh ${1:-r03ab3} 3 > /dev/null || exit 1
python scripts/ab_table.py $O/ab.log
