# Round-3 A/B batch 1: base (HEAD) vs ref64 (refactored triangle test), tri40 (40-B triangle
# records), mtrcp (short reciprocal in Moller-Trumbore); then the strong-scaling projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03ab1}; mkdir -p $O
AB_SCENES="sponza 1920 1080 64;bunny 1920 1080 64" REPS=2 bash scripts/gpu_ab_sweep.sh ${1:-r03ab1} 3 || exit 1
timeout -k 10 300 python scripts/strong_projection.py --scene sponza --reps 1 > $O/strong_sponza.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
cat $O/strong_sponza.jsonl
