set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03probe}; mkdir -p $O
timeout -k 10 120 python scripts/pool_probe.py sponza 64 > $O/regions_sponza.json 2> $O/err.log || { tail $O/err.log; exit 1; }
cat $O/regions_sponza.json
timeout -k 10 120 python scripts/pool_probe.py bunny 64 > $O/regions_bunny.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
cat $O/regions_bunny.json
timeout -k 10 300 python scripts/strong_projection.py --scene sponza --reps 1 > $O/strong_sponza.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
cat $O/strong_sponza.jsonl
