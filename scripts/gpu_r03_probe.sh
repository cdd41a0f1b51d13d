set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03probe}; mkdir -p $O
for sc in sponza bunny; do
  timeout -k 10 120 python scripts/pool_probe.py $sc 256 > $O/regions_$sc.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
  cat $O/regions_$sc.json
done
