# LDS bytes per wave vs frame time (scripts/park_sweep.py), sponza and bunny 64 spp, with the
# resident-wave figures the runtime computes (WGT_DEBUG=1, stderr)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04c}
O=gpurun_out/$T; mkdir -p $O
for S in sponza bunny; do
  WGT_DEBUG=1 timeout -k 10 300 python scripts/park_sweep.py $S 64 > $O/sweep_$S.log 2> $O/sweep_$S.err || { tail -20 $O/sweep_$S.err; exit 1; }
  cat $O/sweep_$S.log; grep resident $O/sweep_$S.err | sort | uniq -c
done
