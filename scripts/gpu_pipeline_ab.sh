# Same-box A/B of ab/*.so with frames in flight (scripts/pipeline_ab.py), alternating, fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-pab}; mkdir -p $OUT
for r in $(seq ${2:-2}); do
  for so in ab/*.so; do
    for sc in "sponza 1920 1080 256 8" "bunny 1920 1080 256 12"; do
      WGT_LIB_PATH=$PWD/$so timeout -k 10 300 python scripts/pipeline_ab.py $sc 2>&1 | grep '^{' | tee -a $OUT/pab.jsonl || exit 1
    done
  done
done
