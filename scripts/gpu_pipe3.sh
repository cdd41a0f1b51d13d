# Frames in flight: 2 (default) vs 3 (three workspace slots) on the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r02p3}; mkdir -p $O
for cfg in "2 2" "3 3" "2 2" "3 3"; do
  set -- $cfg
  WGT_WS_SLOTS=$2 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pipeline $1 --no-cpu-baseline > $O/p$1.log 2>&1 || { tail -20 $O/p$1.log; exit 1; }
  tail -1 $O/p$1.log | python -c "import json,sys; d=json.load(sys.stdin); print('pipeline $1 slots $2', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
