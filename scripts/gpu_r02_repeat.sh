# Repeatability of the driver's bench command: three runs back to back on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-r02rep}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.log 2>&1 || { tail -20 $O/bench20_$i.log; exit 1; }
  tail -1 $O/bench20_$i.log | python -c "import json,sys; d=json.load(sys.stdin); print('run $i', d['value'], d['ms_per_step'], d['kernel_ms'], d['timing']['isolated_launch_ms'], d['roofline']['frac'])"
done
