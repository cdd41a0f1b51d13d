# Round-3 final evidence: every BASELINE config (scripts/gpu_configs.sh, with the GPU suite first),
# then the driver's bench command three times back to back (repeatability).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r03c}
bash scripts/gpu_configs.sh $T || exit 1
O=gpurun_out/$T
for r in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_run$r.log 2>&1 || { tail -20 $O/bench20_run$r.log; exit 1; }
  tail -1 $O/bench20_run$r.log | cut -c1-160
done
