# Frames in flight in the driver's command (bench.py --pipeline 2 / 3 / 4; the context has 4 scheduling
# workspaces since round 4), rounds alternating, after the schedule-invariance parity test.
#   bash scripts/gpu_r04_pipe.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r04pipe}; R=${2:-3}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "schedule_invariance" --timeout 300 --timeout-method thread > $O/pytest_sched.log 2>&1 || { tail -30 $O/pytest_sched.log; exit 1; }
tail -1 $O/pytest_sched.log
for r in $(seq $R); do
  for p in 2 3 4; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --pipeline $p --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_p${p}_$r.log 2>&1 || { tail -20 $O/bench_p${p}_$r.log; exit 1; }
    echo "pipeline $p r$r: $(tail -1 $O/bench_p${p}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
  done
done
# the driver's exact command three times back to back (repeatability of the line on this build)
for r in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_run$r.log 2>&1 || { tail -20 $O/bench20_run$r.log; exit 1; }
  echo "driver command run $r: $(tail -1 $O/bench20_run$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_source'))")"
done
