# Round-5 verification of one build on a fresh box: smoke, the -m gpu suite, the driver's 20-step bench
# command with live PMC (traffic, L2, SQ split) and the CPU baseline, a rocprofv3 kernel-trace summary
# of the same command, the C3 (bunny) line, the node-form A/B (80-B, 64-B, wide) and the two-rank rehearsal (gloo,
# both ranks on cuda:0) with the per-rank timing fields.  Usage: bash scripts/gpu_r05_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05f}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/bench20_kt.log 2>&1 || { tail -20 $O/bench20_kt.log; exit 1; }
tail -1 $O/bench20_kt.log | cut -c1-200
timeout -k 10 600 python bench.py --scene bunny --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_bunny.log 2>&1 || { tail -20 $O/bench_bunny.log; exit 1; }
tail -1 $O/bench_bunny.log | cut -c1-200
for R in 1 2; do
  for C in 2 3 4; do
    WGT_CNODE=$C timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench20_c${C}_$R.log 2>&1 || { tail -20 $O/bench20_c${C}_$R.log; exit 1; }
    echo "cnode=$C r$R: $(tail -1 $O/bench20_c${C}_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
  done
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --width 960 --height 540 --spp 64 > $O/bench_n2.log 2>&1 || { tail -20 $O/bench_n2.log; exit 1; }
tail -1 $O/bench_n2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n2', d['value'], d['check_frames_bit_exact'], d['per_rank'])"
echo done
