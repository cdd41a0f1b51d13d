# Round-6 verification of one build on a fresh box: smoke, the -m gpu suite, the driver's 20-step bench
# command with live PMC and the CPU baseline, a rocprofv3 kernel-trace summary of the same command, the
# C3 (bunny) line, the 4-rank rehearsal line (gloo, all ranks on cuda:0, with live PMC and the CPU
# baseline), the traversal-by-level counters and the strong-scaling chain floor.
#   bash scripts/gpu_r06_final.sh TAG      (SKIP_TESTS=1 skips the suite; BENCH=0, ANALYSIS=0, CONFIGS=0
#   skip the bench lines, the level counters and chain floor, the other configs; STEPS=20)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r06f}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 900 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --pmc off > $O/bench20_kt.log 2>&1 || { tail -20 $O/bench20_kt.log; exit 1; }
tail -1 $O/bench20_kt.log | cut -c1-200
timeout -k 10 600 python bench.py --scene bunny --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_bunny.log 2>&1 || { tail -20 $O/bench_bunny.log; exit 1; }
tail -1 $O/bench_bunny.log | cut -c1-200
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --spp 16 --cpu-rows 4 --pmc on > $O/bench_n4.log 2>&1 || { tail -20 $O/bench_n4.log; exit 1; }
tail -1 $O/bench_n4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n4', d['value'], d['check_frames_bit_exact'], d['per_rank']['roofline_frac'], d['roofline']['traffic_source'], d['cpu_baseline']['value'])"
fi
if [ "${ANALYSIS:-1}" = 1 ]; then
timeout -k 10 300 python scripts/level_stats.py --scene sponza --spp 64 > $O/level_stats_sponza.log 2>&1 || { tail -20 $O/level_stats_sponza.log; exit 1; }
tail -1 $O/level_stats_sponza.log
timeout -k 10 300 python scripts/level_stats.py --scene bunny --spp 64 > $O/level_stats_bunny.log 2>&1 || { tail -20 $O/level_stats_bunny.log; exit 1; }
tail -1 $O/level_stats_bunny.log
timeout -k 10 400 python scripts/chain_floor.py --scene sponza --n 8 > $O/chain_floor.log 2>&1 || { tail -20 $O/chain_floor.log; exit 1; }
tail -1 $O/chain_floor.log | cut -c1-600
fi
if [ "${CONFIGS:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --scene cornell --width 1024 --height 1024 --spp 64 --steps 12 --warmup 2 --cpu-rows 4 > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
  tail -1 $O/c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['ms_per_step'], d['timing']['isolated_launch_ms'], (d.get('cpu_baseline') or {}).get('value'))"
  timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 48 --spp 64 --batch 4 --pipeline 2 > $O/c5_b4_p2.log 2>&1 || { tail $O/c5_b4_p2.log; exit 1; }
  echo "C5 $(tail -1 $O/c5_b4_p2.log)"
  for r in 1 2; do for cn in 2 1; do
    WGT_CNODE=$cn timeout -k 10 400 python bench.py --scene bunny --steps 20 --warmup 3 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bunny_cn${cn}_$r.log 2>&1 || { tail $O/bunny_cn${cn}_$r.log; exit 1; }
    echo "bunny cnode=$cn r$r: $(tail -1 $O/bunny_cn${cn}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['per_launch']['bvh_nodes'])")"
  done; done
fi
echo done
