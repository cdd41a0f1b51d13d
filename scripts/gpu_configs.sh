#!/bin/bash
# Every BASELINE config on one GPU: C2 Cornell 1024^2/64, C3 bunny 1080p/256,
# C4 sponza 1080p/256 (bench default, 1 GPU share), C5 bunny 1080p/64 frames (batch 1/4/8, pipeline 1/2).
#   bash scripts/gpu_configs.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-cfg}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --scene cornell --width 1024 --height 1024 --spp 64 --steps 12 --warmup 2 > $OUT/c2.log 2>&1 || { tail $OUT/c2.log; exit 1; }
timeout -k 10 600 python bench.py --scene bunny --steps 12 --warmup 2 > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
timeout -k 10 900 python bench.py --scene sponza --steps 8 --warmup 2 --no-cpu-baseline > $OUT/c4.log 2>&1 || { tail $OUT/c4.log; exit 1; }
for b in 1 4 8; do for p in 1 2; do
  timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 48 --spp 64 --batch $b --pipeline $p > $OUT/c5_b${b}_p${p}.log 2>&1 || { tail $OUT/c5_b${b}_p${p}.log; exit 1; }
done; done
for f in c2 c3 c4; do tail -1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['config']['workload'], d['value'], d['unit'], 'ms_per_step', d['ms_per_step'], 'launch_ms', d['kernel_ms'], 'isolated', d['timing']['isolated_launch_ms'], 'frac', d['roofline']['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
for f in $OUT/c5_*.log; do echo -n "$(basename $f .log) "; tail -1 $f; done
