#!/bin/bash
# Round-4 evidence on the final build: every BASELINE config (scripts/gpu_configs.sh without its
# pytest step) and the strong-scaling projections (one frame alone; 8-frame jobs, 2 and 4 in flight).
#   bash scripts/gpu_r04_evidence.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04ev}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 2 > $OUT/strong_single.jsonl 2> $OUT/strong_single.err || { tail $OUT/strong_single.err; exit 1; }
cat $OUT/strong_single.jsonl
for p in 2 4; do
  timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 1 --frames 8 --pipeline $p > $OUT/strong_p$p.jsonl 2> $OUT/strong_p$p.err || { tail $OUT/strong_p$p.err; exit 1; }
  cat $OUT/strong_p$p.jsonl
done
timeout -k 10 600 python bench.py --scene cornell --width 1024 --height 1024 --spp 64 --steps 12 --warmup 2 > $OUT/c2.log 2>&1 || { tail $OUT/c2.log; exit 1; }
timeout -k 10 600 python bench.py --scene bunny --steps 12 --warmup 2 > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
for b in 1 4 8; do for p in 1 2; do
  timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 48 --spp 64 --batch $b --pipeline $p > $OUT/c5_b${b}_p${p}.log 2>&1 || { tail $OUT/c5_b${b}_p${p}.log; exit 1; }
done; done
for f in c2 c3; do tail -1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['config']['workload'], d['value'], d['unit'], 'ms_per_step', d['ms_per_step'], 'launch_ms', d['kernel_ms'], 'isolated', d['timing']['isolated_launch_ms'], 'frac', d['roofline']['frac'], 'bound', d['roofline'].get('bound'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
for f in $OUT/c5_*.log; do echo -n "$(basename $f .log) "; tail -1 $f; done
