#!/bin/bash
# Round-4 tail and scaling follow-ups: the strong-scaling projection with the Morton-curve tile
# dealing and 4 frames in flight (dist.tile_ranks, WGT_WS_SLOTS default 4), the cost pre-pass with
# its paths cut at WGT_PQ_DEPTH (isolated and pipelined frame times), and the instruction mix of
# the axis-aligned quad build (scripts/gpu_r04_qmix.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r04tail}; mkdir -p $O
for p in 2 4; do
  timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 1 --frames 8 --pipeline $p > $O/strong_p$p.jsonl 2> $O/strong_p$p.err || { tail $O/strong_p$p.err; exit 1; }
  cat $O/strong_p$p.jsonl
done
timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 2 > $O/strong_single.jsonl 2> $O/strong_single.err || { tail $O/strong_single.err; exit 1; }
cat $O/strong_single.jsonl
for r in 1 2; do for d in 50 8 3; do
  WGT_PQ_DEPTH=$d timeout -k 10 600 python bench.py --scene sponza --steps 20 --warmup 5 --pmc off --no-cpu-baseline --stats-reps 1 > $O/bench_d${d}_$r.log 2>&1 || { tail -20 $O/bench_d${d}_$r.log; exit 1; }
  echo "pq_depth $d r$r: $(tail -1 $O/bench_d${d}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
done; done
[ -f ab/qaxis.so ] && bash scripts/gpu_r04_qmix.sh ${1:-r04tail}_qm
