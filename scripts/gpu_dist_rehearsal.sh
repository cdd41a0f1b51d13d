#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks share cuda:0, gloo gather,
# --check compares the assembled frames with single-launch renders bit for bit;
# weak scaling (a frame per rank) and strong scaling (one frame split over the ranks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist}; mkdir -p $OUT
# sponza: compact nodes at 5 waves/SIMD; bunny: 128-B nodes at 6
for run in "sponza weak" "sponza strong" "bunny weak"; do
  set -- $run
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --no-cpu-baseline --check on \
    --scene $1 --scaling $2 --width 640 --height 360 --spp 16 > $OUT/bench_n2_$1_$2.log 2>&1 || { tail -20 $OUT/bench_n2_$1_$2.log; exit 1; }
  tail -1 $OUT/bench_n2_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['scaling'], 'check', d['check_frames_bit_exact'], d['value'], d['unit'], d['config']['frames_per_step']); sys.exit(0 if d['check_frames_bit_exact'] else 1)" || exit 1
done
