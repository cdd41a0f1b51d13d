# N = 2 rehearsal on one GPU (two ranks share cuda:0 over gloo): the untimed self-check runs by default
# and the line must carry check_frames_bit_exact; weak (default) and strong scaling
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03n2}; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline > $O/weak.log 2>&1 || { tail -30 $O/weak.log; exit 1; }
grep '^{' $O/weak.log | tail -1 | cut -c1-400
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --scaling strong --no-cpu-baseline > $O/strong.log 2>&1 || { tail -30 $O/strong.log; exit 1; }
grep '^{' $O/strong.log | tail -1 | cut -c1-400
