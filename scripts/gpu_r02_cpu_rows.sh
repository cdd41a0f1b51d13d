# CPU-baseline rows for C2 and C3 beside their GPU numbers (bench.py's cpu_baseline leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r02cpu}; mkdir -p $O
timeout -k 10 600 python bench.py --scene cornell --width 1024 --height 1024 --spp 64 --steps 6 --warmup 2 > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
timeout -k 10 600 python bench.py --scene bunny --steps 6 --warmup 2 > $O/c3.log 2>&1 || { tail $O/c3.log; exit 1; }
for f in c2 c3; do tail -1 $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['unit'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline']['sample'][:160])"; done
