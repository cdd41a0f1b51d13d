# Round-2 evidence: default 20-step bench (the driver's command), profile (kernel trace + PMC), N=2 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r02f}; mkdir -p $O
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "== bench 20/5"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-300
bash scripts/gpu_profile.sh ${1:-r02f} || exit 1
bash scripts/gpu_dist_rehearsal.sh ${1:-r02f}_dist || exit 1
