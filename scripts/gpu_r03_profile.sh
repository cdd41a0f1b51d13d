# Round-3 evidence for one build: the driver's bench command, then the profile (kernel trace +
# separate PMC passes) of sponza (C4) and bunny (C3).  Usage: bash scripts/gpu_r03_profile.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r03p}
O=gpurun_out/$T; mkdir -p $O
echo "== bench 20/5"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-300
bash scripts/gpu_profile.sh $T || exit 1
bash scripts/gpu_profile.sh ${T}_bunny --scene bunny || exit 1
