set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02crec; mkdir -p $O
WGT_CNODE=1 WGT_LIB_PATH=$PWD/ab/crec8.so timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_crec8.log 2>&1 || { tail -20 $O/pytest_crec8.log; exit 1; }
tail -1 $O/pytest_crec8.log
for r in 1 2; do
 for so in base crec8; do
  for cn in 2 1; do
   for sc in "bunny 1920 1080 256" "sponza 1920 1080 256"; do
    echo -n "$so cn$cn r$r $sc " >> $O/ab.log
    WGT_CNODE=$cn WGT_LIB_PATH=$PWD/ab/$so.so SWEEP_ONLY=2 REPS=3 timeout -k 10 300 python scripts/sweep_wf.py $sc 2>&1 | grep '"ms"' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['nodes'])" >> $O/ab.log || exit 1
   done
  done
 done
done
cat $O/ab.log
