# 7 waves per SIMD (WGT_PS7 build: 72 VGPRs, service state spilled to scratch around the traversal loop, a
# 28-entry stack bound so that 28 waves' LDS stacks fit): GPU suite at 7 waves on that build, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03ps7}; mkdir -p $O
WGT_LIB_PATH=$PWD/ab/ps7.so WGT_PS_WAVES=7 WGT_STACK_LIMIT=28 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sponza or bunny or schedule" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
E="WGT_PS_WAVES=6;WGT_PS_WAVES=7,WGT_STACK_LIMIT=28;WGT_PS_WAVES=6,WGT_STACK_LIMIT=28;WGT_PS_WAVES=7,WGT_STACK_LIMIT=28;WGT_PS_WAVES=6"
for sc in sponza bunny; do
  WGT_LIB_PATH=$PWD/ab/ps7.so REUPLOAD=1 REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 256 "$E" > $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["env"], d["ms"], d["nodes"], d["trav_util"], d["bvh"]["bvh_stack"], d["identical"])
PY
done
