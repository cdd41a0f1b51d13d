# 5 against 6 waves per SIMD on the final kernel (WGT_PS_WAVES=5 forces the 4-byte stack at 96 VGPRs), scene
# re-uploaded per setting, one frame per render (min of 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03waves}; mkdir -p $O
E="WGT_PS_WAVES=0;WGT_PS_WAVES=5;WGT_PS_WAVES=0;WGT_PS_WAVES=5;WGT_PS_WAVES=0"
for sc in bunny sponza; do
  for spp in 256 64; do
    REUPLOAD=1 REPS=2 timeout -k 10 500 python scripts/sweep_env.py $sc 1920 1080 $spp "$E" >> $O/$sc.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
  python - $O/$sc.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["scene"], d["spp"], d["env"], d["ms"], d["trav_util"], d["identical"])
PY
done
