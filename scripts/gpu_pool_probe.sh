# Pool-kernel probes (scripts/pool_probe.py) over knob settings, one GPU process each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-poolprobe}; mkdir -p $O
SC=${SCENE:-sponza}; SPP=${SPP:-64}
run() { echo "== $*"; env "$@" timeout -k 10 120 python scripts/pool_probe.py $SC $SPP >> $O/probe.jsonl 2>> $O/probe.err || { tail -5 $O/probe.err; exit 1; }; tail -1 $O/probe.jsonl; }
run WGT_POOL=0
run WGT_POOL=6 WGT_POOL_PARK=0
run WGT_POOL=6 WGT_POOL_PARK=1
run WGT_POOL=5 WGT_POOL_PARK=0
run WGT_POOL=5 WGT_POOL_PARK=1
run WGT_POOL=5 WGT_POOL_PARK=1 WGT_POOL_ADOPT=16
