set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-poolprobe2}; mkdir -p $O
run() { echo "== $*"; env "$@" timeout -k 10 120 python scripts/pool_probe.py sponza 64 >> $O/probe.jsonl 2>> $O/probe.err || { tail -5 $O/probe.err; exit 1; }; tail -1 $O/probe.jsonl | cut -c1-330; }
run WGT_POOL=0 WGT_PS_TO_TRAV=32 WGT_PS_TO_SERVICE=30
run WGT_POOL=5 WGT_PS_TO_TRAV=32 WGT_PS_TO_SERVICE=30
run WGT_POOL=5 WGT_PS_TO_TRAV=40 WGT_PS_TO_SERVICE=38
run WGT_POOL=5 WGT_PS_TO_TRAV=48 WGT_PS_TO_SERVICE=46 WGT_PS_SVC_FRAC=0
