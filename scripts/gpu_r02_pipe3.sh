set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r02pipe3}; mkdir -p $O
PROBE_REPS=3 timeout -k 10 300 python scripts/pipeline_probe.py bunny 1920 1080 256 8 2>&1 | grep -v amdgpu.ids | tee $O/probe_bunny.jsonl || exit 1
PROBE_REPS=2 timeout -k 10 500 python scripts/pipeline_probe.py sponza 1920 1080 256 6 2>&1 | grep -v amdgpu.ids | tee $O/probe_sponza.jsonl || exit 1
