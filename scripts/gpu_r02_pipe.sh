# Round 2: GPU parity suite with workspace slots, then the stream-pipelining probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r02pipe}; mkdir -p $O
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== probe"
timeout -k 10 400 python scripts/pipeline_probe.py sponza 1920 1080 256 6 2>&1 | grep -v amdgpu.ids | tee $O/probe_sponza.jsonl || exit 1
timeout -k 10 300 python scripts/pipeline_probe.py bunny 1920 1080 256 8 2>&1 | grep -v amdgpu.ids | tee $O/probe_bunny.jsonl || exit 1
