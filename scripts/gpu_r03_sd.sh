# traversal always in units of the compact step (t.inv = s/d; device 128-B planes and triangle boxes stored / s):
# the whole GPU suite on the working tree, then same-box timing against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03sd}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -30 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
WGT_POOL=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bunny_render or sponza_render" > $O/pytest_pool.log 2>&1 || { tail -30 $O/pytest_pool.log; exit 1; }
tail -1 $O/pytest_pool.log
AB_SCENES="sponza 1920 1080 256;bunny 1920 1080 256;sponza 1920 1080 64" REPS=2 bash scripts/ab_run.sh ${1:-r03sd} 3 > /dev/null || exit 1
python scripts/ab_table.py $O/ab.log
