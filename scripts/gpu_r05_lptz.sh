# Round 5: the LPT sort that re-zeroes its workspace (no memset kernel per frame, 256 threads) against HEAD, same box:
# the whole GPU parity suite on the new build, then the driver's bench command, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05tf}; R=${2:-2}; O=gpurun_out/$T; mkdir -p $O
WGT_LIB_PATH=$PWD/ab/b_lptz.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_product.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in $(seq $R); do
  for so in ab/*.so; do
    n=$(basename $so .so)
    for sc in ${SCENES:-sponza bunny}; do
      st=20; [ $sc = bunny ] && st=30
      WGT_LIB_PATH=$PWD/$so timeout -k 10 600 python bench.py --scene $sc --steps $st --warmup 5 --pmc off \
        --no-cpu-baseline --stats-reps 1 > $O/bench_${n}_${sc}_$r.log 2>&1 || { tail -20 $O/bench_${n}_${sc}_$r.log; exit 1; }
      echo "$n $sc r$r: $(tail -1 $O/bench_${n}_${sc}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_launch']; print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'], round(p['node_visits']/p['traced_rays'],3), round(p['tri_tests']/p['traced_rays'],3), d['simt_utilisation'])")"
    done
  done
done
