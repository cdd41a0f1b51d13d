# C5 with PNG output (the reference writes every frame): encoder threads 1 against the CPU share, then the
# PNG/CLI product tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5png}; mkdir -p $O
for t in 1 0; do
  rm -rf /tmp/wgt_c5png; timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 48 --spp 64 --batch 4 --pipeline 2 \
    --out /tmp/wgt_c5png --png-threads $t > $O/png_t$t.log 2>&1 || { tail $O/png_t$t.log; exit 1; }
  echo "threads=$t $(tail -1 $O/png_t$t.log) files=$(ls /tmp/wgt_c5png | wc -l)"
done
rm -rf /tmp/wgt_c5png
timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 48 --spp 64 --batch 4 --pipeline 2 > $O/render_only.log 2>&1 && echo "render only $(tail -1 $O/render_only.log)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_product.py -x -q --timeout 300 --timeout-method thread -k "png or cli or frames" > $O/pytest.log 2>&1; tail -1 $O/pytest.log
