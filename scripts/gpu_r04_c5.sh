# C5 at its size: 600 frames of the bunny stand-in at 1080p/64 spp (render.cpp:494-497 NNN.png) through
# webgputracer_amd.frames, on one rank and as 8 ranks (torch.distributed.run, all on the box's one GPU:
# the frame dealing of an 8-GPU node, each rank 75 frames); the two runs' 600 PNG files must be identical.
#   bash scripts/gpu_r04_c5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r04c5}; mkdir -p $O
D1=/tmp/wgt_c5_1; D8=/tmp/wgt_c5_8; rm -rf $D1 $D8
timeout -k 10 300 python -m webgputracer_amd.frames --frame 1 600 --spp 64 > $O/c5_600_render.log 2>&1 || { tail $O/c5_600_render.log; exit 1; }
tail -1 $O/c5_600_render.log
timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 600 --spp 64 --out $D1 > $O/c5_600_png.log 2>&1 || { tail $O/c5_600_png.log; exit 1; }
tail -1 $O/c5_600_png.log
(cd $D1 && ls | wc -l && du -sh . && md5sum *.png) > $O/c5_600_png_md5.txt; rm -rf $D1
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 -m webgputracer_amd.frames --frame 1 600 --spp 64 --out $D8 > $O/c5_600_8ranks.log 2>&1 || { tail -30 $O/c5_600_8ranks.log; exit 1; }
grep '"rank"' $O/c5_600_8ranks.log
(cd $D8 && ls | wc -l && du -sh . && md5sum *.png) > $O/c5_600_8ranks_md5.txt; rm -rf $D8
head -2 $O/c5_600_png_md5.txt; head -2 $O/c5_600_8ranks_md5.txt
if diff <(tail -n +3 $O/c5_600_png_md5.txt) <(tail -n +3 $O/c5_600_8ranks_md5.txt) > /dev/null; then echo "600 PNGs identical between 1 and 8 ranks"; else echo "PNG MISMATCH"; exit 1; fi
