# Round 5: C5 at its size on the final build: 600 frames of the bunny stand-in at 1080p/64 spp written as
# PNGs (render.cpp:494-497 NNN.png); their md5 list is compared on the host with round 4's
# (profiles/configs/r04c5_600_png_md5.txt): the same images, bit for bit, two rounds of kernels apart.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r05c5}; mkdir -p $O
D1=/tmp/wgt_c5_1; rm -rf $D1
timeout -k 10 300 python -m webgputracer_amd.frames --frame 1 600 --spp 64 > $O/c5_600_render.log 2>&1 || { tail $O/c5_600_render.log; exit 1; }
tail -1 $O/c5_600_render.log
timeout -k 10 600 python -m webgputracer_amd.frames --frame 1 600 --spp 64 --out $D1 > $O/c5_600_png.log 2>&1 || { tail $O/c5_600_png.log; exit 1; }
tail -1 $O/c5_600_png.log
(cd $D1 && ls | wc -l && du -sh . && md5sum *.png) > $O/c5_600_png_md5.txt; rm -rf $D1
head -3 $O/c5_600_png_md5.txt
