#!/bin/bash
# Tail probes: bash scripts/gpu_tail.sh <tag> ["scene W H spp T" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-tail}; mkdir -p $OUT; shift
[ $# -gt 0 ] || set -- "bunny 1920 1080 64 8" "sponza 1920 1080 16 8"
for cfg in "$@"; do
  timeout -k 10 300 python scripts/tail_probe.py $cfg 2>&1 | grep -v amdgpu.ids | tee -a $OUT/tail.log || exit 1
done
