#!/bin/bash
# Build libwgt.so of a git revision into ab/<name>.so for same-box A/B timing.
#   scripts/ab_build.sh <rev> <name>     (rev "WORK" = the working tree)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ab"
if [ "$1" = "WORK" ]; then
  make -s -C "$ROOT/webgputracer_amd" -j8 libwgt.so
  cp "$ROOT/webgputracer_amd/libwgt.so" "$ROOT/ab/$2.so"
  # a flagged variant must not stay behind as the tree's library (GPU runs load the in-tree build)
  if [ -n "$WGT_FLAGS" ]; then WGT_FLAGS= make -s -C "$ROOT/webgputracer_amd" -j8 libwgt.so; fi
else
  D=$(mktemp -d /tmp/wgt_ab.XXXX)
  git -C "$ROOT" archive "$1" webgputracer_amd include | tar -x -C "$D"
  make -s -C "$D/webgputracer_amd" -j8 libwgt.so
  cp "$D/webgputracer_amd/libwgt.so" "$ROOT/ab/$2.so"
  rm -rf "$D"
fi
