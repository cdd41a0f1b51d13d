# Historical (round 5): k_render_ps2 / WGT_PS_WAVES=4 / WGT_PX2_* were removed after commit 050a6a2.
# Round 5: two pixels per lane, diagnostics: STATS counters at 16 and 256 spp (bunny).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r05px2c}; O=gpurun_out/$T; mkdir -p $O
for spp in 16 256; do
  timeout -k 10 300 python scripts/px2_stats.py bunny $spp base= px2=WGT_PS_WAVES:4 > $O/stats_bunny_$spp.jsonl 2>&1 \
    || { tail -20 $O/stats_bunny_$spp.jsonl; exit 1; }
  cat $O/stats_bunny_$spp.jsonl
done
