# Final-build evidence: C2 (Cornell 1024^2/64 spp) with the cost pre-pass's paths at depth 6 (default) and
# 50 (before), alternating; the strong-scaling projections (a frame alone; 8-frame jobs, 4 in flight).
#   bash scripts/gpu_r04_last.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r04last}; mkdir -p $O
for r in 1 2 3; do for d in 6 50; do
  WGT_PQ_DEPTH=$d timeout -k 10 300 python bench.py --scene cornell --width 1024 --height 1024 --spp 64 --steps 12 --warmup 2 --pmc off --no-cpu-baseline --stats-reps 1 > $O/c2_d${d}_$r.log 2>&1 || { tail -20 $O/c2_d${d}_$r.log; exit 1; }
  echo "c2 pq_depth $d r$r: $(tail -1 $O/c2_d${d}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['timing']['isolated_launch_ms'])")"
done; done
timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 2 > $O/strong_single.jsonl 2> $O/strong_single.err || { tail $O/strong_single.err; exit 1; }
cat $O/strong_single.jsonl
timeout -k 10 300 python -u scripts/strong_projection.py --scene sponza --reps 1 --frames 8 --pipeline 4 > $O/strong_p4.jsonl 2> $O/strong_p4.err || { tail $O/strong_p4.err; exit 1; }
cat $O/strong_p4.jsonl
