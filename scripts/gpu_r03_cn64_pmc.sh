# 64-B compact nodes: L2 requests and HBM bytes per frame (separate PMC passes, sponza C4 one frame) for
# HEAD (base.so) and WGT_CN64 (cn64.so), then 4 more timing rounds in the opposite order
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-r03cn64p}; mkdir -p $O
for so in cn64 base; do
  for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    N=$(echo $C | cut -d' ' -f1)
    WGT_LIB_PATH=$PWD/ab/$so.so timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${so}_$N -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline > $O/${so}_$N.log 2>&1 || { tail -20 $O/${so}_$N.log; exit 1; }
  done
done
python - $O <<'PY'
import csv, glob, os, sys, collections
o = sys.argv[1]
for so in ("base", "cn64"):
    agg = collections.defaultdict(float)
    for d in glob.glob(f"{o}/{so}_*"):
        p = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(p): continue
        for r in csv.DictReader(open(p)):
            if "k_render_ps<false, false, true" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    req = agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"]
    print(so, {k: f"{v:.4g}" for k, v in sorted(agg.items())}, "tcc_requests", f"{req:.4g}",
          "hit_rate", round(agg["TCC_HIT_sum"] / max(req, 1), 4), "hbm_GB", round(2 * agg["FETCH_SIZE"] * 1024 / 1e9, 1))
PY
AB_SCENES="sponza 1920 1080 256" REPS=2 bash -c 'cd ab && mv base.so zbase.so && cd .. && bash scripts/ab_run.sh '"${1:-r03cn64p}"' 4; cd ab && mv zbase.so base.so'
python scripts/ab_table.py $O/ab.log
