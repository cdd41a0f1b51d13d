"""Summarise rocprofv3 --pmc directories of one-frame bench child runs named <variant>_<counters>
(gpurun_out/<tag>/): per variant, the dominant k_render_ps launch's counters, HBM bytes
((2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB, MI355X_MICROARCH.md §HBM), L2 hit rate and requests, and the
wave-cycle split.  Usage: python scripts/summarize_pmc_variants.py gpurun_out/r04b > out.md"""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
var = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(src, "*_*"))):
    if not os.path.isdir(d):
        continue
    name = os.path.basename(d)
    parts = name.split("_")
    key = "_".join(parts[:2]) if parts[1].startswith("c") else parts[0]
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_render_ps<false, false" in k:
                var[key][r["Counter_Name"]] = var[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                var[key]["kernel"] = k.split("(")[0].replace("void ", "")
print(f"# PMC passes, one frame per pass ({src})\n")
print("| variant | kernel | counter | value |\n|---|---|---|---|")
for v, c in sorted(var.items()):
    for k, x in sorted(c.items()):
        if k != "kernel":
            print(f"| {v} | `{c['kernel']}` | {k} | {x:,.0f} |")
print("\n| variant | HBM GB / frame | of which writes GB | L2 requests | L2 hit rate | issuing / waiting / issue-stalled |")
print("|---|---|---|---|---|---|")
for v, c in sorted(var.items()):
    hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e9 if "FETCH_SIZE" in c else None
    wr = c.get("WRITE_SIZE", 0) * 1024 / 1e9 if "WRITE_SIZE" in c else None
    req = c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)
    hit = c.get("TCC_HIT_sum", 0) / req if req else None
    wc = c.get("SQ_WAVE_CYCLES")
    split = (f"{c['SQ_ACTIVE_INST_ANY'] / wc:.3f} / {c['SQ_WAIT_ANY'] / wc:.3f} / {c['SQ_WAIT_INST_ANY'] / wc:.3f}"
             if wc and "SQ_WAIT_ANY" in c else "")
    f = lambda x, p: "" if x is None else f"{x:.{p}f}"  # noqa: E731
    print(f"| {v} | {f(hbm, 1)} | {f(wr, 2)} | {req:,.0f} | {f(hit, 4)} | {split} |")
